"""Adversarial probes of the reference-box certificates.

A face carrying the certificate (TriRec64.box bit 30, `box_certified` in rt_host.cpp) lets the accept
path skip the reference's own box predicate (`intersectBox`, src/flyscene.cpp:484-507, as called from
calculateMinimumFace :381-391 and shadow :510-526) for every ray whose object-space origin o2 has
|o2|_inf <= Ro (the certified range). The argument is analytic; these tests aim
rays exactly where it could break:

* origins with |o2|_inf uniform in [0.5, 1.0] x Ro (inside the range, where the skip is taken) and in
  (1.0, 1.05] x Ro (just beyond it, where the exact predicate runs again);
* targets on CERTIFIED faces only: vertices, edge midpoints, the point of the face nearest its reference
  box's boundary, and points just outside the triangle beside that point (where the reference's inclusive
  float edge tests decide by rounding);
* grazing directions: rays nearly parallel to a certified face whose vertex lies nearest a reference-box
  plane, aimed at that vertex;
* a rotated and a non-uniformly scaled model matrix, under which the object-space face normals no longer
  match the world triangles and no face may be certified: whole frames against the oracle.

Every closest-hit and shadow result must equal the CPU oracle's bit for bit; the tests report how many
rays' final hits took the certified skip.
"""
import numpy as np
import pytest

from conftest import PARITY_REPORT, scene_path
from test_gpu_far import look_at
from test_gpu_fullframe import THREADS, frame_errors
from test_oracle_pinning import same_bits

pytestmark = pytest.mark.gpu
CERT = 0x40000000


@pytest.fixture(scope="module", autouse=True)
def need_gpu(rt):
    if rt.device_count() == 0:
        pytest.skip("no GPU")


def _scene_pair(rt, orc, name):
    if name == "soup":
        mesh, v, f = rt.soup_mesh(1_000_000)
        return mesh, rt.Scene(mesh), orc.Scene(orc.Mesh.from_arrays(v, f, np.array([rt.SOUP_MATERIAL], np.float32)))
    mesh = rt.Mesh.load_obj(scene_path(name + ".obj"))
    return mesh, rt.Scene(mesh), orc.Scene(orc.Mesh.load_obj(scene_path(name + ".obj")))


def _face_boxes(sc, nf):
    """object-space reference box [nf, 6] (lo xyz, hi xyz) of every face, from the partition's face order"""
    b6, cnt, order = sc.ref_boxes()
    box_of = np.repeat(np.arange(len(cnt)), cnt)
    fb = np.zeros((nf, 6), np.float64)
    fb[np.asarray(order, np.int64)] = np.asarray(b6, np.float64)[box_of]
    return fb


def _probe_rays(rng, n, ov, fidx, fbox, cert_faces, Ro, M):
    """n rays (world-space origins, unit directions, object-space origin norm) aimed at certified faces."""
    f = cert_faces[rng.integers(0, len(cert_faces), n)]
    w = ov[fidx[f]]  # [n, 3, 3] object-space vertices
    lo, hi = fbox[f, :3], fbox[f, 3:]
    # distance of each vertex to its box's boundary (smallest over the six planes)
    dv = np.minimum(w - lo[:, None, :], hi[:, None, :] - w).min(2)  # [n, 3]
    near = np.argmin(dv, 1)
    kind = rng.integers(0, 4, n)
    bary = np.zeros((n, 3))
    bary[np.arange(n), rng.integers(0, 3, n)] = 1.0  # kind 0: a vertex
    e = rng.integers(0, 3, n)
    mid = np.full((n, 3), 0.5)
    mid[np.arange(n), e] = 0.0
    bary[kind == 1] = mid[kind == 1]  # kind 1: an edge midpoint
    nb = np.zeros((n, 3))
    nb[np.arange(n), near] = 1.0
    bary[kind == 2] = nb[kind == 2]  # kind 2: the vertex nearest the box boundary
    # kind 3: just outside the triangle beside that vertex (negative weights of 1e-7 .. 1e-4)
    eps = 10.0 ** rng.uniform(-7, -4, n)
    out = nb * (1.0 + 2 * eps[:, None]) - (1.0 - nb) * eps[:, None]
    bary[kind == 3] = out[kind == 3]
    tgt_o = np.einsum("nk,nkc->nc", bary, w)
    # object-space origin with |o2|_inf uniform in [0.5, 1.0] Ro (a quarter of them in (1.0, 1.05] Ro)
    beyond = rng.random(n) < 0.25
    mag = np.where(beyond, rng.uniform(1.0, 1.05, n), rng.uniform(0.5, 1.0, n)) * Ro
    u = rng.normal(size=(n, 3))
    u /= np.abs(u).max(1, keepdims=True)  # |u|_inf = 1
    o2 = u * mag[:, None]
    # grazing set (every 8th ray): origin in the face's plane direction, nearly parallel to the face
    g = np.arange(n) % 8 == 7
    if g.any():
        wg = w[g]
        nrm = np.cross(wg[:, 1] - wg[:, 0], wg[:, 2] - wg[:, 0])
        nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
        tv = np.einsum("nk,nkc->nc", nb[g], wg)  # the vertex nearest the box boundary
        inplane = rng.normal(size=(g.sum(), 3))
        inplane -= np.einsum("nc,nc->n", inplane, nrm)[:, None] * nrm
        inplane /= np.linalg.norm(inplane, axis=1, keepdims=True)
        tilt = 10.0 ** rng.uniform(-6, -2, g.sum()) * np.sign(rng.normal(size=g.sum()))
        dirg = inplane + tilt[:, None] * nrm
        dirg /= np.linalg.norm(dirg, axis=1, keepdims=True)
        # the origin about the sampled |o2| magnitude away, along -dirg from the vertex
        o2[g] = tv - dirg * mag[g][:, None]
        tgt_o[g] = tv
    Mm = np.asarray(M, np.float64).reshape(4, 4).T  # column-major Affine3f
    o = (Mm[:3, :3] @ o2.T).T + Mm[:3, 3]
    t = (Mm[:3, :3] @ tgt_o.T).T + Mm[:3, 3]
    d = t - o
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    return o.astype(np.float32), d.astype(np.float32), np.abs(o2).max(1), f


@pytest.mark.parametrize("name", ["bunny", "soup"])
def test_certified_faces_adversarial_queries(rt, orc, name):
    mesh, sc, osc = _scene_pair(rt, orc, name)
    ex = mesh.export()
    ov = np.asarray(ex["v4"], np.float64)
    ov = ov[:, :3] / ov[:, 3:4]
    fidx = np.asarray(ex["fidx"], np.int64)
    ff, Ro = sc.face_flags()
    cert_faces = np.nonzero(ff & CERT)[0]
    assert Ro > 0 and len(cert_faces) > 0.8 * len(ff)
    fbox = _face_boxes(sc, len(ff))
    rng = np.random.default_rng(2024 if name == "bunny" else 2025)
    n = 131072 if name == "bunny" else 51200  # closest + shadow: >= 100k rays per scene
    o, d, o2n, aimed = _probe_rays(rng, n, ov, fidx, fbox, cert_faces, Ro, ex["M16"])
    face, t, P = sc.trace_closest(o, d)
    oface, ot, oP = osc.closest(o, d)
    mism = int((face != oface).sum())
    tm = int((~same_bits(t, ot)).sum())
    hit = oface >= 0
    # final hits that took the skip: a certified face, object-space origin within the range
    skipped = int((hit & ((ff[np.maximum(oface, 0)] & CERT) != 0) & (o2n <= Ro)).sum())
    # shadow(): from P = the same origins towards the same directions (box test from P, triangles from
    # P + 0.003 L, flyscene.cpp:510-526)
    blk = sc.trace_shadow(o, d)
    oblk = osc.shadow(o, d)
    smism = int((blk != oblk).sum())
    PARITY_REPORT.append(
        f"certificate probe ({name}, {n} rays aimed at certified faces, |o2| in [0.5, 1.05] x Ro, 1/8 grazing): "
        f"{int(hit.sum())} hits, {skipped} final hits through the certified skip, {int((o2n > Ro).sum())} "
        f"origins beyond Ro; face mismatches {mism}, t mismatches {tm}; shadow: {int(oblk.sum())} blocked, "
        f"mismatches {smism}")
    assert hit.sum() > n // 4 and skipped > n // 8
    assert mism == 0 and tm == 0
    assert same_bits(P[hit], oP[hit]).all()
    assert smism == 0


def _rotation(ax_deg, ay_deg):
    a, b = np.radians(ax_deg), np.radians(ay_deg)
    rx = np.array([[1, 0, 0], [0, np.cos(a), -np.sin(a)], [0, np.sin(a), np.cos(a)]])
    ry = np.array([[np.cos(b), 0, np.sin(b)], [0, 1, 0], [-np.sin(b), 0, np.cos(b)]])
    m = np.eye(4)
    m[:3, :3] = ry @ rx
    return m.T.astype(np.float32).reshape(16)


MODELS = {"rotated": _rotation(20, 30),
          "stretched": np.diag([1.0, 0.8, 1.5, 1.0]).astype(np.float32).reshape(16)}


@pytest.mark.parametrize("model", sorted(MODELS))
@pytest.mark.parametrize("mode", ["primary", "full"])
def test_model_matrix_frames_match_oracle(rt, orc, model, mode):
    """Model::modelMatrix rotated or non-uniformly scaled (the reference keeps the object-space face normals
    against the world vertices in calculateDistance, flyscene.cpp:444-478): no certificate may be issued,
    and whole frames equal the oracle's."""
    path = scene_path("bunny.obj")
    om = orc.Mesh.load_obj(path)
    om.set_model(MODELS[model])
    M16 = om.export()["M16"]
    sc = rt.Scene(rt.Mesh.load_obj(path), shape_model_matrix=M16)
    osc = orc.Scene(om)
    assert sc.record_flags()[2] == 0
    W, H = 480, 360
    eye = np.array([0.4, 0.3, 2.2])
    full = mode == "full"
    rgb, face, t, _ = sc.render(look_at(rt, W, H, eye, (0, 0, 0), (0, 1, 0), 45.0), rt.DEFAULT_LIGHTS, W, H,
                                mode=rt.RT_MODE_FULL if full else rt.RT_MODE_PRIMARY, want_hits=True)
    orgb, oface, ot = osc.render(look_at(orc, W, H, eye, (0, 0, 0), (0, 1, 0), 45.0), orc.DEFAULT_LIGHTS, W, H,
                                 full=full, threads=THREADS)
    e = frame_errors(rgb, face, t, orgb, oface, ot)
    hits = int((np.asarray(oface) >= 0).sum())
    PARITY_REPORT.append(f"bunny with a {model} model matrix {W}x{H} {mode}: {hits} hit pixels, face mismatches "
                         f"{e['face_mismatch']}, t mismatches {e['t_mismatch']}, colour L_inf {e['linf']:.3g}")
    assert hits > W * H // 20
    assert e["face_mismatch"] == 0 and e["t_mismatch"] == 0 and e["nan_mismatch"] == 0, e
    assert e["linf"] < 1e-4, e
