"""Exactness of BVH culling for every ray origin the reference accepts.

The reference tests every box of its flat partition and culls nothing (src/flyscene.cpp:381-391), and its
fly camera can move anywhere (dependencies/tucano/tucano/utils/flycamera.hpp:196-202). The GPU culls with
a BVH whose boxes carry a static, scene-scale pad plus a per-ray pad proportional to the ray origin's
magnitude (setup_cull, rt_device.hip). These tests put the origin where the rounding
of the reference's hit point P = o + t d is largest relative to the scene -- eyes at 50 and 500 scene
extents (narrow fields of view, so the scene still fills the frame), eyes at 3-7 extents (inside the range
where certified faces skip the reference box predicate), a grazing view along a face plane,
ray-list queries from up to 1e7 extents aimed at vertices and edges, and origins beyond the certified
range (brute-force boxes) -- and hold the GPU to the CPU oracle: face and t bit-exact, colour L_inf < 1e-4.
"""
import math

import numpy as np
import pytest

from conftest import PARITY_REPORT, scene_path
from test_gpu_fullframe import THREADS, frame_errors
from test_oracle_pinning import same_bits

pytestmark = pytest.mark.gpu
TOL = 1e-4


@pytest.fixture(scope="module", autouse=True)
def need_gpu(rt):
    if rt.device_count() == 0:
        pytest.skip("no GPU")


def look_at(mod, W, H, eye, target, up, fovy):
    """A camera of either module (GPU binding or oracle) at `eye` looking at `target`: view matrix =
    world -> camera (rows right, up, -forward), column-major as Tucano's Affine3f."""
    eye = np.asarray(eye, np.float64)
    f = np.asarray(target, np.float64) - eye
    f /= np.linalg.norm(f)
    r = np.cross(f, up)
    r /= np.linalg.norm(r)
    u = np.cross(r, f)
    R = np.stack([r, u, -f])
    t = -R @ eye
    M = np.eye(4)
    M[:3, :3] = R
    M[:3, 3] = t
    c = mod.Camera()
    for k, v in enumerate(np.asarray(M, np.float32).T.reshape(-1)):
        (c.view_matrix if hasattr(c, "view_matrix") else c.view)[k] = float(v)
    c.viewport[0], c.viewport[1], c.viewport[2], c.viewport[3] = 0.0, 0.0, float(W), float(H)
    c.fovy = float(fovy)
    if hasattr(c, "aspect_ratio"):
        c.aspect_ratio = W / H
    else:
        c.aspect = W / H
    return c


@pytest.fixture(scope="module")
def scenes(rt, orc):
    out = {}
    for name in ("bunny", "cube"):
        out[name] = (rt.Scene(rt.Mesh.load_obj(scene_path(name + ".obj"))),
                     orc.Scene(orc.Mesh.load_obj(scene_path(name + ".obj"))))
    mesh, v, f = rt.soup_mesh(1_000_000)
    out["soup"] = (rt.Scene(mesh), orc.Scene(orc.Mesh.from_arrays(v, f, np.array([rt.SOUP_MATERIAL], np.float32))))
    return out


# (scene, eye distance in scene extents, eye direction, mode, frame)
FAR_VIEWS = [
    ("bunny", 50, (0, 0, 1), "primary", (640, 480)),
    ("bunny", 500, (0, 0, 1), "primary", (640, 480)),
    ("bunny", 500, (1, 1, 1), "full", (480, 360)),
    ("soup", 50, (0, 0, 1), "primary", (640, 360)),
    ("soup", 500, (1, -0.5, 1), "primary", (640, 360)),
    ("cube", 500, (0, 0, 1), "full", (320, 240)),
    # inside the reference-box certificates' origin range (|o2| <= 16 x the largest object coordinate):
    # certified faces skip the box predicate for these rays
    ("bunny", 3, (1, 0.5, 1), "full", (480, 360)),
    ("bunny", 7, (0, 0, 1), "primary", (640, 480)),
    ("soup", 6, (0.3, 1, 1), "primary", (640, 360)),
]


@pytest.mark.parametrize("case", FAR_VIEWS, ids=lambda c: f"{c[0]}-{c[1]}x-{c[3]}-{'_'.join(map(str, c[2]))}")
def test_far_eye_frames_match_oracle(rt, orc, scenes, case):
    name, dist, direction, mode, (W, H) = case
    sc, osc = scenes[name]
    u = np.asarray(direction, np.float64)
    u /= np.linalg.norm(u)
    eye = dist * u  # the normalised model puts the scene around the origin with extent ~1
    up = (0.0, 1.0, 0.0) if abs(u[1]) < 0.9 else (1.0, 0.0, 0.0)
    fovy = math.degrees(2 * math.atan(0.6 / dist))  # ~1.2 scene units of view at the scene
    full = mode == "full"
    m = rt.RT_MODE_FULL if full else rt.RT_MODE_PRIMARY
    rgb, face, t, _ = sc.render(look_at(rt, W, H, eye, (0, 0, 0), up, fovy), rt.DEFAULT_LIGHTS, W, H, mode=m,
                                want_hits=True)
    orgb, oface, ot = osc.render(look_at(orc, W, H, eye, (0, 0, 0), up, fovy), orc.DEFAULT_LIGHTS, W, H,
                                 full=full, threads=THREADS)
    e = frame_errors(rgb, face, t, orgb, oface, ot)
    hits = int((np.asarray(oface) >= 0).sum())
    PARITY_REPORT.append(f"far eye {name} at {dist} extents dir {direction} {W}x{H} {mode}: {hits} hit pixels, "
                         f"face mismatches {e['face_mismatch']}, t mismatches {e['t_mismatch']}, "
                         f"colour L_inf {e['linf']:.3g}")
    assert hits > W * H // 20, "the view must hit the scene"
    assert e["face_mismatch"] == 0 and e["t_mismatch"] == 0 and e["nan_mismatch"] == 0, e
    assert e["linf"] < TOL, e


def test_grazing_view_matches_oracle(rt, orc, scenes):
    """Rays nearly parallel to the cube's top face plane, from 200 extents: the hit points' rounding across
    that plane decides the reference's inclusive edge tests."""
    sc, osc = scenes["cube"]
    W, H = 320, 240
    # the cube's faces are axis aligned; look along -z from just above the top face's plane
    b6, _, _ = osc.boxes()
    top = float(b6[:, 4].max())  # object-space high y of the reference boxes
    eye = (0.0, 0.0, 200.0)
    fovy = math.degrees(2 * math.atan(0.8 / 200.0))
    rgb, face, t, _ = sc.render(look_at(rt, W, H, eye, (0, 0, 0), (0, 1, 0), fovy), rt.DEFAULT_LIGHTS, W, H,
                                mode=rt.RT_MODE_FULL, want_hits=True)
    orgb, oface, ot = osc.render(look_at(orc, W, H, eye, (0, 0, 0), (0, 1, 0), fovy), orc.DEFAULT_LIGHTS, W, H,
                                 full=True, threads=THREADS)
    e = frame_errors(rgb, face, t, orgb, oface, ot)
    PARITY_REPORT.append(f"grazing view cube from 200 extents (top {top:.3g}): face mismatches "
                         f"{e['face_mismatch']}, t mismatches {e['t_mismatch']}, colour L_inf {e['linf']:.3g}")
    assert int((np.asarray(oface) >= 0).sum()) > 0
    assert e["face_mismatch"] == 0 and e["t_mismatch"] == 0 and e["linf"] < TOL, e


def _targets(sc_np_vertices, faces, rng, n):
    """Points on random faces: vertices, edge midpoints and interior points (where the reference's
    inclusive edge tests are decided by rounding)."""
    fi = rng.integers(0, len(faces), n)
    w = sc_np_vertices[faces[fi]]  # [n, 3 vertices, 3]
    kind = rng.integers(0, 3, n)
    bary = rng.dirichlet((1, 1, 1), n)
    bary[kind == 0] = np.eye(3)[rng.integers(0, 3, (kind == 0).sum())]
    e = rng.integers(0, 3, (kind == 1).sum())
    mid = np.full(((kind == 1).sum(), 3), 0.5)
    mid[np.arange(len(e)), e] = 0.0
    bary[kind == 1] = mid
    return np.einsum("nk,nkc->nc", bary, w)


def test_far_origin_ray_queries_match_oracle(rt, orc, scenes):
    """rt_trace_closest / rt_trace_shadow (calculateMinimumFace, shadow()) from origins up to 1e7 scene
    extents away, aimed at vertices, edge midpoints and interior points of the bunny's faces."""
    sc, osc = scenes["bunny"]
    rng = np.random.default_rng(11)
    ex = rt.Mesh.load_obj(scene_path("bunny.obj")).export()
    M = np.asarray(ex["M16"], np.float64).reshape(4, 4).T  # column-major Affine3f
    v = np.asarray(ex["v4"], np.float64)
    wv = (M[:3, :3] @ (v[:, :3] / v[:, 3:4]).T).T + M[:3, 3]
    n = 4096
    tgt = _targets(wv, np.asarray(ex["fidx"], np.int64), rng, n)
    dists = 10.0 ** rng.uniform(1, 7, n)
    u = rng.normal(size=(n, 3))
    u /= np.linalg.norm(u, axis=1, keepdims=True)
    o = (tgt + dists[:, None] * u).astype(np.float32)
    d = (-u).astype(np.float32)
    face, t, P = sc.trace_closest(o, d)
    oface, ot, oP = osc.closest(o, d)
    hits = int((oface >= 0).sum())
    mism = int((face != oface).sum())
    tm = int((~same_bits(t, ot)).sum())
    PARITY_REPORT.append(f"far-origin queries (bunny, 10..1e7 extents, {n} rays): {hits} hits, face mismatches "
                         f"{mism}, t mismatches {tm}")
    assert hits > n // 10
    assert mism == 0 and tm == 0
    assert same_bits(P[face >= 0], oP[oface >= 0]).all()
    # shadow(): the ray from P (+0.003 L for the triangle tests) towards L passes through the target
    L = u.astype(np.float32)
    Pf = (tgt - dists[:, None] * u).astype(np.float32)
    blk = sc.trace_shadow(Pf, L)
    oblk = osc.shadow(Pf, L)
    assert (blk == oblk).all(), int((blk != oblk).sum())
    assert int(oblk.sum()) > n // 10


def test_uncertified_origins_brute_force(rt, orc, scenes):
    """Origins beyond 1e18, directions below 1e-12 or above 1e18 in every component, and non-finite
    input: the culling pad is unbounded (every box entered, every triangle tested exactly), so the GPU
    still returns the reference's answer."""
    sc, osc = scenes["cube"]
    rng = np.random.default_rng(5)
    n = 256
    u = rng.normal(size=(n, 3))
    u /= np.linalg.norm(u, axis=1, keepdims=True)
    o = (1e20 * u).astype(np.float32)
    d = (-u).astype(np.float32)
    o[:16] = rng.uniform(-0.2, 0.2, (16, 3)).astype(np.float32) + np.float32([0, 0, 3])
    d[:16] = np.float32([0, 0, -1e-14])  # tiny direction (brute force), still aimed at the cube
    d[16:20] = np.float32([0, 0, -1e20])  # huge direction
    o[16:20] = np.float32([0.1, 0.1, 3])
    o[20:22] = np.float32([np.nan, 0, 3])
    o[22:24] = np.float32([np.inf, 0, 3])
    face, t, P = sc.trace_closest(o, d)
    oface, ot, oP = osc.closest(o, d)
    assert (face == oface).all(), np.nonzero(face != oface)
    assert same_bits(t, ot).all()
    blk = sc.trace_shadow(o, -d)
    oblk = osc.shadow(o, -d)
    assert (blk == oblk).all()
