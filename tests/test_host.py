"""CPU tests of the product library's host side (no GPU needed): the C-ABI loads and exports every
declared symbol, and the host-side stages of the path (Tucano ingest, camera, reference box
partition, BVH build, PPM writer, Eigen-order math) agree bit for bit with the pinned oracle."""
import os
import re

import numpy as np
import pytest

from conftest import GOLDEN, ROOT, scene_path
from test_oracle_pinning import read_kat, same_bits

HEADER = os.path.join(ROOT, "include", "rt", "rt_api.h")
SCENES = ["cube", "plane", "testding", "cornell", "dodgeColorTest", "bunny"]


def test_header_symbols_exported(rt):
    decl = set(re.findall(r"\b(rt_[a-z_0-9]+)\s*\(", open(HEADER).read()))
    assert decl == set(rt.EXPORTS), decl ^ set(rt.EXPORTS)
    L = rt.lib()
    for name in sorted(decl):
        assert hasattr(L, name), name
    want = int(re.search(r"#define RT_API_VERSION (\d+)", open(HEADER).read()).group(1))
    assert L.rt_version() == want == 4
    ident = rt.build_identity()
    assert ident["matches_tree"], ident


def test_no_device_is_reported_not_faked(rt):
    # in the CPU container there is no GPU: render entry points must fail loudly
    if rt.device_count() > 0:
        pytest.skip("GPU visible")
    mesh = rt.Mesh.load_obj(scene_path("cube.obj"))
    with pytest.raises(rt.RTError, match="no HIP device"):
        rt.Scene(mesh)
    sc = rt.Scene(mesh, device=rt.RT_DEVICE_NONE)
    with pytest.raises(rt.RTError, match="host-only"):
        sc.render(rt.flycam(64, 64), rt.DEFAULT_LIGHTS, 64, 64)
    # a multi-device scene without devices: the same loud failure, never a smaller scene
    for devs in ([0, 1], [0, 0], rt.RT_DEVICES_ALL):
        with pytest.raises(rt.RTError, match="no HIP device"):
            rt.Scene(mesh, devices=devs)


def test_device_list_rules_without_gpu(rt, tmp_path):
    """rt_scene_opts.n_devices / devices (API 4): a host-only scene lists no devices; the list length is
    bounded; rt_scene_load applies the same rules; the ctypes mirror has the C struct's size."""
    import ctypes as C
    mesh = rt.Mesh.load_obj(scene_path("cube.obj"))
    with pytest.raises(rt.RTError, match="lists no devices"):
        rt.Scene(mesh, device=rt.RT_DEVICE_NONE, devices=[0, 1])
    sc = rt.Scene(mesh, device=rt.RT_DEVICE_NONE)
    assert sc.info()["n_devices"] == 0
    p = str(tmp_path / "cube.rtscene")
    sc.save(p)
    with pytest.raises(rt.RTError, match="lists no devices"):
        rt.Scene.load(p, device=rt.RT_DEVICE_NONE, devices=[0])
    with pytest.raises(ValueError):
        rt.scene_opts(devices=list(range(rt.RT_MAX_DEVICES + 1)))
    o = rt.scene_opts(devices=[3, 3, 1])
    assert o.n_devices == 3 and list(o.devices[:3]) == [3, 3, 1]
    # struct layout: n_devices right after wide_tree, devices[16] after it (rt_api.h)
    assert rt.SceneOpts.n_devices.offset == rt.SceneOpts.wide_tree.offset + 4
    assert C.sizeof(rt.SceneOpts) == rt.SceneOpts.devices.offset + 4 * rt.RT_MAX_DEVICES


@pytest.mark.parametrize("name", SCENES)
def test_ingest_matches_oracle(rt, orc, name):
    a = rt.Mesh.load_obj(scene_path(name + ".obj")).export()
    b = orc.Mesh.load_obj(scene_path(name + ".obj")).export()
    for k in ("v4", "vn3", "fidx", "fn3", "fmat", "mats", "M16"):
        assert a[k].shape == b[k].shape, k
        assert same_bits(a[k], b[k]).all() if a[k].dtype == np.float32 else (a[k] == b[k]).all(), k


def test_soup_generator_matches_oracle(rt, orc):
    a = rt.generate_soup(20000, 12345)
    b = orc.generate_soup(20000, 12345)
    assert a.tobytes() == b.tobytes()
    assert np.abs(a).max() <= 0.51


@pytest.mark.parametrize("dxyz", [(0, 0, 0), (0, 0, 20), (3, -2, 7)])
@pytest.mark.parametrize("WH", [(256, 256), (1920, 1080), (37, 11)])
def test_camera_matches_oracle(rt, orc, dxyz, WH):
    a = rt.flycam(*WH, *dxyz)
    b = orc.flycam(*WH, *dxyz)
    for f in ("view", "viewport"):
        pass
    assert list(a.view_matrix) == list(b.view)
    assert list(a.viewport) == list(b.viewport)
    assert a.fovy == b.fovy and a.aspect_ratio == b.aspect


@pytest.mark.parametrize("dxyz", [(0, 0, 0), (0, 0, 20), (3, -2, 7), (-0.2, 0.0, 0.2)])
def test_camera_path_matches_flycam(rt, dxyz):
    """The moving-camera path (rtamd.CameraPath: Flyscene::simulate's WASD translate per frame, float
    accumulation of Flycamera::translation_vector) starts at exactly the pose rt_camera_flycam gives for the same
    translate, and every step moves the pose by the reference's 0.2 x speed 0.05 per held key."""
    W, H = 1920, 1080
    p = rt.CameraPath(W, H, *dxyz)
    a, b = p.camera(), rt.flycam(W, H, *dxyz)
    assert list(a.view_matrix) == list(b.view_matrix)
    assert list(a.viewport) == list(b.viewport) and a.fovy == b.fovy and a.aspect_ratio == b.aspect_ratio
    cams = p.take(120)
    t = np.array([[c.view_matrix[12], c.view_matrix[13], c.view_matrix[14]] for c in cams], np.float64)
    step = np.abs(np.diff(t, axis=0))
    assert np.allclose(step[:, 0], 0.01, atol=1e-6) and np.allclose(step[:, 2], 0.01, atol=1e-6)
    assert (step[:, 1] == 0).all()
    # the path turns round (W <-> S every 40 frames, D <-> A every 25): bounded, and every frame a new pose
    assert np.ptp(t[:, 2]) <= 0.41 and np.ptp(t[:, 0]) <= 0.26
    assert len({tuple(x) for x in t}) > 100


def test_moving_camera_prediction_geometry(rt):
    """The moving camera's cost-map prediction (rt_kernels.h wave_clock_end, FrameParams::pred): a hit at distance t
    along pixel (px, py)'s view-space direction (a px + b, c py + e, -1), moved by the camera's last step
    (rt_device.hip camera_step: the translation of V_n V_(n-1)^-1) and projected back, lands on the pixel where the
    same world point appears in the path's next frame. The same algebra as the kernel, in float64, against the
    reference camera path's actual next pose (WASD translate, Flyscene::simulate)."""
    W, H = 1920, 1080
    cams = rt.CameraPath(W, H).take(30)

    def V(c):
        return np.array(c.view_matrix, np.float64).reshape(4, 4).T

    def pixel(c, p):
        q = V(c) @ np.append(p, 1.0)
        xs, ys = c.aspect_ratio * np.tan(np.radians(c.fovy / 2)), np.tan(np.radians(c.fovy / 2))
        nx, ny = (q[0] / -q[2]) / xs, (q[1] / -q[2]) / ys
        return np.array([(nx + 1) / 2 * c.viewport[2] + c.viewport[0], (1 - ny) / 2 * c.viewport[3] + c.viewport[1]]), q

    rng = np.random.default_rng(7)
    for n in (1, 10, 24, 25, 26):  # frame 25 moves A after 25 frames of D: a one-frame miss of the prediction
        prev, cur, nxt = cams[n - 1], cams[n], cams[n + 1]
        xs, ys = cur.aspect_ratio * np.tan(np.radians(cur.fovy / 2)), np.tan(np.radians(cur.fovy / 2))
        vp = np.array(cur.viewport, np.float64)
        a, b = 2 * xs / vp[2], -(2 * vp[0] / vp[2] + 1) * xs
        c, e = -2 * ys / vp[3], (1 + 2 * vp[1] / vp[3]) * ys
        step = (V(cur) @ np.linalg.inv(V(prev)))[:3, 3]
        for p in rng.uniform([-0.5, -0.5, -0.6], [0.5, 0.5, 0.2], (20, 3)):
            (px, py), q = pixel(cur, p)
            t = np.linalg.norm(q[:3])
            dx, dy = a * px + b, c * py + e
            k = t / np.sqrt(dx * dx + dy * dy + 1)
            qx, qy, qz = dx * k + step[0], dy * k + step[1], step[2] - k
            pred = np.array([(qx / -qz - b) / a, (qy / -qz - e) / c])
            true, _ = pixel(nxt, p)
            if n == 25:  # the step reverses: the prediction misses (by twice the x step)
                assert np.abs(pred - true).max() > 1e-3
            else:
                assert np.abs(pred - true).max() < 1e-6


def test_moving_pose_fixture_matches_bench():
    """The committed moving-camera digests (tools/gen_fullframe_digests.py) are of the pose bench.py and the GPU
    test check: the same MOVE_POSE, and the fixture records the view translation that pose has."""
    import importlib.util
    import json

    def load(name, path):
        spec = importlib.util.spec_from_file_location(name, path)
        m = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(m)
        return m
    bench = load("bench_mp", os.path.join(ROOT, "bench.py"))
    gen = load("gen_mp", os.path.join(ROOT, "tools", "gen_fullframe_digests.py"))
    src = open(os.path.join(ROOT, "tests", "test_gpu_fullframe.py")).read()
    assert bench.MOVE_POSE == gen.MOVE_POSE and f"MOVE_POSE = {bench.MOVE_POSE}" in src
    dig = json.load(open(os.path.join(GOLDEN, "fullframe_digests.json")))
    import importlib
    rt = importlib.import_module("conftest").rtamd
    for case in ("C3-moving", "C5-moving"):
        d = dig[case]
        assert d["camera_path_pose"] == bench.MOVE_POSE
        p = rt.CameraPath(d["W"], d["H"])
        p.take(bench.MOVE_POSE)
        c = p.camera()
        assert [c.view_matrix[12], c.view_matrix[13], c.view_matrix[14]] == d["view_translation"]


@pytest.mark.parametrize("sec", read_kat(), ids=lambda s: f"op{s[0]}")
def test_host_math_matches_eigen(rt, sec):
    op, n, il, ol, inp, exp = sec
    got = rt.debug_math(op, inp, n, ol, device=False)
    bad = (~same_bits(got, exp)).reshape(n, ol).any(1)
    assert bad.sum() == 0, f"op {op}: {bad.sum()} cases differ"


def pow_cases(seed=7, n=20000):
    """Inputs of op 17 (calcSingleColor's std::pow, flyscene.cpp:562): specular dots in [-1, 1] plus
    special values, against integer exponents (the fast path) and non-integer / out-of-range ones."""
    rng = np.random.default_rng(seed)
    xs = np.concatenate([rng.uniform(-1, 1, n), rng.uniform(0.9, 1.0, n), rng.uniform(-4, 4, n // 4),
                         [0.0, -0.0, 1.0, -1.0, 1e-30, -1e-30, 3e38, np.inf, -np.inf, np.nan, 1e-45]]).astype(np.float32)
    ints = np.array([0, 1, 2, 3, 5, 16, 32, 100, 1000, 1023], np.float32)
    frac = np.array([0.5, 1.5, 10.25, 32.5, 1024, 2000, -1, -2.5], np.float32)
    return xs, ints, frac


def pairs(xs, ys):
    return np.stack(np.broadcast_arrays(xs[:, None], ys[None, :]), -1).reshape(-1, 2).astype(np.float32)


def ulp_diff(a, b):
    ai, bi = a.view(np.int32).astype(np.int64), b.view(np.int32).astype(np.int64)
    ai = np.where(ai < 0, -(ai & 0x7FFFFFFF), ai)
    bi = np.where(bi < 0, -(bi & 0x7FFFFFFF), bi)
    d = np.abs(ai - bi)
    return np.where(np.isnan(a) & np.isnan(b), 0, d)


def test_host_pow_integer_fast_path(rt):
    """op 17 on the host: integer exponents use fp64 binary exponentiation; the float result must be the
    correctly rounded x^n (fp64 pow rounded once) and within 1 ulp of the reference's glibc powf."""
    xs, ints, frac = pow_cases()
    for ys in (ints, frac):
        inp = pairs(xs, ys)
        got = rt.debug_math(17, inp.reshape(-1), len(inp), 1, device=False).reshape(-1)
        with np.errstate(all="ignore"):
            cr = np.power(inp[:, 0].astype(np.float64), inp[:, 1].astype(np.float64)).astype(np.float32)
            pf = np.power(inp[:, 0], inp[:, 1])  # float32 power: the C library's powf
        assert same_bits(got, cr).all(), f"{int((~same_bits(got, cr)).sum())} cases differ from fp64 pow"
        assert ulp_diff(got, pf).max() <= 1


@pytest.mark.parametrize("name", ["cube", "dodgeColorTest", "bunny"])
def test_reference_boxes_match_oracle(rt, orc, name):
    sc = rt.Scene(rt.Mesh.load_obj(scene_path(name + ".obj")), device=rt.RT_DEVICE_NONE)
    osc = orc.Scene(orc.Mesh.load_obj(scene_path(name + ".obj")))
    b6, cnt, order = sc.ref_boxes()
    ob6, ocnt, oorder = osc.boxes()
    assert len(cnt) == len(ocnt)
    assert (cnt == ocnt).all() and (order == oorder).all()
    assert same_bits(b6, ob6).all()


def test_reference_boxes_soup_match_oracle(rt, orc):
    n = 200000
    mesh, v, f = rt.soup_mesh(n)
    sc = rt.Scene(mesh, device=rt.RT_DEVICE_NONE)
    om = orc.Mesh.from_arrays(v, f, np.array([rt.SOUP_MATERIAL], np.float32))
    osc = orc.Scene(om)
    b6, cnt, order = sc.ref_boxes()
    ob6, ocnt, oorder = osc.boxes()
    assert (cnt == ocnt).all() and (order == oorder).all() and same_bits(b6, ob6).all()
    info = sc.info()
    assert info["n_ref_boxes"] == len(ocnt)
    assert 0 < info["bvh_depth"] <= 60
    assert info["bvh_nodes"] >= 1 and info["bvh_leaves"] >= n // 16


def test_bvh_bounds_sane_for_empty_and_single(rt):
    # a single triangle and a one-leaf scene build a valid root
    v = np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0]], np.float32)
    mesh = rt.Mesh.from_arrays(v, np.array([[0, 1, 2]], np.uint32), np.array([rt.SOUP_MATERIAL], np.float32))
    info = rt.Scene(mesh, device=rt.RT_DEVICE_NONE).info()
    assert info["n_faces"] == 1 and info["bvh_nodes"] == 1 and info["n_ref_boxes"] == 1
    empty = rt.Mesh.from_arrays(np.zeros((0, 3), np.float32), np.zeros((0, 3), np.uint32),
                                np.array([rt.SOUP_MATERIAL], np.float32), groups=[])
    info = rt.Scene(empty, device=rt.RT_DEVICE_NONE).info()
    assert info["n_faces"] == 0 and info["bvh_nodes"] == 0


def _soup(rt, n, seed=3, scale=1.0, flat_axis=None):
    v = rt.generate_soup(n, seed) * np.float32(scale)
    if flat_axis is not None:
        v[:, flat_axis] = np.float32(0.25 * scale)
    return rt.Mesh.from_arrays(v, np.arange(3 * n, dtype=np.uint32).reshape(-1, 3),
                               np.array([rt.SOUP_MATERIAL], np.float32))


@pytest.mark.parametrize("case", ["cube", "dodgeColorTest", "bunny", "soup200k", "flat", "tiny", "huge",
                                  "coincident", "single", "two"])
def test_bvh_trees_sound(rt, case):
    """Binary and 4-wide trees: every triangle inside every ancestor box (the wide boxes dequantised
    exactly as the kernel does) -- for a spatial-split tree every reference's part inside its path's
    boxes and every face covered by its leaves' regions --, every triangle record in exactly one leaf;
    depth fits the stacks."""
    if case in ("cube", "dodgeColorTest", "bunny"):
        mesh = rt.Mesh.load_obj(scene_path(case + ".obj"))
    elif case == "soup200k":
        mesh = _soup(rt, 200_000)
    elif case == "flat":
        mesh = _soup(rt, 20_000, flat_axis=2)
    elif case == "tiny":
        mesh = _soup(rt, 20_000, scale=1e-6)
    elif case == "huge":
        mesh = _soup(rt, 20_000, scale=1e6)
    elif case == "coincident":
        v = np.tile(np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0]], np.float32), (500, 1))
        mesh = rt.Mesh.from_arrays(v, np.arange(1500, dtype=np.uint32).reshape(-1, 3),
                                   np.array([rt.SOUP_MATERIAL], np.float32))
    else:
        mesh = _soup(rt, 1 if case == "single" else 2)
    sc = rt.Scene(mesh, device=rt.RT_DEVICE_NONE, wide_tree=1)
    r = sc.validate_bvh()  # the fp32 4-wide tree too (violations count all three trees)
    assert r["ok"] and r["violations"] == 0, r
    info = sc.info()
    assert info["wide_nodes"] >= 1 or info["bvh_nodes"] <= 1
    assert 3 * info["wide_depth"] + 4 <= 128
    nf = info["n_faces"]
    # every triangle record in exactly one leaf; spatial splits may reference a face from several leaves
    # (the validator then checks that the faces' leaf regions cover them), within the reference budget
    assert nf <= r["covered2"] <= 1.5 * nf + 1 and r["covered4"] == r["covered2"]
    assert r["nodes4"] >= 1 and r["depth4"] <= r["depth2"] and 3 * r["depth4"] + 4 <= 128


def test_record_layout_keeps_wide_offsets_below_leaf_bit(rt):
    # a wide interior handle is its record's byte offset and bit 31 marks a leaf, so
    # the wide copies are placed only while every record offset stays below 2^31 (else binary tree only)
    assert rt.record_layout(0, 0, 0) == (0, 0)
    nb, wb = rt.record_layout(1_145_405, 1_190_000, 400_000)  # the 1M soup's sizes: wide tree placed
    base = (1_145_405 + 1_190_000) * 64
    assert wb == (base + 127) // 128 * 128 and nb == wb + 8 * 400_000 * 128
    for n_wide in (1, 10, 1000):
        # largest binary + triangle records for which the wide copies still end at or below 2^31
        room = 2 ** 31 - 8 * n_wide * 128
        nn = room // 64 // 2
        nt = room // 64 - nn
        nb, wb = rt.record_layout(nn, nt, n_wide)
        assert wb != 0 and wb + 8 * n_wide * 128 - 128 < 2 ** 31 and nb <= 2 ** 31
        # one more record pushes the last wide record to 2^31: dropped, the binary tree serves alone
        nb, wb = rt.record_layout(nn, nt + 2, n_wide)
        assert wb == 0 and nb == (nn + nt + 2) * 64
    # a ~7M-face SBVH scene (the advisor's case: ~2.2 GiB of binary + triangle records) keeps no wide tree
    nb, wb = rt.record_layout(8_000_000, 8_300_000, 2_700_000)
    assert wb == 0 and nb == 16_300_000 * 64
    # records beyond 4 GiB cannot be addressed at all
    assert rt.record_layout(2 ** 26, 1, 0) == (0, 0)


def test_ppm_writer_format(rt, tmp_path):
    rgb = np.array([[[0.0, 0.5, 1.0], [1.5, -0.25, 0.999]]], np.float32)
    p = tmp_path / "x.ppm"
    rt.write_ppm(str(p), rgb)
    # writePPMImage: "P3\nW H\n255\n", min(255,(int)(255*c)) with " " after each value, "\n" per row
    assert p.read_text() == "P3\n2 1\n255\n0 127 255 255 -63 254 \n"


def test_invalid_inputs_rejected(rt, tmp_path):
    with pytest.raises(rt.RTError, match="Cannot open"):
        rt.Mesh.load_obj(str(tmp_path / "missing.obj"))
    bad = tmp_path / "bad.obj"
    bad.write_text("v 0 0 0\nv 1 0 0\nf 1 2\n")
    with pytest.raises(rt.RTError, match="multiple of 3"):
        rt.Mesh.load_obj(str(bad))
    # out-of-range indices are rejected before anything indexes with them (the reference's
    # computeNormals would write out of bounds: objimporter.hpp:81-106)
    for faces in ("f 1 2 9", "f 0 1 2", "f -1 2 3"):
        bad.write_text("v 0 0 0\nv 1 0 0\nv 0 1 0\n" + faces + "\n")
        with pytest.raises(rt.RTError, match="out of range"):
            rt.Mesh.load_obj(str(bad))


def test_host_code_under_sanitizers():
    """Host entry points (OBJ ingest incl. malformed files, host-only scenes, BVH validation, the scene
    cache with truncated / bit-flipped files, PPM writers, lights) under AddressSanitizer + UBSan +
    LeakSanitizer: tools/asan/run.sh rebuilds the host translation units instrumented and fails on any
    report."""
    import shutil
    import subprocess
    if not os.path.exists("/opt/rocm/bin/hipcc") or shutil.which("make") is None:
        pytest.skip("needs hipcc + make")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run(["bash", os.path.join(root, "tools", "asan", "run.sh")], capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0 and "host_asan: ok" in r.stdout, (r.stdout[-2000:] + r.stderr[-4000:])


@pytest.mark.parametrize("name", ["cube", "bunny"])
def test_scene_cache_roundtrip(rt, tmp_path, name):
    """f1 binary scene cache: save -> load restores the same boxes, face order and BVHs (re-saving the
    loaded scene reproduces the file byte for byte); damaged files are rejected."""
    sc = rt.Scene(rt.Mesh.load_obj(scene_path(name + ".obj")), device=rt.RT_DEVICE_NONE)
    p1, p2 = tmp_path / "a.rtscene", tmp_path / "b.rtscene"
    sc.save(p1)
    ld = rt.Scene.load(p1, device=rt.RT_DEVICE_NONE)
    a, b = sc.info(), ld.info()
    for k in ("n_faces", "n_vertices", "n_ref_boxes", "bvh_nodes", "bvh_leaves", "bvh_depth"):
        assert a[k] == b[k], k
    for x, y in zip(sc.ref_boxes(), ld.ref_boxes()):
        np.testing.assert_array_equal(x, y)
    assert ld.validate_bvh()["ok"]
    ld.save(p2)
    assert p1.read_bytes() == p2.read_bytes()
    raw = p1.read_bytes()
    bad = tmp_path / "bad.rtscene"
    for damaged in (raw[: len(raw) // 2], raw[:100] + bytes([raw[100] ^ 1]) + raw[101:], b"NOTASCENE" + raw[9:]):
        bad.write_bytes(damaged)
        with pytest.raises(rt.RTError):
            rt.Scene.load(bad, device=rt.RT_DEVICE_NONE)


# cache sections (version 2): header, wv, ov3, vnn, fnn, fdist, fidx, fmat, mats, boxes, box faces,
# face_rank, face_box, nodes, nodes4, tris
NODES = 13


def _cache_sections(raw):
    """Split a scene cache (rt_cache.cpp) into its written chunks: header, then the arrays in write order."""
    import struct
    nv, nf, nm, nb, nbf, nn, nn4, nt = struct.unpack_from("<8i", raw, 16)
    assert struct.unpack_from("<I", raw, 12)[0] == 256
    sizes = [256, 12 * nv, 12 * nv, 12 * nv, 12 * nf, 4 * nf, 12 * nf, 4 * nf, 48 * nm, 44 * nb, 4 * nbf, 4 * nf, 4 * nf,
             64 * nn, 64 * nn4, 64 * nt]
    out, off = [], 0
    for n in sizes:
        out.append(bytearray(raw[off:off + n]))
        off += n
    assert off + 8 == len(raw)
    return out


def _cache_sign(sections):
    """Re-assemble a cache with a valid content hash (the Hasher of rt_cache.cpp, chunk by chunk)."""
    M = (1 << 64) - 1
    h = 0x9E3779B97F4A7C15
    for b in sections:
        n = len(b)
        if n == 0:
            continue
        words = np.frombuffer(bytes(b[: n - n % 8]), "<u8")
        for w in words.tolist():
            h = ((h ^ w) * 0xBF58476D1CE4E5B9) & M
            h ^= h >> 31
        w = int.from_bytes(bytes(b[n - n % 8:]).ljust(8, b"\0"), "little")
        h = ((h ^ w ^ n) * 0x94D049BB133111EB) & M
        h ^= h >> 29
    return b"".join(bytes(x) for x in sections) + h.to_bytes(8, "little")


def test_scene_cache_rejects_crafted_trees(rt, tmp_path):
    """a cache whose content hash is valid but whose BVH is not a tree (a self-referencing
    child) or is deeper than the 64-entry wave stack is rejected on load; the depth is recomputed from
    the nodes, never trusted from the header."""
    import struct
    sc = rt.Scene(rt.Mesh.load_obj(scene_path("cube.obj")), device=rt.RT_DEVICE_NONE)
    p = tmp_path / "cube.rtscene"
    sc.save(p)
    raw = p.read_bytes()
    sec = _cache_sections(raw)
    assert _cache_sign(sec) == raw  # the re-signer reproduces the library's hash
    bad = tmp_path / "crafted.rtscene"
    # 1. node 0 (the root) lists itself as child 0
    s1 = [bytearray(x) for x in sec]
    struct.pack_into("<I", s1[NODES], 48, 0)
    bad.write_bytes(_cache_sign(s1))
    with pytest.raises(rt.RTError, match="not a tree"):
        rt.Scene.load(bad, device=rt.RT_DEVICE_NONE)
    # 2. a 70-level chain (each node once, so a tree) under a header that claims depth 3
    n = 70
    leaf0 = 0x80000000  # leaf handle: triangle 0, count 1
    chain = bytearray()
    for i in range(n):
        rec = bytearray(sec[NODES][:64])
        struct.pack_into("<II", rec, 48, i + 1 if i + 1 < n else leaf0, leaf0)
        chain += rec
    s2 = [bytearray(x) for x in sec]
    s2[NODES] = chain
    struct.pack_into("<i", s2[0], 36, n)        # n_nodes
    struct.pack_into("<i", s2[0], 40, 0)        # no wide tree
    struct.pack_into("<i", s2[0], 52, 3)        # depth (a lie)
    s2[NODES + 1] = bytearray()
    bad.write_bytes(_cache_sign(s2))
    with pytest.raises(rt.RTError, match="deeper than the traversal stack"):
        rt.Scene.load(bad, device=rt.RT_DEVICE_NONE)
    # 3. the same chain at 40 levels loads, with its real depth
    s3 = [bytearray(x) for x in s2]
    s3[NODES] = chain[: 40 * 64]
    struct.pack_into("<II", s3[NODES], 39 * 64 + 48, leaf0, leaf0)
    struct.pack_into("<i", s3[0], 36, 40)
    bad.write_bytes(_cache_sign(s3))
    assert rt.Scene.load(bad, device=rt.RT_DEVICE_NONE).info()["bvh_depth"] == 41
    # 4. ADVICE r2: a face-less file (no triangles, no boxes) with one interior node and its root handle
    # beyond the node table: rejected before the tree walk (which would index the node table with it)
    s4 = [bytearray(x) for x in sec]
    nv = struct.unpack_from("<i", s4[0], 16)[0]
    rec = bytearray(sec[NODES][:64])
    struct.pack_into("<II", rec, 48, 0, 0)  # both children: node 0 (interior)
    s4[NODES] = rec
    for k in range(4, 13):  # fnn, fdist, fidx, fmat, mats (kept), boxes, box faces, face_rank, face_box
        if k != 8:
            s4[k] = bytearray()
    s4[NODES + 1] = bytearray()
    s4[NODES + 2] = bytearray()
    struct.pack_into("<8i", s4[0], 16, nv, 0, struct.unpack_from("<i", s4[0], 24)[0], 0, 0, 1, 0, 0)
    struct.pack_into("<I", s4[0], 48, 7)  # root: node 7 of 1
    bad.write_bytes(_cache_sign(s4))
    with pytest.raises(rt.RTError, match="bad BVH root"):
        rt.Scene.load(bad, device=rt.RT_DEVICE_NONE)
    # 5. ADVICE r3: the records' flag bits (safe normal, box certificate) are recomputed on load, never
    # trusted: a file with every flag set loads with the flags the geometry earns
    want = sc.record_flags()
    s5 = [bytearray(x) for x in sec]
    tris = np.frombuffer(bytes(s5[NODES + 2]), "<u4").reshape(-1, 16).copy()
    tris[:, 15] |= 0xC0000000
    s5[NODES + 2] = bytearray(tris.tobytes())
    bad.write_bytes(_cache_sign(s5))
    assert rt.Scene.load(bad, device=rt.RT_DEVICE_NONE).record_flags() == want
    # 6. a record whose box index is not its face's reference box is rejected
    s6 = [bytearray(x) for x in sec]
    tris = np.frombuffer(bytes(s6[NODES + 2]), "<u4").reshape(-1, 16).copy()
    nb = struct.unpack_from("<i", s6[0], 28)[0]
    tris[0, 15] = (tris[0, 15] & 0xC0000000) | ((int(tris[0, 15] & 0x3FFFFFFF) + 1) % max(nb, 2))
    s6[NODES + 2] = bytearray(tris.tobytes())
    bad.write_bytes(_cache_sign(s6))
    with pytest.raises(rt.RTError, match="bad triangle record"):
        rt.Scene.load(bad, device=rt.RT_DEVICE_NONE)


def _rotation(ax_deg, ay_deg):
    """column-major 4x4 rotation about x then y (an Affine3f modelMatrix)"""
    a, b = np.radians(ax_deg), np.radians(ay_deg)
    rx = np.array([[1, 0, 0], [0, np.cos(a), -np.sin(a)], [0, np.sin(a), np.cos(a)]])
    ry = np.array([[np.cos(b), 0, np.sin(b)], [0, 1, 0], [-np.sin(b), 0, np.cos(b)]])
    m = np.eye(4)
    m[:3, :3] = ry @ rx
    return m.T.astype(np.float32).reshape(16)  # column-major


def test_box_certificates_need_a_similarity_and_matching_normals(rt, orc):
    """the box certificates argue from the world triangle, whose normal is the face normal only
    under the loader's own normalisation; a rotated or non-uniformly scaled model matrix (the face normals
    stay the object-space ones, as in the reference) leaves the edge tests' accepted region tilted, so no
    face may be certified then. A uniform scale keeps them."""
    path = scene_path("bunny.obj")
    base = rt.Scene(rt.Mesh.load_obj(path), device=rt.RT_DEVICE_NONE)
    n, safe, cert = base.record_flags()
    assert cert > 0.8 * n, (n, safe, cert)
    cases = {"rotated": _rotation(20, 30), "stretched": np.diag([1.0, 1.0, 1.5, 1.0]).astype(np.float32).reshape(16),
             "uniform": np.diag([2.0, 2.0, 2.0, 1.0]).astype(np.float32).reshape(16)}
    for name, model in cases.items():
        om = orc.Mesh.load_obj(path)
        om.set_model(model)
        M16 = om.export()["M16"]
        sc = rt.Scene(rt.Mesh.load_obj(path), device=rt.RT_DEVICE_NONE, shape_model_matrix=M16)
        n2, _, cert2 = sc.record_flags()  # references (a spatial-split tree's count depends on the pose)
        if name == "uniform":
            assert cert2 > 0.8 * n2, (name, cert2)
        else:
            assert cert2 == 0, (name, cert2)


@pytest.mark.parametrize("model", ["rotated", "stretched"])
def test_tilted_normals_trees_bound_the_accept_region(rt, orc, model):
    """Under a rotating or non-uniformly scaling model matrix the reference tests world edges against the
    object-space face normal n (flyscene.cpp:444-478, 573-590), so the hit points it accepts lie on the world
    triangle projected along n onto n's plane (rt_host.cpp accept_region), up to a few % of a triangle's
    size away from the world triangle. The oracle's hits must lie in that projection's box (the theory), a
    good share of them outside the world triangle's box (why the builders must bound the projection), and
    every tree must hold the projections (the validator, which checks bound_vert boxes)."""
    path = scene_path("bunny.obj")
    M = _rotation(20, 30) if model == "rotated" else np.diag([1.0, 0.8, 1.5, 1.0]).astype(np.float32).reshape(16)
    om = orc.Mesh.load_obj(path)
    om.set_model(M)
    ex = om.export()
    osc = orc.Scene(om)
    for builder in (rt.RT_BUILDER_SBVH, rt.RT_BUILDER_SAH):
        sc = rt.Scene(rt.Mesh.load_obj(path), device=rt.RT_DEVICE_NONE, shape_model_matrix=ex["M16"], builder=builder)
        v = sc.validate_bvh()
        assert v["ok"] and v["violations"] == 0, (builder, v)
    Mm = np.asarray(ex["M16"], np.float64).reshape(4, 4).T
    v4 = np.asarray(ex["v4"], np.float64)
    wv = (Mm[:3, :3] @ (v4[:, :3] / v4[:, 3:4]).T).T + Mm[:3, 3]
    fidx = np.asarray(ex["fidx"], np.int64)
    n = np.asarray(ex["fn3"], np.float64)
    n /= np.linalg.norm(n, axis=1, keepdims=True)
    w = wv[fidx]  # [nf, 3, 3]
    s = (np.einsum("fkc,fc->fk", w, n) - np.einsum("fc,fc->f", w[:, 0], n)[:, None])
    proj = w - s[..., None] * n[:, None, :]
    rng = np.random.default_rng(5)
    lo, hi = wv.min(0), wv.max(0)
    eye = np.array([0.4, 0.3, 2.2])
    tgt = lo + rng.random((3000, 3)) * (hi - lo)
    d = tgt - eye
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    o = np.broadcast_to(eye, d.shape).astype(np.float32)
    face, t, P = osc.closest(o, d.astype(np.float32))
    hit = face >= 0
    assert hit.sum() > 500
    f = face[hit]
    P = np.asarray(P, np.float64)[hit]
    diam = np.linalg.norm(w[f] - np.roll(w[f], 1, axis=1), axis=2).max(1)
    tol = 1e-4 * diam[:, None] + 1e-6
    pb_lo, pb_hi = proj[f].min(1), proj[f].max(1)
    assert ((P >= pb_lo - tol) & (P <= pb_hi + tol)).all()
    wb_lo, wb_hi = w[f].min(1), w[f].max(1)
    outside_world = ~((P >= wb_lo - tol) & (P <= wb_hi + tol)).all(1)
    assert outside_world.sum() > 0.01 * len(f), int(outside_world.sum())


def test_ppm_rgb8_writer_matches_float_writer(rt, tmp_path):
    """f3: the 8-bit P3 writer produces writePPMImage's exact bytes for in-range values."""
    rng = np.random.default_rng(3)
    rgb = rng.uniform(0, 1, (37, 53, 3)).astype(np.float32)
    rgb[0, 0] = [0.0, 1.0, 0.999]
    a, b = tmp_path / "a.ppm", tmp_path / "b.ppm"
    rt.write_ppm(a, rgb)
    v = np.minimum(255, (np.float32(255) * rgb).astype(np.int64)).astype(np.uint8)
    rt.write_ppm_rgb8(b, v)
    assert a.read_bytes() == b.read_bytes()


def test_box_colors_random_matches_glibc(rt, orc):
    """RENDER_BOUNDINGBOX_COLORED_TRIANGLES colours: setRandomColor per box in creation order
    (BoundingBox.cpp:163-165) = Vector3f(rand() / (float)RAND_MAX, x3) from the C library's own srand(1) +
    rand(), the constructor's arguments evaluated as g++ compiles the reference's expression (right to
    left: tests/golden/boxcolor_kat.bin from oracle/boxcolor_kat.cpp)."""
    kat = np.fromfile(os.path.join(GOLDEN, "boxcolor_kat.bin"), np.float32).reshape(-1, 3)
    got = rt.box_colors_random(4480)
    assert got.tobytes() == kat.tobytes()
    assert got.tobytes() == orc.box_colors_glibc(4480).tobytes()
    r = rt.Rand(7)
    a = rt.box_colors_random(10, r)
    b = rt.box_colors_random(10, r)  # the state advances: 30 rand() calls per 10 boxes
    r2 = rt.Rand(7)
    seq = np.array([r2() for _ in range(60)], np.float32).reshape(-1, 3)[:, ::-1] / np.float32(2147483647)
    assert np.concatenate([a, b]).reshape(-1).tobytes() == np.ascontiguousarray(seq).reshape(-1).tobytes()


def test_scene_box_colors_arguments(rt):
    sc = rt.Scene(rt.Mesh.load_obj(scene_path("dodgeColorTest.obj")), device=rt.RT_DEVICE_NONE)
    nb = sc.info()["n_ref_boxes"]
    sc.set_box_colors()
    sc.set_box_colors(np.ones((nb, 3), np.float32))
    with pytest.raises(ValueError):
        sc.set_box_colors(np.ones((nb + 1, 3), np.float32))
    assert rt.lib().rt_scene_set_box_colors(None, None) == -1


def test_rand_matches_glibc(rt):
    """f4: rt_rand reproduces the C library's rand() the reference calls (glibc, unseeded = seed 1)."""
    import ctypes
    libc = ctypes.CDLL("libc.so.6")
    for seed in (1, 12345, 0xFFFFFFFF):
        libc.srand(ctypes.c_uint(seed))
        ref = [libc.rand() for _ in range(2000)]
        r = rt.Rand(seed)
        assert [r() for _ in range(2000)] == ref, seed


def test_spherical_light_expansion(rt):
    """f4: sphericalLight + addLight('s') restated in float32 with the same rand() sequence."""
    import ctypes
    libc = ctypes.CDLL("libc.so.6")
    libc.srand(ctypes.c_uint(1))
    pos, col, radius, n = (0.3, -1.25, 2.5), (0.9, 0.6, 0.3), 0.35, 6
    got = rt.spherical_light(pos, col, radius, n, rng=rt.Rand(1))
    f = np.float32
    q = f(2147483647) / (f(radius) * f(2))
    div = f(n + 1)
    for i in range(n):
        off = [-f(radius) + (f(libc.rand()) / q) for _ in range(3)]
        exp = tuple(f(pos[k]) + off[k] for k in range(3))
        assert np.array_equal(np.array(got[i][0], f), np.array(exp, f)), i
        assert np.array_equal(np.array(got[i][1], f), np.array(col, f) / div)
    assert np.array_equal(np.array(got[n][0], f), np.array(pos, f))
    assert len(got) == n + 1


def test_directional_light_is_screen_centre(rt, orc):
    """f4: addLight('d') stores screenToWorld(viewport centre): normalising (that - eye) gives the oracle's
    primary-ray direction of the centre pixel bit for bit."""
    for W, H, dz in ((1920, 1080, 20), (256, 256, 0)):
        cam = rt.flycam(W, H, 0, 0, dz)
        v, _, kind = rt.directional_light(cam, (1, 1, 1))
        assert kind == rt.RT_LIGHT_DIRECTIONAL
        o, d = orc.camera_ray(orc.flycam(W, H, 0, 0, dz), W // 2, H // 2)
        diff = np.array(v, np.float32) - np.array(o, np.float32)
        n = np.float32(np.sqrt(np.float32(diff[0] * diff[0] + (diff[1] * diff[1] + diff[2] * diff[2]))))
        assert np.array_equal((diff / n).astype(np.float32), np.array(d, np.float32))


def test_face_limit_rejected_before_reading(rt):
    """Scenes beyond the 32-bit record addressing limit (2^25 - 1 faces, rt_api.h) are refused up front,
    before any array is read (the descriptor's pointers still describe the 12-face cube)."""
    import ctypes as C
    m = rt.Mesh.load_obj(scene_path("cube.obj"))
    d = m.desc()
    o = rt.SceneOpts()
    rt.lib().rt_scene_opts_default(C.byref(o))
    o.device = rt.RT_DEVICE_NONE
    h = C.c_void_p()
    for n in (1 << 25, 1 << 26):
        d.n_faces = n
        rc = rt.lib().rt_scene_create(C.byref(d), C.byref(o), C.byref(h))
        assert rc != 0 and not h.value, n
        assert "face limit" in rt.lib().rt_last_error().decode()


def test_builder_selected_through_abi(rt, tmp_path):
    """the tree's builder is a scene option (RT_BUILDER_SBVH_GPU default, which a host-only
    scene builds as RT_BUILDER_SBVH; RT_BUILDER_SAH on request), reported in rt_scene_info and kept by the
    scene cache -- no environment variable."""
    o = rt.SceneOpts()
    rt.lib().rt_scene_opts_default(rt.C.byref(o))
    assert o.builder == rt.RT_BUILDER_SBVH_GPU and o.wide_tree == 0
    mesh = _soup(rt, 20_000)
    sb = rt.Scene(mesh, device=rt.RT_DEVICE_NONE)
    sa = rt.Scene(mesh, device=rt.RT_DEVICE_NONE, builder=rt.RT_BUILDER_SAH)
    assert sb.info()["builder"] == rt.RT_BUILDER_SBVH and sa.info()["builder"] == rt.RT_BUILDER_SAH
    assert sb.validate_bvh()["ok"] and sa.validate_bvh()["ok"]
    # the spatial-split tree references clipped faces from several leaves; the SAH tree each face once
    assert sa.validate_bvh()["covered2"] == 20_000 <= sb.validate_bvh()["covered2"]
    for sc, b in ((sb, rt.RT_BUILDER_SBVH), (sa, rt.RT_BUILDER_SAH)):
        p = tmp_path / f"b{b}.rtscene"
        sc.save(p)
        assert rt.Scene.load(p, device=rt.RT_DEVICE_NONE).info()["builder"] == b


def test_sbvh_build_is_deterministic(rt, tmp_path):
    """the spatial-split builder's reference budget is shared out per subtree, so the tree does
    not depend on the order its parallel subtree tasks run in: two builds save byte-identical caches."""
    mesh = _soup(rt, 200_000)
    paths = []
    for k in range(2):
        sc = rt.Scene(mesh, device=rt.RT_DEVICE_NONE)
        assert sc.info()["builder"] == rt.RT_BUILDER_SBVH
        p = tmp_path / f"s{k}.rtscene"
        sc.save(p)
        paths.append(p)
    assert paths[0].read_bytes() == paths[1].read_bytes()


def test_graft_entry_library_check(rt):
    # build()'s final step (the driver's "does it build" check): the library's API version against the header
    import importlib.util
    spec = importlib.util.spec_from_file_location("graft_entry", os.path.join(ROOT, "__graft_entry__.py"))
    g = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(g)
    g.check_library()
