"""Full-frame parity of the benchmark configurations.

Every pixel of the C2 (bunny PRIMARY), C3 (1M-triangle soup PRIMARY) and C5 (bunny FULL) frames at
1920x1080 is rendered by the gfx950 kernels and by the CPU oracle (oracle/rt_oracle.c, the restatement
of the reference's traceRay loop, src/flyscene.cpp:299-371), here, on the box's cores. Bar (BASELINE
north_star): face index and t bit-exact on every pixel, colour L_inf < 1e-4 per channel.

The oracle's own outputs are also held to the committed full-frame digests (tests/golden/
fullframe_digests.json, tools/gen_fullframe_digests.py, generated in the build container), which ties
the oracle build on the box to the one that made the fixtures. C4 (the soup at 3840x2160 split over 8
tile shards) is checked against its committed digests (8.3 M pixels) plus a live oracle sample.
"""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, PARITY_REPORT, scene_path
from test_oracle_pinning import same_bits

pytestmark = pytest.mark.gpu
TOL = 1e-4
DIG = json.load(open(os.path.join(GOLDEN, "fullframe_digests.json")))
# the box's CPU share for one GPU (OMP_NUM_THREADS there); all cores of this process otherwise
THREADS = max(1, min(len(os.sched_getaffinity(0)), int(os.environ.get("OMP_NUM_THREADS", "16") or 16)))


@pytest.fixture(scope="module", autouse=True)
def need_gpu(rt):
    if rt.device_count() == 0:
        pytest.skip("no GPU")


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.fixture(scope="module")
def scenes(rt, orc):
    """GPU and oracle scenes of the bunny and the C3/C4 soup (built once per module)."""
    bunny = rt.Mesh.load_obj(scene_path("bunny.obj"))
    mesh, v, f = rt.soup_mesh(1_000_000)
    return {
        "bunny": (rt.Scene(bunny), orc.Scene(orc.Mesh.load_obj(scene_path("bunny.obj")))),
        "soup": (rt.Scene(mesh), orc.Scene(orc.Mesh.from_arrays(v, f, np.array([rt.SOUP_MATERIAL], np.float32)))),
        "soup_mesh": mesh,
        "bunny_mesh": bunny,
    }


def frame_errors(rgb, face, t, orgb, oface, ot):
    face = np.asarray(face).reshape(-1)
    oface = np.asarray(oface).reshape(-1)
    tb = same_bits(np.asarray(t, np.float32).reshape(-1), np.asarray(ot, np.float32).reshape(-1))
    a = np.asarray(rgb, np.float64).reshape(-1, 3)
    b = np.asarray(orgb, np.float64).reshape(-1, 3)
    err = np.abs(a - b)
    err = np.where(np.isnan(a) & np.isnan(b), 0.0, err)
    return {"pixels": int(face.size), "face_mismatch": int((face != oface).sum()), "t_mismatch": int((~tb).sum()),
            "linf": float(np.nanmax(err)) if err.size else 0.0,
            "nan_mismatch": int((np.isnan(a) != np.isnan(b)).sum()),
            "rgb_bitwise": bool(np.asarray(rgb, np.float32).tobytes() == np.asarray(orgb, np.float32).reshape(np.shape(rgb)).tobytes())}


def gpu_frame(rt, sc, W, H, mode, max_depth=0, shard=(0, 1)):
    m = rt.RT_MODE_FULL if mode == "full" else rt.RT_MODE_PRIMARY
    rgb, face, t, _ = sc.render(rt.flycam(W, H, 0, 0, 20), rt.DEFAULT_LIGHTS, W, H, mode=m, want_hits=True,
                                max_depth=max_depth, shard=shard)
    return rgb, face, t


@pytest.mark.parametrize("case", ["C2", "C3", "C5"])
def test_full_frame_matches_oracle(rt, orc, scenes, case):
    d = DIG[case]
    W, H, mode = d["W"], d["H"], d["mode"]
    sc, osc = scenes[d["scene"]]
    rgb, face, t = gpu_frame(rt, sc, W, H, mode)
    orgb, oface, ot = osc.render(orc.flycam(W, H, 0, 0, 20), orc.DEFAULT_LIGHTS, W, H, full=(mode == "full"),
                                 threads=THREADS)
    # the oracle on this host reproduces the committed fixture (same build, same bits)
    assert sha(oface) == d["face_sha256"] and sha(ot) == d["t_sha256"] and sha(orgb) == d["rgb_sha256"], case
    e = frame_errors(rgb, face, t, orgb, oface, ot)
    PARITY_REPORT.append(f"{case} {d['scene']} {W}x{H} {mode}: {e['pixels']} pixels, face mismatches "
                         f"{e['face_mismatch']}, t mismatches {e['t_mismatch']}, colour L_inf {e['linf']:.3g}, "
                         f"colour bit-identical {e['rgb_bitwise']} (oracle on {THREADS} threads)")
    assert e["face_mismatch"] == 0 and e["t_mismatch"] == 0 and e["nan_mismatch"] == 0, e
    assert e["linf"] < TOL, e
    assert int((face >= 0).sum()) == d["hits"]


@pytest.mark.parametrize("case", ["C3-full", "bunny-depth3"])
def test_full_frame_matches_committed_digests(rt, scenes, case):
    """Configurations too slow for a live full-frame oracle run on the box (C3 FULL: 7 M rays) or the
    runtime recursion limit (bunny, max_depth 3): face and t of every pixel against the committed oracle
    digests, colour against the committed strided oracle sample (every 257th pixel)."""
    d = DIG[case]
    W, H, mode = d["W"], d["H"], d["mode"]
    sc, _ = scenes[d["scene"]]
    rgb, face, t = gpu_frame(rt, sc, W, H, mode, max_depth=d["max_depth"] or 0)
    smp = np.load(os.path.join(GOLDEN, "fullframe_samples.npz"))
    idx = smp[case + "_idx"]
    e = frame_errors(rgb.reshape(-1, 3)[idx], face.reshape(-1)[idx], t.reshape(-1)[idx], smp[case + "_rgb"],
                     smp[case + "_face"], smp[case + "_t"])
    rgb_same = sha(rgb.reshape(-1, 3)) == d["rgb_sha256"]
    PARITY_REPORT.append(f"{case} {d['scene']} {W}x{H} {mode} depth {d['max_depth'] or 2}: face/t digests of all "
                         f"{W * H} pixels equal the oracle's; sampled colour L_inf {e['linf']:.3g}; "
                         f"colour digest equal {rgb_same}")
    assert sha(face) == d["face_sha256"], "face ids differ from the oracle's full frame"
    assert sha(t) == d["t_sha256"], "t differs from the oracle's full frame"
    assert e["face_mismatch"] == 0 and e["linf"] < TOL, e


def stitch_shards(rt, sc, W, H, n, mode="primary"):
    """Render the frame as n tile shards (the multi-GPU partition, rt_frame_shard_tiles) and stitch."""
    rgb = np.full((H, W, 3), np.nan, np.float32)
    face = np.full((H, W), -7, np.int32)
    t = np.full((H, W), np.nan, np.float32)
    covered = np.zeros((H, W), np.int32)
    for k in range(n):
        prgb, pface, pt = gpu_frame(rt, sc, W, H, mode, shard=(k, n))
        mask = rt.shard_mask(W, H, k, n)
        covered += mask
        rgb[mask], face[mask], t[mask] = prgb[mask], pface[mask], pt[mask]
    assert (covered == 1).all(), "the shards do not partition the frame"
    return rgb, face, t


def test_c4_eight_shards_match_oracle(rt, orc, scenes):
    """C4: the 1M soup at 3840x2160 as 8 tile shards (the 8-GPU partition, one device here): the
    stitched frame equals the single-device frame bit for bit, its face / t digests over all 8.3 M
    pixels equal the oracle's, and a live oracle run on a strided sample matches (L_inf < 1e-4)."""
    d = DIG["C4"]
    W, H = d["W"], d["H"]
    sc, osc = scenes["soup"]
    one = gpu_frame(rt, sc, W, H, "primary")
    eight = stitch_shards(rt, sc, W, H, 8)
    for a, b in zip(one, eight):
        assert np.asarray(a).tobytes() == np.asarray(b).tobytes()
    rgb, face, t = eight
    assert sha(face) == d["face_sha256"] and sha(t) == d["t_sha256"]
    idx = np.arange(13, W * H, 97)
    pix = np.stack([idx % W, idx // W], 1).astype(np.int32)
    orgb, oface, ot = osc.render(orc.flycam(W, H, 0, 0, 20), orc.DEFAULT_LIGHTS, W, H, pixels=pix, threads=THREADS)
    e = frame_errors(rgb.reshape(-1, 3)[idx], face.reshape(-1)[idx], t.reshape(-1)[idx], orgb, oface, ot)
    rgb_same = sha(rgb.reshape(-1, 3)) == d["rgb_sha256"]
    PARITY_REPORT.append(f"C4 soup {W}x{H} primary, 8 shards stitched == 1 device; face/t digests of all {W * H} "
                         f"pixels equal the oracle's; live oracle sample of {len(idx)} pixels: colour L_inf "
                         f"{e['linf']:.3g}; colour digest equal {rgb_same}")
    assert e["face_mismatch"] == 0 and e["t_mismatch"] == 0 and e["linf"] < TOL, e


@pytest.mark.parametrize("scene", ["cornell", "bunny"])
@pytest.mark.parametrize("depth", [0, 1, 2, 3, 5])
@pytest.mark.parametrize("mode", ["primary", "full"])
def test_max_depth_matches_oracle(rt, orc, scenes, scene, depth, mode):
    """Runtime recursion limit (rt_frame.max_depth; the reference's Flyscene::max_depth, flyscene.hpp:142,
    traceRay flyscene.cpp:317-371): every pixel against the oracle's traceRay with the same limit, with
    shadows (FULL) and without (PRIMARY). depth 0 = the mode's own (PRIMARY 1, FULL 2)."""
    if scene == "bunny":
        sc, osc = scenes["bunny"]
        W, H, dz = 480, 270, 20
    else:
        sc = rt.Scene(rt.Mesh.load_obj(scene_path("cornell.obj")))
        osc = orc.Scene(orc.Mesh.load_obj(scene_path("cornell.obj")))
        W, H, dz = 160, 120, 0
    m = rt.RT_MODE_FULL if mode == "full" else rt.RT_MODE_PRIMARY
    rgb, face, t, _ = sc.render(rt.flycam(W, H, 0, 0, dz), rt.DEFAULT_LIGHTS, W, H, mode=m, want_hits=True,
                                max_depth=depth)
    orgb, oface, ot = osc.render(orc.flycam(W, H, 0, 0, dz), orc.DEFAULT_LIGHTS, W, H, full=(mode == "full"),
                                 threads=THREADS, max_depth=depth or None)
    e = frame_errors(rgb, face, t, orgb, oface, ot)
    assert e["face_mismatch"] == 0 and e["t_mismatch"] == 0 and e["nan_mismatch"] == 0 and e["linf"] < TOL, e
    if depth >= 2:  # a deeper limit changes colours somewhere (reflections of reflections)
        assert (face >= 0).any()


def test_generic_depth_kernel_equals_tuned_kernels(rt, scenes):
    """The generic traceRay kernel (variant bit 65536 forces it) renders exactly the tuned kernels'
    frames at their own depths: PRIMARY / 1 (k_primary_fused) and FULL / 2 (k_render_full)."""
    sc, _ = scenes["bunny"]
    W, H = 960, 540
    for mode in ("primary", "full"):
        prev = rt.set_variant(0)
        try:
            a = gpu_frame(rt, sc, W, H, mode)
            rt.set_variant(65536)
            b = gpu_frame(rt, sc, W, H, mode)
        finally:
            rt.set_variant(prev)
        for x, y in zip(a, b):
            assert np.asarray(x).tobytes() == np.asarray(y).tobytes(), mode


def test_max_depth_out_of_range_rejected(rt, scenes):
    sc, _ = scenes["bunny"]
    with pytest.raises(rt.RTError, match="max_depth"):
        sc.render(rt.flycam(64, 48), rt.DEFAULT_LIGHTS, 64, 48, max_depth=17)
    with pytest.raises(rt.RTError, match="max_depth"):
        sc.render(rt.flycam(64, 48), rt.DEFAULT_LIGHTS, 64, 48, max_depth=-1)


@pytest.mark.parametrize("case", ["C2", "C5"])
def test_gpu_lbvh_frames_match_oracle_digests(rt, scenes, case):
    """f2 against the oracle directly: the device-built LBVH scene renders the C2 / C5 frames whose face
    and t digests over every pixel equal the oracle's committed ones (not only the host SAH scene's)."""
    d = DIG[case]
    lb = rt.Scene(scenes["bunny_mesh"], builder=rt.RT_BUILDER_LBVH_GPU)
    assert lb.info()["builder"] == rt.RT_BUILDER_LBVH_GPU
    rgb, face, t = gpu_frame(rt, lb, d["W"], d["H"], d["mode"])
    assert sha(face) == d["face_sha256"] and sha(t) == d["t_sha256"], case


def test_gpu_lbvh_soup_matches_oracle_digests(rt, scenes):
    """f2 on the C3 scene: the LBVH scene's full 1080p frame has the oracle's face / t digests."""
    lb = rt.Scene(scenes["soup_mesh"], builder=rt.RT_BUILDER_LBVH_GPU)
    W, H = 1920, 1080
    rgb, face, t = gpu_frame(rt, lb, W, H, "primary")
    assert sha(face) == DIG["C3"]["face_sha256"] and sha(t) == DIG["C3"]["t_sha256"]


@pytest.mark.parametrize("case,builder", [("C2", "ploc"), ("C3", "ploc"), ("C5", "ploc"), ("C3", "sahgpu"), ("C3", "sbvhgpu"), ("C5", "sbvhgpu")])
def test_gpu_ploc_frames_match_oracle_digests(rt, scenes, case, builder):
    """f2 PLOC and the device binned SAH on the BASELINE configs: the device-built tree's full 1080p frames
    (C2 bunny PRIMARY, C3 soup PRIMARY, C5 bunny FULL) have the oracle's face / t digests."""
    d = DIG[case]
    mesh = scenes["bunny_mesh"] if d["scene"] == "bunny" else scenes["soup_mesh"]
    bid = {"ploc": rt.RT_BUILDER_PLOC_GPU, "sahgpu": rt.RT_BUILDER_SAH_GPU, "sbvhgpu": rt.RT_BUILDER_SBVH_GPU}[builder]
    pl = rt.Scene(mesh, builder=bid)
    assert pl.info()["builder"] == bid
    rgb, face, t = gpu_frame(rt, pl, d["W"], d["H"], d["mode"])
    assert sha(face) == d["face_sha256"] and sha(t) == d["t_sha256"], case


@pytest.mark.parametrize("case,builder", [("C2", "sbvh"), ("C3", "sbvh"), ("C3", "sah"), ("C4", "sbvh")])
def test_wide_tree_frames_match_oracle_digests(rt, scenes, case, builder):
    """The fp32 4-wide tree (rt_scene_opts.wide_tree, traverse_wide_fast for PRIMARY octant packets;
    mixed-octant packets on the binary tree) renders every pixel of C2 / C3 / C4 with the oracle's face
    and t digests, over spatial-split and plain SAH trees; the counting run walks the same tree (node
    visits drop, records are 128 B)."""
    d = DIG[case]
    mesh = scenes["bunny_mesh"] if d["scene"] == "bunny" else scenes["soup_mesh"]
    b = rt.RT_BUILDER_SBVH if builder == "sbvh" else rt.RT_BUILDER_SAH
    w = rt.Scene(mesh, builder=b, wide_tree=1)
    info = w.info()
    assert info["wide_nodes"] > 0 and info["builder"] == b
    rgb, face, t = gpu_frame(rt, w, d["W"], d["H"], d["mode"])
    assert sha(face) == d["face_sha256"] and sha(t) == d["t_sha256"], case
    if case == "C3":
        st = w.render(rt.flycam(d["W"], d["H"], 0, 0, 20), rt.DEFAULT_LIGHTS, d["W"], d["H"], flags=rt.RT_FRAME_STATS)[-1]
        assert st["wave_node_bytes"] > 64 * 0 and st["wave_node_fetches"] > 0
        assert st["wave_node_bytes"] > 64 * st["wave_node_fetches"]  # 128-B wide records dominate


MOVE_POSE = 37  # bench.py / tools/gen_fullframe_digests.py MOVE_POSE


@pytest.mark.parametrize("case", ["C3-moving", "C5-moving"])
@pytest.mark.parametrize("fif", [1, 4])
def test_moving_camera_frames_match_oracle_digests(rt, scenes, case, fif):
    """The reference's moving camera: a scene renders frames 0 .. MOVE_POSE - 1 of the camera
    path one at a time (rtamd.CameraPath: WASD held, flyscene.cpp:116-127), so every frame is dispatched
    longest-first by a cost map an earlier pose recorded (re-sorted, dilated, after every moving frame of the
    L2-resident bunny; every 8th frame of the soup); the frame at pose
    MOVE_POSE then equals the oracle's committed digests of that pose (face ids and t bits of every pixel) -- the
    dispatch order, stale or fresh, never changes a pixel. fif 4: frames of a 4-slot scene rendered synchronously
    (rt_render) share one scene-level map."""
    d = DIG[case]
    W, H, mode = d["W"], d["H"], d["mode"]
    mesh = scenes["soup_mesh" if d["scene"] == "soup" else "bunny_mesh"]
    sc = rt.Scene(mesh, frames_in_flight=fif)
    m = rt.RT_MODE_FULL if mode == "full" else rt.RT_MODE_PRIMARY
    p = rt.CameraPath(W, H)
    for _ in range(MOVE_POSE):
        sc.render(p.next(), rt.DEFAULT_LIGHTS, W, H, mode=m)
    lpt = sc.lpt_stats()
    assert lpt["frames"] == MOVE_POSE and lpt["valid"], lpt
    if d["scene"] == "bunny":  # L2-resident: every moving frame re-sorts from its own (dilated) wave costs
        assert lpt["sorts"] == MOVE_POSE, lpt
    else:  # large scene: the 8-frame refresh (the first frame, then every 8th)
        assert lpt["sorts"] == (MOVE_POSE + 7) // 8, lpt
    rgb, face, t, _ = sc.render(p.camera(), rt.DEFAULT_LIGHTS, W, H, mode=m, want_hits=True)
    assert sha(face) == d["face_sha256"] and sha(t) == d["t_sha256"], case
    assert int((np.asarray(face) >= 0).sum()) == d["hits"]
    smp = np.load(os.path.join(GOLDEN, "fullframe_samples.npz"))
    idx = smp[case + "_idx"]
    err = np.abs(np.asarray(rgb, np.float64).reshape(-1, 3)[idx] - smp[case + "_rgb"].astype(np.float64))
    assert float(np.nanmax(err)) < TOL
    PARITY_REPORT.append(f"{case} (pose {MOVE_POSE} of the moving camera, {fif} slot(s), {lpt['sorts']} re-sorts): "
                         f"face/t digests of all {W * H} pixels equal the oracle's")
