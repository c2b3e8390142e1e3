"""In-process multi-device rendering.

The reference renders a frame in one process (Flyscene::raytraceScene's thread loop,
src/flyscene.cpp:266-289). The drop-in's equivalent is a multi-device scene (rt_scene_opts.n_devices /
devices): the scene built once, replicated to every listed device by peer copy, the frame's 64x64
super-tiles interleaved over the devices, every device's tiles assembled in the caller's buffers. On the
one-GPU test box the device list repeats device 0 ({0, 0}, {0, 0, 0}): each replica still has its own copy
of the device data, its own streams and its own frame buffers, and the assembly runs the same code.

Bar: the assembled frame equals the one-device frame bit for bit, and its face / t digests equal the
oracle's committed full-frame digests (tests/golden/fullframe_digests.json).
"""
import ctypes as C
import hashlib
import json
import os
import tempfile

import numpy as np
import pytest

from conftest import GOLDEN, PARITY_REPORT, scene_path

pytestmark = pytest.mark.gpu
DIG = json.load(open(os.path.join(GOLDEN, "fullframe_digests.json")))


@pytest.fixture(scope="module", autouse=True)
def need_gpu(rt):
    if rt.device_count() == 0:
        pytest.skip("no GPU")


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.fixture(scope="module")
def soup(rt):
    mesh, _, _ = rt.soup_mesh(1_000_000)
    return {"mesh": mesh, "one": rt.Scene(mesh), "two": rt.Scene(mesh, devices=[0, 0])}


@pytest.fixture(scope="module")
def bunny(rt):
    mesh = rt.Mesh.load_obj(scene_path("bunny.obj"))
    return {"mesh": mesh, "one": rt.Scene(mesh), "three": rt.Scene(mesh, devices=[0, 0, 0])}


def frame(rt, sc, W, H, mode, shard=(0, 1), max_depth=0):
    m = rt.RT_MODE_FULL if mode == "full" else rt.RT_MODE_PRIMARY
    rgb, face, t, st = sc.render(rt.flycam(W, H, 0, 0, 20), rt.DEFAULT_LIGHTS, W, H, mode=m, want_hits=True,
                                 shard=shard, max_depth=max_depth)
    return rgb, face, t, st


def test_scene_info_lists_devices(rt, soup):
    one, two = soup["one"].info(), soup["two"].info()
    assert one["n_devices"] == 1 and two["n_devices"] == 2
    assert two["device"] == 0
    # each device holds its own copy of the scene's device data
    assert two["device_bytes"] == 2 * one["device_bytes"]
    assert two["replicate_ms"] > 0


def test_c4_two_devices_equal_one_device_and_oracle(rt, soup):
    """C4 (1M soup, 3840x2160 PRIMARY) on devices {0, 0}: rgb / face / t bit-identical to the one-device
    frame; face / t digests of all 8.3 M pixels equal the oracle's."""
    d = DIG["C4"]
    W, H = d["W"], d["H"]
    one = frame(rt, soup["one"], W, H, "primary")
    two = frame(rt, soup["two"], W, H, "primary")
    for a, b in zip(one[:3], two[:3]):
        assert np.asarray(a).tobytes() == np.asarray(b).tobytes()
    assert sha(two[1]) == d["face_sha256"] and sha(two[2]) == d["t_sha256"]
    st = two[3]
    assert st["primary_rays"] == W * H  # summed over the devices
    PARITY_REPORT.append(f"C4 soup {W}x{H} primary on devices {{0,0}} (one process): assembled frame == 1 device "
                         f"bit for bit; face/t digests of all {W * H} pixels equal the oracle's")


def test_c5_three_devices_equal_one_device_and_oracle(rt, bunny):
    """C5 (bunny FULL, 1920x1080) on devices {0, 0, 0}: bit-identical to one device, digests = oracle's."""
    d = DIG["C5"]
    W, H = d["W"], d["H"]
    one = frame(rt, bunny["one"], W, H, "full")
    three = frame(rt, bunny["three"], W, H, "full")
    for a, b in zip(one[:3], three[:3]):
        assert np.asarray(a).tobytes() == np.asarray(b).tobytes()
    assert sha(three[1]) == d["face_sha256"] and sha(three[2]) == d["t_sha256"]
    # (colour: equal to the one-device frame above; against the oracle within one float ulp of powf,
    # test_gpu_fullframe.py)


@pytest.mark.parametrize("case", ["C4", "C5"])
def test_distinct_devices_equal_one_device_and_oracle(rt, soup, bunny, case):
    """The same frames on DISTINCT GPUs (devices 0..n-1 of the node: peer access, hipMemcpyPeerAsync over xGMI,
    one enqueue worker per GPU, assembly across devices). Skipped on a one-GPU box: there the
    in-process multi-device path is verified only with replicas sharing device 0 (the tests above)."""
    n = rt.device_count()
    if n < 2:
        pytest.skip(f"{n} GPU visible: distinct-device replication needs 2 or more")
    d = DIG[case]
    W, H = d["W"], d["H"]
    mode = "primary" if case == "C4" else "full"
    src = soup if case == "C4" else bunny
    devs = list(range(min(n, rt.RT_MAX_DEVICES)))
    sc = rt.Scene(src["mesh"], devices=devs)
    assert sc.info()["n_devices"] == len(devs)
    one = frame(rt, src["one"], W, H, mode)
    many = frame(rt, sc, W, H, mode)
    for a, b in zip(one[:3], many[:3]):
        assert np.asarray(a).tobytes() == np.asarray(b).tobytes()
    assert sha(many[1]) == d["face_sha256"] and sha(many[2]) == d["t_sha256"]
    img8 = []
    for s in (src["one"], sc):
        s.render(rt.flycam(W, H, 0, 0, 20), rt.DEFAULT_LIGHTS, W, H,
                 mode=rt.RT_MODE_FULL if mode == "full" else rt.RT_MODE_PRIMARY)
        img8.append(s.download_rgb8(W, H)[0])
    assert img8[0].tobytes() == img8[1].tobytes()
    PARITY_REPORT.append(f"{case} on distinct devices {devs}: assembled frame == 1 device bit for bit; digests = oracle's")


def test_per_device_stats_cover_the_frame(rt, soup):
    """rt_synchronize_devices: one entry per device, their rays add up to the frame, the totals' kernel time
    is the slowest device's."""
    W, H = 1920, 1080
    sc = soup["two"]
    cam = rt.flycam(W, H, 0, 0, 20)
    for _ in range(3):
        sc.render_async(cam, rt.DEFAULT_LIGHTS, W, H)
    tot, per = sc.synchronize_devices()
    assert len(per) == 2
    assert sum(p["primary_rays"] for p in per) == tot["primary_rays"] == W * H
    assert all(p["primary_rays"] > 0.4 * W * H for p in per)  # interleaved super-tiles: a near-even split
    assert tot["kernel_ms"] == max(p["kernel_ms"] for p in per) > 0
    assert all(p["launches"] == 3 for p in per)


def test_caller_shard_on_multi_device_scene(rt, soup):
    """A caller's own shard (multi-process x multi-device): shard 1 of 3 on devices {0, 0} writes exactly
    that shard's tiles, equal to the one-device shard, and leaves every other pixel of the buffer alone."""
    W, H = 1920, 1080
    cam = rt.flycam(W, H, 0, 0, 20)
    L = rt.Scene._lights(rt.DEFAULT_LIGHTS)
    fr = rt.Frame(W, H, rt.RT_MODE_PRIMARY, 1, 3, 0, 0)
    bufs = []
    for sc in (soup["one"], soup["two"]):
        out = np.full((H, W, 3), -7.0, np.float32)
        st = rt.Stats()
        rt.check(rt.lib().rt_render(sc.h, C.byref(cam), C.cast(L, C.c_void_p), 1, C.byref(fr),
                                    out.ctypes.data_as(C.c_void_p), C.byref(st)))
        bufs.append(out)
    mask = rt.shard_mask(W, H, 1, 3)
    assert bufs[0].tobytes() == bufs[1].tobytes()
    assert (bufs[1][~mask] == -7.0).all() and not (bufs[1][mask] == -7.0).any()


def test_rgb8_download_matches_one_device(rt, bunny):
    """f3 output path on a multi-device scene: the 8-bit frame assembled from the devices' packed tiles equals the
    one-device frame's, with the exactness flag."""
    W, H = 1920, 1080
    cam = rt.flycam(W, H, 0, 0, 20)
    out = []
    for sc in (bunny["one"], bunny["three"]):
        sc.render(cam, rt.DEFAULT_LIGHTS, W, H, mode=rt.RT_MODE_FULL)
        out.append(sc.download_rgb8(W, H))
    assert out[0][0].tobytes() == out[1][0].tobytes()
    assert out[0][1] is True and out[1][1] is True


@pytest.fixture
def device_assembly(rt):
    """The multi-device frame assembled on device 0 (RT_ASM_DEVICE, an A/B knob) instead of on the host."""
    rt.lib().rt_debug_env_knobs(1)
    os.environ["RT_ASM_DEVICE"] = "1"
    try:
        yield
    finally:
        os.environ.pop("RT_ASM_DEVICE", None)
        rt.lib().rt_debug_env_knobs(1 if os.environ.get("RTAMD_DEBUG_KNOBS") == "1" else 0)


@pytest.mark.parametrize("case", ["C4", "C5"])
def test_device_side_assembly_matches_one_device(rt, soup, bunny, device_assembly, case):
    """The device-side assembly of a multi-device scene (peer copies of every replica's packed
    tiles to device 0, one unpack kernel, one chunked copy to the host) gives the one-device frame bit for bit --
    float rgb, face, t and the 8-bit frame with its flag -- like the host-side assembly the other tests run."""
    d = DIG[case]
    W, H = d["W"], d["H"]
    mode = "primary" if case == "C4" else "full"
    src = soup if case == "C4" else bunny
    multi = src["two"] if case == "C4" else src["three"]
    one = frame(rt, src["one"], W, H, mode)
    m = rt.RT_MODE_FULL if mode == "full" else rt.RT_MODE_PRIMARY
    src["one"].render(rt.flycam(W, H, 0, 0, 20), rt.DEFAULT_LIGHTS, W, H, mode=m)
    ref8 = src["one"].download_rgb8(W, H)
    got = frame(rt, multi, W, H, mode)  # device-side path (the fixture's knob)
    got8 = multi.download_rgb8(W, H)
    for a, b in zip(one[:3], got[:3]):
        assert np.asarray(a).tobytes() == np.asarray(b).tobytes()
    assert ref8[0].tobytes() == got8[0].tobytes() and ref8[1] == got8[1]


def test_rgb8_exact_flag_on_nan_colours(rt):
    """The exactness flag survives the assembly: a non-integer specular exponent makes pow() of the reference's
    negative R.E base NaN, which survives its max / clamp and which the 8-bit frame
    cannot hold (flag 0), on one device and on two; the bytes still agree."""
    v = np.array([[-1, -1, 0], [1, -1, 0], [0, 1, 0], [-1, -1, -0.5], [1, -1, -0.5], [0, 1, -0.5]], np.float32)
    f = np.array([[0, 1, 2], [3, 4, 5]], np.uint32)
    mat = np.array([[0.1, 0.1, 0.1, 0.7, 0.7, 0.7, 0.5, 0.5, 0.5, 2.5, 1, 1]], np.float32)
    mesh = rt.Mesh.from_arrays(v, f, mat)
    W, H = 64, 64
    cam = rt.flycam(W, H)
    res = []
    for devs in (None, [0, 0]):
        sc = rt.Scene(mesh, devices=devs)
        rgb, _ = sc.render(cam, rt.DEFAULT_LIGHTS, W, H)
        assert np.isnan(rgb).any()
        res.append(sc.download_rgb8(W, H))
    assert res[0][1] is False and res[1][1] is False
    assert res[0][0].tobytes() == res[1][0].tobytes()
    # and a frame without NaN reports exact on both
    cube = rt.Mesh.load_obj(scene_path("cube.obj"))
    for devs in (None, [0, 0]):
        sc = rt.Scene(cube, devices=devs)
        sc.render(cam, rt.DEFAULT_LIGHTS, W, H)
        assert sc.download_rgb8(W, H)[1] is True


def test_box_colour_frames_on_multi_device_scene(rt, bunny):
    """RT_MODE_BOX_COLORS: caller-set colours reach every replica."""
    W, H = 640, 360
    cam = rt.flycam(W, H, 0, 0, 20)
    nb = bunny["one"].info()["n_ref_boxes"]
    cols = np.random.default_rng(5).random((nb, 3), dtype=np.float32)
    out = []
    for sc in (bunny["one"], bunny["three"]):
        sc.set_box_colors(cols)
        rgb, _ = sc.render(cam, rt.DEFAULT_LIGHTS, W, H, mode=rt.RT_MODE_BOX_COLORS)
        out.append(rgb)
        sc.set_box_colors(None)
    assert out[0].tobytes() == out[1].tobytes()


def test_default_box_colours_on_fresh_multi_device_scene(rt, bunny):
    """RT_MODE_BOX_COLORS on a fresh {0, 0, 0} scene whose colours were never set (the reference's default
    setRandomColor path): the colours are drawn once on the caller's thread before any replica's
    worker runs; the frame equals a fresh one-device scene's bit for bit, twice in a row."""
    W, H = 640, 360
    cam = rt.flycam(W, H, 0, 0, 20)
    out = []
    for devs in (None, [0, 0, 0]):
        sc = rt.Scene(bunny["mesh"], devices=devs)
        a, _ = sc.render(cam, rt.DEFAULT_LIGHTS, W, H, mode=rt.RT_MODE_BOX_COLORS)
        b, _ = sc.render(cam, rt.DEFAULT_LIGHTS, W, H, mode=rt.RT_MODE_BOX_COLORS)
        assert a.tobytes() == b.tobytes()
        out.append(a)
        del sc
    assert out[0].tobytes() == out[1].tobytes()
    assert np.asarray(out[0]).any()


def test_scene_cache_load_on_multi_device(rt, bunny):
    """rt_scene_load with a device list: the loaded scene is replicated like a built one, same bits."""
    W, H = 640, 360
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "bunny.rtscene")
        bunny["one"].save(p)
        sc = rt.Scene.load(p, devices=[0, 0])
    assert sc.info()["n_devices"] == 2
    a = frame(rt, bunny["one"], W, H, "full")
    b = frame(rt, sc, W, H, "full")
    for x, y in zip(a[:3], b[:3]):
        assert np.asarray(x).tobytes() == np.asarray(y).tobytes()


def test_frames_in_flight_on_multi_device_scene(rt, soup):
    """rt_render_async frames overlap on every device; the last frame downloads whole and equal."""
    W, H = 1920, 1080
    cam = rt.flycam(W, H, 0, 0, 20)
    ref = frame(rt, soup["one"], W, H, "primary")[0]
    sc = soup["two"]
    for _ in range(6):
        sc.render_async(cam, rt.DEFAULT_LIGHTS, W, H)
    sc.synchronize()
    assert sc.download(W, H).tobytes() == ref.tobytes()


def test_device_list_validation(rt):
    mesh = rt.Mesh.load_obj(scene_path("cube.obj"))
    n = rt.device_count()
    with pytest.raises(rt.RTError):
        rt.Scene(mesh, devices=[0, n])  # not visible
    o = rt.scene_opts()
    o.n_devices = rt.RT_MAX_DEVICES + 1
    h = C.c_void_p()
    d = mesh.desc()
    assert rt.lib().rt_scene_create(C.byref(d), C.byref(o), C.byref(h)) == -1  # RT_ERR_INVALID
    sc = rt.Scene(mesh, devices=rt.RT_DEVICES_ALL)
    assert sc.info()["n_devices"] == min(n, rt.RT_MAX_DEVICES)
    # ray-list queries run on the first device of a multi-device scene
    two = rt.Scene(mesh, devices=[0, 0])
    o3 = np.array([[0.0, 0.0, 2.0]], np.float32)
    d3 = np.array([[0.0, 0.0, -1.0]], np.float32)
    assert rt.Scene(mesh).trace_closest(o3, d3)[0][0] == two.trace_closest(o3, d3)[0][0] >= 0


def test_pack_shard_refused_on_multi_device_scene(rt, bunny):
    import torch
    W, H = 256, 256
    sc = bunny["three"]
    sc.render(rt.flycam(W, H), rt.DEFAULT_LIGHTS, W, H)
    buf = torch.empty(rt.shard_bytes(W, H, 1), dtype=torch.uint8, device="cuda")
    with pytest.raises(rt.RTError):
        sc.pack_shard_rgb8(buf.data_ptr())
