"""GPU parity tests (MI355X): the gfx950 path through the C ABI against the pinned CPU oracle.

Bar (BASELINE.json north_star): per-pixel hit records (face index, t) bit-exact; colours within
L_inf < 1e-4 per channel (the only non-bit-exact op is powf, evaluated in fp64 on the device).
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN, ROOT, scene_path
from test_oracle_pinning import read_kat, same_bits

pytestmark = pytest.mark.gpu
TOL = 1e-4


@pytest.fixture(scope="module", autouse=True)
def need_gpu(rt):
    if rt.device_count() == 0:
        pytest.skip("no GPU")


def compare(rgb, face, t, orgb, oface, ot, what):
    face = np.asarray(face).reshape(-1)
    oface = np.asarray(oface).reshape(-1)
    nbad_face = int((face != oface).sum())
    tb = same_bits(np.asarray(t).reshape(-1), np.asarray(ot).reshape(-1))
    err = np.abs(np.asarray(rgb, np.float64).reshape(-1, 3) - np.asarray(orgb, np.float64).reshape(-1, 3))
    err = np.where(np.isnan(err) & np.isnan(np.asarray(rgb).reshape(-1, 3)) & np.isnan(np.asarray(orgb).reshape(-1, 3)), 0, err)
    linf = float(np.nanmax(err)) if err.size else 0.0
    assert nbad_face == 0, f"{what}: {nbad_face} pixels hit a different face"
    assert tb.all(), f"{what}: {int((~tb).sum())} pixels differ in t bits"
    assert linf < TOL, f"{what}: colour L_inf {linf:.3g} >= {TOL}"
    return linf


@pytest.mark.parametrize("sec", read_kat(), ids=lambda s: f"op{s[0]}")
def test_device_math_matches_eigen(rt, sec):
    op, n, il, ol, inp, exp = sec
    if op == 16:
        pytest.skip("screenToWorld's tan() runs on the host in the product; device libm tan is not pinned")
    got = rt.debug_math(op, inp, n, ol, device=True)
    bad = (~same_bits(got, exp)).reshape(n, ol).any(1)
    assert bad.sum() == 0, f"op {op}: {bad.sum()} of {n} cases differ on the device"


def test_device_pow_matches_host(rt):
    """op 17 in a gfx950 kernel: the integer-exponent path is bit-identical to the host's; other exponents
    go to the device libm pow (fp64), within 1 ulp of the host C library's."""
    from test_host import pairs, pow_cases, ulp_diff
    xs, ints, frac = pow_cases()
    for ys, exact in ((ints, True), (frac, False)):
        inp = pairs(xs, ys)
        dev = rt.debug_math(17, inp.reshape(-1), len(inp), 1, device=True).reshape(-1)
        host = rt.debug_math(17, inp.reshape(-1), len(inp), 1, device=False).reshape(-1)
        if exact:
            assert same_bits(dev, host).all(), f"{int((~same_bits(dev, host)).sum())} cases differ"
        else:
            assert ulp_diff(dev, host).max() <= 1


def golden_keys():
    g = np.load(os.path.join(GOLDEN, "images.npz"))
    return sorted({k.rsplit("_", 1)[0] for k in g.files})


@pytest.mark.parametrize("key", golden_keys())
def test_golden_images(rt, key):
    g = np.load(os.path.join(GOLDEN, "images.npz"))
    scene_name, mode, W, H = key.split("__")
    W, H = int(W), int(H)
    sc = rt.Scene(rt.Mesh.load_obj(scene_path(scene_name + ".obj")))
    m = rt.RT_MODE_FULL if mode == "full" else rt.RT_MODE_PRIMARY
    rgb, face, t, st = sc.render(rt.flycam(W, H), rt.DEFAULT_LIGHTS, W, H, mode=m, want_hits=True)
    compare(rgb, face, t, g[key + "_rgb"], g[key + "_face"], g[key + "_t"], key)


def sample_pixels(W, H, step_x, step_y, off=0):
    return np.array([(i, j) for j in range(off % step_y, H, step_y) for i in range(off % step_x, W, step_x)], np.int32)


@pytest.mark.parametrize("mode", ["primary", "full"])
def test_bunny_1080p(rt, orc, mode):
    """C2 / C5: bunny, 1920x1080, eye (0,0,1) = Flycamera translate(0,0,20); oracle on a pixel sample."""
    W, H = 1920, 1080
    sc = rt.Scene(rt.Mesh.load_obj(scene_path("bunny.obj")))
    m = rt.RT_MODE_FULL if mode == "full" else rt.RT_MODE_PRIMARY
    rgb, face, t, st = sc.render(rt.flycam(W, H, 0, 0, 20), rt.DEFAULT_LIGHTS, W, H, mode=m, want_hits=True)
    osc = orc.Scene(orc.Mesh.load_obj(scene_path("bunny.obj")))
    pix = sample_pixels(W, H, 7, 5, off=3)
    orgb, oface, ot = osc.render(orc.flycam(W, H, 0, 0, 20), orc.DEFAULT_LIGHTS, W, H, full=(mode == "full"),
                                 pixels=pix, threads=16)
    i, j = pix[:, 0], pix[:, 1]
    compare(rgb[j, i], face[j, i], t[j, i], orgb, oface, ot, f"bunny-{mode}")
    assert 0.2 < (face >= 0).mean() < 0.5


@pytest.fixture(scope="module")
def soup(rt, orc):
    mesh, v, f = rt.soup_mesh(1_000_000)
    # the host SBVH tree (also the quantised 4-wide tree of the W4 variant); device builders are compared with it
    sc = rt.Scene(mesh, builder=rt.RT_BUILDER_SBVH)
    osc = orc.Scene(orc.Mesh.from_arrays(v, f, np.array([rt.SOUP_MATERIAL], np.float32)))
    return sc, osc


def test_soup_1m_1080p_primary(rt, orc, soup):
    """C3: 1M random triangles, 1920x1080 primary, eye (0,0,1): full GPU frame, oracle on a sample."""
    sc, osc = soup
    W, H = 1920, 1080
    rgb, face, t, st = sc.render(rt.flycam(W, H, 0, 0, 20), rt.DEFAULT_LIGHTS, W, H, want_hits=True)
    pix = sample_pixels(W, H, 41, 37, off=5)
    orgb, oface, ot = osc.render(orc.flycam(W, H, 0, 0, 20), orc.DEFAULT_LIGHTS, W, H, pixels=pix, threads=16)
    i, j = pix[:, 0], pix[:, 1]
    compare(rgb[j, i], face[j, i], t[j, i], orgb, oface, ot, "soup-1M")
    assert 0.8 < (face >= 0).mean() < 0.98
    # size-independent properties of the whole frame: determinism, range
    rgb2, face2, t2, _ = sc.render(rt.flycam(W, H, 0, 0, 20), rt.DEFAULT_LIGHTS, W, H, want_hits=True)
    assert rgb.tobytes() == rgb2.tobytes() and face.tobytes() == face2.tobytes()
    assert np.nanmin(rgb) >= 0.0 and np.nanmax(rgb) <= 1.0


def test_soup_shards_stitch_bitwise(rt, soup):
    """Tile sharding (multi-GPU partition) on one device: N shards stitched == single render."""
    sc, _ = soup
    W, H = 1920, 1080
    cam = rt.flycam(W, H, 0, 0, 20)
    ref, _ = sc.render(cam, rt.DEFAULT_LIGHTS, W, H)
    for n in (2, 3, 8):
        out = np.full((H, W, 3), np.nan, np.float32)
        for k in range(n):
            part, st = sc.render(cam, rt.DEFAULT_LIGHTS, W, H, shard=(k, n))
            tiles = rt.shard_mask(W, H, k, n)
            assert st["primary_rays"] == int(tiles.sum())
            out[tiles] = part[tiles]
        assert out.tobytes() == ref.tobytes(), n


def test_trace_queries_match_oracle(rt, orc):
    """calculateMinimumFace and shadow() on arbitrary rays (ray-list entry points)."""
    sc = rt.Scene(rt.Mesh.load_obj(scene_path("bunny.obj")))
    osc = orc.Scene(orc.Mesh.load_obj(scene_path("bunny.obj")))
    rng = np.random.default_rng(7)
    n = 4096
    o = rng.uniform(-1.0, 1.0, (n, 3)).astype(np.float32)
    tgt = rng.uniform(-0.3, 0.3, (n, 3)).astype(np.float32)
    d = tgt - o
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    d = d.astype(np.float32)
    face, t, P = sc.trace_closest(o, d)
    oface, ot, oP = osc.closest(o, d)
    assert (face == oface).all() and same_bits(t, ot).all() and same_bits(P[face >= 0], oP[oface >= 0]).all()
    L = rng.normal(size=(n, 3)).astype(np.float32)
    L /= np.linalg.norm(L, axis=1, keepdims=True)
    hitP = P[face >= 0]
    Lh = L[: len(hitP)].astype(np.float32)
    assert (sc.trace_shadow(hitP, Lh) == osc.shadow(hitP, Lh)).all()


@pytest.mark.parametrize("WH", [(37, 11), (1, 1), (9, 17)])
def test_ragged_frame_sizes(rt, orc, WH):
    W, H = WH
    sc = rt.Scene(rt.Mesh.load_obj(scene_path("cube.obj")))
    osc = orc.Scene(orc.Mesh.load_obj(scene_path("cube.obj")))
    for full in (False, True):
        rgb, face, t, _ = sc.render(rt.flycam(W, H), rt.DEFAULT_LIGHTS, W, H,
                                    mode=rt.RT_MODE_FULL if full else rt.RT_MODE_PRIMARY, want_hits=True)
        orgb, oface, ot = osc.render(orc.flycam(W, H), orc.DEFAULT_LIGHTS, W, H, full=full)
        compare(rgb, face, t, orgb, oface, ot, f"cube-{W}x{H}-{full}")


def test_empty_scene_is_background(rt):
    empty = rt.Mesh.from_arrays(np.zeros((0, 3), np.float32), np.zeros((0, 3), np.uint32),
                                np.array([rt.SOUP_MATERIAL], np.float32), groups=[])
    sc = rt.Scene(empty)
    rgb, face, t, _ = sc.render(rt.flycam(64, 48), rt.DEFAULT_LIGHTS, 64, 48, want_hits=True)
    assert (face == -1).all() and np.isinf(t).all()
    np.testing.assert_array_equal(rgb, np.float32(0.9))


def test_multiple_lights(rt, orc):
    lights = [((-0.5, 2.0, 3.0), (0.6, 0.6, 0.6)), ((1.5, 0.5, 1.0), (0.3, 0.5, 0.2)), ((0.0, -2.0, 2.0), (0.2, 0.2, 0.4))]
    W, H = 160, 120
    sc = rt.Scene(rt.Mesh.load_obj(scene_path("cornell.obj")))
    osc = orc.Scene(orc.Mesh.load_obj(scene_path("cornell.obj")))
    for full in (False, True):
        rgb, face, t, _ = sc.render(rt.flycam(W, H), lights, W, H,
                                    mode=rt.RT_MODE_FULL if full else rt.RT_MODE_PRIMARY, want_hits=True)
        orgb, oface, ot = osc.render(orc.flycam(W, H), lights, W, H, full=full, threads=8)
        compare(rgb, face, t, orgb, oface, ot, f"cornell-3lights-{full}")


def test_stats_counting_run(rt, soup):
    sc, _ = soup
    W, H = 1920, 1080
    sc.render_async(rt.flycam(W, H, 0, 0, 20), rt.DEFAULT_LIGHTS, W, H, flags=rt.RT_FRAME_STATS)
    st = sc.synchronize()
    assert st["primary_rays"] == W * H
    assert st["node_visits"] > W * H and st["tri_tests"] > W * H
    assert st["wave_node_fetches"] * 16 < st["node_visits"]  # coherence: one fetch serves many rays


# variant bits the product library serves itself (rt_api.h rt_debug_set_variant)
VARIANTS = {"xcd-order": 4, "xcd-runs-4": 512, "dispatch-order": 1536, "full-8-waves": 8192, "full-small-build": 16384,
            "split-primary": 32768, "generic-depth-kernel": 65536}
# the A/B kernels of the variants library only (rt_variants.hip, `make variants`)
VARIANTS_LIB = {"vgpr-stack": 1, "wide4": 2, "full-pipeline": 16, "pipeline-lane-refl": 48,
                "pipeline-lane-all": 16 | 32 | 64 | 128, "two-rays-per-lane": 256, "persistent": 2048,
                "persistent-no-steal": 2048 | 4096, "dual-chain": 1048576}


def variant_frames_identical(rt, scenes, bits):
    """Render bunny (PRIMARY + FULL, 1080p) and the 1M soup (FULL 640x360, PRIMARY 1000x563) with the default
    kernels and with kernel variant `bits`; returns the cases whose rgb / face / t differ."""
    bunny, soup = scenes
    cases = [(bunny, 1920, 1080, rt.RT_MODE_PRIMARY), (bunny, 1920, 1080, rt.RT_MODE_FULL),
             (soup, 640, 360, rt.RT_MODE_FULL), (soup, 1000, 563, rt.RT_MODE_PRIMARY)]
    bad = []
    for sc, W, H, m in cases:
        cam = rt.flycam(W, H, 0, 0, 20)
        prev = rt.set_variant(0)
        try:
            ref = sc.render(cam, rt.DEFAULT_LIGHTS, W, H, mode=m, want_hits=True)
            rt.set_variant(bits)
            got = sc.render(cam, rt.DEFAULT_LIGHTS, W, H, mode=m, want_hits=True)
        finally:
            rt.set_variant(prev)
        if any(np.asarray(a).tobytes() != np.asarray(b).tobytes() for a, b in zip(ref[:3], got[:3])):
            bad.append((W, H, m))
    return bad


@pytest.mark.parametrize("name", sorted(VARIANTS))
def test_kernel_variants_render_identical_bits(rt, soup, name):
    """Every kernel variant of the product library (tile orders, FULL builds, the two-kernel PRIMARY, the
    generic traceRay kernel) renders exactly the default kernels' frame (rgb, face, t) on bunny (PRIMARY +
    FULL) and the 1M soup (FULL, 640x360 crop of the C3 camera)."""
    bunny = rt.Scene(rt.Mesh.load_obj(scene_path("bunny.obj")))
    assert variant_frames_identical(rt, (bunny, soup[0]), VARIANTS[name]) == []


def test_product_library_refuses_variant_only_kernels(rt, soup):
    """The A/B kernels (VGPR stack, quantised 4-wide tree, FULL pipeline, two rays per lane, persistent
    threads, dual chain) are not in the product library: selecting one fails loudly instead of silently
    rendering with the default kernels."""
    sc, _ = soup
    cam = rt.flycam(64, 64, 0, 0, 20)
    for name, bits in sorted(VARIANTS_LIB.items()):
        prev = rt.set_variant(bits)
        try:
            mode = rt.RT_MODE_FULL if bits & 16 else rt.RT_MODE_PRIMARY
            with pytest.raises(rt.RTError, match="A/B build option"):
                sc.render(cam, rt.DEFAULT_LIGHTS, 64, 64, mode=mode)
        finally:
            rt.set_variant(prev)


def test_variants_library_renders_identical_bits(rt):
    """Every A/B kernel of the variants library (rt_variants.hip) renders the default kernels' frames bit for
    bit: tests/variants_check.py in a child process with RTAMD_LIB = lib/librtamd_variants.so (one library
    per process), the same four frames per variant as above; and the FULL stage pipeline (variant 16) refuses a
    sharded frame with an error (its ray lists are sized for whole frames)."""
    import json
    import subprocess
    import sys
    lib = os.path.join(ROOT, "ray-tracing-project_amd", "lib", "librtamd_variants.so")
    if not os.path.exists(lib):
        pytest.skip("variants library not built (make variants)")
    env = dict(os.environ, RTAMD_LIB=lib)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "variants_check.py")], env=env,
                       capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    res = json.loads(p.stdout.strip().splitlines()[-1])
    assert set(res) == set(VARIANTS_LIB) | {"_pipeline_shard_refused"}, res
    bad = {k: v for k, v in res.items() if v}
    assert not bad, bad


def test_frames_in_flight_are_independent(rt, soup):
    """Frames queued back to back overlap on the scene's frame slots (default 4 in flight, each with its
    own stream and buffers); every frame is still complete and independent: the downloaded last frame
    equals the same camera rendered alone, for 1, 2 and 4 slots, across frame-size changes."""
    _, osc = soup
    mesh = rt.Mesh.load_obj(scene_path("bunny.obj"))
    cams = [(1920, 1080, 0, 0, 20), (640, 360, 0, 0, 15), (1920, 1080, 1, 0, 20), (1280, 720, 0, 1, 18)]
    ref = {}
    solo = rt.Scene(mesh, frames_in_flight=1)
    for c in cams:
        W, H = c[0], c[1]
        ref[c] = solo.render(rt.flycam(*c), rt.DEFAULT_LIGHTS, W, H, mode=rt.RT_MODE_FULL)[0]
    for fif in (1, 2, 4):
        sc = rt.Scene(mesh, frames_in_flight=fif)
        for k in range(9):
            c = cams[k % len(cams)]
            sc.render_async(rt.flycam(*c), rt.DEFAULT_LIGHTS, c[0], c[1], mode=rt.RT_MODE_FULL)
        sc.synchronize()
        c = cams[8 % len(cams)]
        out = np.zeros((c[1], c[0], 3), np.float32)
        rt.lib().rt_frame_download(sc.h, out.shape[0] * out.shape[1], out.ctypes.data, None, None)
        assert out.tobytes() == ref[c].tobytes(), fif


def test_scene_cache_renders_identical_bits(rt, tmp_path):
    """A scene restored from the binary cache renders the original's frame bit for bit (PRIMARY + FULL)."""
    orig = rt.Scene(rt.Mesh.load_obj(scene_path("bunny.obj")))
    p = tmp_path / "bunny.rtscene"
    orig.save(p)
    ld = rt.Scene.load(p)
    W, H = 960, 540
    cam = rt.flycam(W, H, 0, 0, 20)
    for m in (rt.RT_MODE_PRIMARY, rt.RT_MODE_FULL):
        a = orig.render(cam, rt.DEFAULT_LIGHTS, W, H, mode=m, want_hits=True)
        b = ld.render(cam, rt.DEFAULT_LIGHTS, W, H, mode=m, want_hits=True)
        for x, y in zip(a[:3], b[:3]):
            assert np.asarray(x).tobytes() == np.asarray(y).tobytes()


def test_rgb8_output_path(rt, tmp_path):
    """f3: the device-side 8-bit conversion equals writePPMImage's numbers from the float frame, the PPM
    written from it is byte-identical, and out-of-range colours are flagged (exact = False)."""
    sc = rt.Scene(rt.Mesh.load_obj(scene_path("bunny.obj")))
    W, H = 1920, 1080
    cam = rt.flycam(W, H, 0, 0, 20)
    rgb, _ = sc.render(cam, rt.DEFAULT_LIGHTS, W, H, mode=rt.RT_MODE_FULL)
    v8, exact = sc.download_rgb8(W, H)
    assert exact
    ref = np.minimum(255, (np.float32(255) * rgb).astype(np.int64))
    np.testing.assert_array_equal(v8, ref.astype(np.uint8))
    a, b = tmp_path / "f.ppm", tmp_path / "b.ppm"
    rt.write_ppm(a, rgb)
    rt.write_ppm_rgb8(b, v8)
    assert a.read_bytes() == b.read_bytes()
    neg = rt.Scene(rt.Mesh.load_obj(scene_path("cube.obj")), background=(-0.5, 0.9, 2.0))
    neg.render(rt.flycam(64, 48), rt.DEFAULT_LIGHTS, 64, 48)
    v8, exact = neg.download_rgb8(64, 48)
    assert not exact and v8[0, 0].tolist() == [0, 229, 255]


def test_shard_pack_gather_unpack(rt, soup):
    """f3 multi-GPU assembly on one device: every shard's packed 8-bit tiles, concatenated as an RCCL
    gather would, unpack to the single-device frame's 8-bit values."""
    import torch
    sc, _ = soup
    W, H = 1000, 600  # ragged: partial tiles at the right and bottom edges
    cam = rt.flycam(W, H, 0, 0, 20)
    sc.render(cam, rt.DEFAULT_LIGHTS, W, H)
    ref, exact = sc.download_rgb8(W, H)
    assert exact
    for n in (1, 2, 3, 8):
        slice_b = rt.shard_bytes(W, H, n)
        packed = torch.zeros(n * slice_b, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()  # torch's fill must land before the library's own streams write
        for k in range(n):
            sc.render(cam, rt.DEFAULT_LIGHTS, W, H, shard=(k, n))
            sc.pack_shard_rgb8(packed.data_ptr() + k * slice_b)
        frame = torch.zeros(H * W * 3, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        rt.unpack_shards_rgb8(packed.data_ptr(), n, W, H, frame.data_ptr(), torch.cuda.current_device())
        np.testing.assert_array_equal(frame.cpu().numpy().reshape(H, W, 3), ref)


def test_spherical_and_directional_lights(rt, orc):
    """f4: a spherical light (jittered point lights from the reference's rand() sequence) plus a
    directional light (the reference's stored screen-centre vector), FULL and PRIMARY, against the oracle."""
    W, H = 480, 270
    cam = rt.flycam(W, H, 0, 0, 20)
    sph = rt.spherical_light((-0.5, 2.0, 3.0), (1.0, 1.0, 1.0), 0.4, 5, rng=rt.Rand(1))
    dl = rt.directional_light(cam, (0.3, 0.25, 0.2))
    lights = sph + [dl]
    sc = rt.Scene(rt.Mesh.load_obj(scene_path("bunny.obj")))
    osc = orc.Scene(orc.Mesh.load_obj(scene_path("bunny.obj")))
    for full in (False, True):
        rgb, face, t, _ = sc.render(cam, lights, W, H, mode=rt.RT_MODE_FULL if full else rt.RT_MODE_PRIMARY,
                                    want_hits=True)
        orgb, oface, ot = osc.render(orc.flycam(W, H, 0, 0, 20), sph, W, H, full=full, threads=16,
                                     dir_lights=[(dl[0], dl[1])])
        compare(rgb, face, t, orgb, oface, ot, f"bunny-lights-{full}")


@pytest.mark.parametrize("name", ["bunny", "soup"])
def test_gpu_lbvh_builder(rt, soup, name):
    """f2: the device LBVH build gives a sound tree (host containment / coverage check) and the frame of
    the host-SAH scene bit for bit (PRIMARY and FULL)."""
    if name == "bunny":
        mesh = rt.Mesh.load_obj(scene_path("bunny.obj"))
        ref = rt.Scene(mesh)
        W, H = 1920, 1080
    else:
        ref, _ = soup
        mesh = ref.mesh
        W, H = 960, 540
    lb = rt.Scene(mesh, builder=rt.RT_BUILDER_LBVH_GPU)
    info = lb.info()
    assert info["builder"] == rt.RT_BUILDER_LBVH_GPU and info["bvh_gpu_ms"] > 0
    v = lb.validate_bvh()
    assert v["ok"] and v["covered2"] == info["n_faces"], v
    cam = rt.flycam(W, H, 0, 0, 20)
    for m in (rt.RT_MODE_PRIMARY, rt.RT_MODE_FULL):
        a = ref.render(cam, rt.DEFAULT_LIGHTS, W, H, mode=m, want_hits=True)
        b = lb.render(cam, rt.DEFAULT_LIGHTS, W, H, mode=m, want_hits=True)
        for x, y in zip(a[:3], b[:3]):
            assert np.asarray(x).tobytes() == np.asarray(y).tobytes(), (name, m)


@pytest.mark.parametrize("builder", ["ploc", "sahgpu", "sbvhgpu"])
@pytest.mark.parametrize("name", ["bunny", "soup", "cube"])
def test_gpu_ploc_builder(rt, soup, name, builder):
    """f2 "LBVH/PLOC" and the device binned SAH (rt_build.hip) give a sound tree -- every triangle inside every
    ancestor box, every face in exactly one leaf, leaves of at most 4 triangles -- and the frame of the
    host-SBVH scene bit for bit (PRIMARY and FULL); the 12-triangle cube takes the small-task paths only."""
    bid = {"ploc": rt.RT_BUILDER_PLOC_GPU, "sahgpu": rt.RT_BUILDER_SAH_GPU, "sbvhgpu": rt.RT_BUILDER_SBVH_GPU}[builder]
    if name == "cube":
        mesh = rt.Mesh.load_obj(scene_path("cube.obj"))
        ref = rt.Scene(mesh)
        W, H = 320, 240
    elif name == "bunny":
        mesh = rt.Mesh.load_obj(scene_path("bunny.obj"))
        ref = rt.Scene(mesh)
        W, H = 1920, 1080
    else:
        ref, _ = soup
        mesh = ref.mesh
        W, H = 960, 540
    pl = rt.Scene(mesh, builder=bid)
    info = pl.info()
    assert info["builder"] == bid and info["bvh_gpu_ms"] > 0
    assert info["bvh_depth"] <= 62
    v = pl.validate_bvh()
    # spatial splits reference a straddling face from several leaves: the validator's split-aware check (every
    # reference's clipped box inside its ancestors, every face covered) instead of one leaf per face
    if builder == "sbvhgpu":
        assert v["ok"] and v["covered2"] >= info["n_faces"], v
    else:
        assert v["ok"] and v["covered2"] == info["n_faces"], v
    cam = rt.flycam(W, H, 0, 0, 20)
    for m in (rt.RT_MODE_PRIMARY, rt.RT_MODE_FULL):
        a = ref.render(cam, rt.DEFAULT_LIGHTS, W, H, mode=m, want_hits=True)
        b = pl.render(cam, rt.DEFAULT_LIGHTS, W, H, mode=m, want_hits=True)
        for x, y in zip(a[:3], b[:3]):
            assert np.asarray(x).tobytes() == np.asarray(y).tobytes(), (name, m)


def test_trace_color_and_debug_ray(rt, orc):
    """f4 single-ray queries: traceRay colours of camera rays equal the FULL frame's pixels bit for bit;
    the debug ray's first segment is that pixel's ray, colour and hit distance, and each reflection
    segment starts 0.001 along its direction from the previous hit."""
    W, H = 480, 270
    sc = rt.Scene(rt.Mesh.load_obj(scene_path("bunny.obj")))
    cam = rt.flycam(W, H, 0, 0, 20)
    rgb, face, t, _ = sc.render(cam, rt.DEFAULT_LIGHTS, W, H, mode=rt.RT_MODE_FULL, want_hits=True)
    ocam = orc.flycam(W, H, 0, 0, 20)
    pix = [(i, j) for j in range(3, H, 17) for i in range(5, W, 23)]
    od = [orc.camera_ray(ocam, i, j) for i, j in pix]
    o = np.array([a for a, _ in od], np.float32)
    d = np.array([b for _, b in od], np.float32)
    c, f, tt = sc.trace_color(o, d, rt.DEFAULT_LIGHTS)
    ii = np.array([p[0] for p in pix]); jj = np.array([p[1] for p in pix])
    assert c.tobytes() == rgb[jj, ii].tobytes()
    assert (f == face[jj, ii]).all() and tt.tobytes() == t[jj, ii].tobytes()
    hits = [(i, j) for i, j in pix if face[j, i] >= 0][:20]
    assert hits
    for i, j in hits:
        segs = sc.debug_ray(cam, rt.DEFAULT_LIGHTS, float(i), float(j), max_depth=3)
        o0, d0 = orc.camera_ray(ocam, i, j)
        assert segs[0][0].tobytes() == np.asarray(o0, np.float32).tobytes()
        assert segs[0][1].tobytes() == np.asarray(d0, np.float32).tobytes()
        assert segs[0][2] == t[j, i] and segs[0][3].tobytes() == rgb[j, i].tobytes()
        for a, b in zip(segs, segs[1:]):
            hitp = a[0] + a[2] * a[1]
            assert np.allclose(b[0], hitp + np.float32(0.001) * b[1], atol=1e-5)
            assert (b[3] == segs[0][3]).all()


def test_counting_frame_among_frames_in_flight(rt, soup):
    """A counting (RT_FRAME_STATS) frame queued between ordinary frames in flight reports the same
    counters as a counting frame rendered alone (the shared counters are not disturbed)."""
    sc, _ = soup
    W, H = 1920, 1080
    cam = rt.flycam(W, H, 0, 0, 20)
    sc.render_async(cam, rt.DEFAULT_LIGHTS, W, H, flags=rt.RT_FRAME_STATS)
    alone = sc.synchronize()
    for k in range(3):
        sc.render_async(cam, rt.DEFAULT_LIGHTS, W, H)
    sc.render_async(cam, rt.DEFAULT_LIGHTS, W, H, flags=rt.RT_FRAME_STATS)
    mixed = sc.synchronize()
    for key in ("node_visits", "tri_tests", "wave_node_fetches", "wave_tri_fetches", "hits", "total_rays"):
        assert mixed[key] == alone[key], key


def test_cli_flyscene_mirror(rt, tmp_path):
    """The Flyscene-shaped host (rt_render_cli: initialize -> translate -> raytraceScene -> result.ppm):
    its PPM (8-bit download path) is byte-identical to writePPMImage of the library's float frame, also
    when the scene comes from the binary cache, the GPU LBVH or the host build, and when several devices render
    the frame in the one process (--devices: replicas sharing the test box's GPU, or every visible GPU)."""
    import subprocess
    cli = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ray-tracing-project_amd", "lib",
                       "rt_render_cli")
    obj = scene_path("bunny.obj")
    W, H = 320, 180
    sc = rt.Scene(rt.Mesh.load_obj(obj))
    rgb, _ = sc.render(rt.flycam(W, H, 0, 0, 20), rt.DEFAULT_LIGHTS, W, H, mode=rt.RT_MODE_FULL)
    ref = tmp_path / "ref.ppm"
    rt.write_ppm(ref, rgb)
    cache = tmp_path / "bunny.rtscene"
    setups = {}
    for extra in ([], ["--cache", str(cache)], ["--cache", str(cache)], ["--lbvh", "--gpu-boxes"], ["--host-build"],
                  ["--devices", "0,0"], ["--devices", "all"], ["--cache", str(cache), "--devices", "0,0,0"]):
        out = tmp_path / "out.ppm"
        log = subprocess.run([cli, obj, str(W), str(H), "--dz", "20", "--out", str(out)] + extra, check=True,
                             capture_output=True, text=True).stdout
        assert out.read_bytes() == ref.read_bytes(), extra
        line = [x for x in log.splitlines() if x.startswith("scene setup:")]
        assert len(line) == 1, log
        setups[" ".join(extra)] = line[0]
    assert cache.exists()
    # the drop-in builds what the benchmarks measure: the library default, the device SBVH
    # and the device box partition; --host-build opts out
    assert "builder sbvh-gpu, boxes gpu" in setups[""], setups[""]
    assert "builder sbvh-host, boxes host" in setups["--host-build"], setups["--host-build"]
    assert "builder lbvh-gpu" in setups["--lbvh --gpu-boxes"]
    print("rt_render_cli:", setups)


def _tie_arrays(n, seed):
    """Faces whose coordinates come from a tiny set incl. -0.0 / +0.0: ties in every min / max, many
    impossible split axes (axis retries) and duplicate faces."""
    rng = np.random.default_rng(seed)
    vals = np.array([-1.0, -0.0, 0.0, 0.25, 1.0], np.float32)
    v = vals[rng.integers(0, len(vals), size=(3 * n, 3))]
    f = np.arange(3 * n, dtype=np.uint32).reshape(-1, 3)
    return v, f


def _box_case(rt, orc, soup, name):
    """(product mesh, oracle mesh, min_faces) of a box-partition case"""
    mat = np.array([rt.SOUP_MATERIAL], np.float32)
    if name in ("soup", "ties", "same"):
        if name == "soup":
            v, f = rt.generate_soup(1_000_000), np.arange(3_000_000, dtype=np.uint32).reshape(-1, 3)
            return soup[0].mesh, orc.Mesh.from_arrays(v, f, mat), 300
        if name == "ties":
            v, f = _tie_arrays(20000, 7)
            mf = 20
        else:  # every face identical: all three axes fail, one box
            v = np.tile(np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0]], np.float32), (400, 1))
            f = np.arange(1200, dtype=np.uint32).reshape(-1, 3)
            mf = 300
        return rt.Mesh.from_arrays(v, f, mat), orc.Mesh.from_arrays(v, f, mat), mf
    scene, mf = name.split(":")
    return rt.Mesh.load_obj(scene_path(scene + ".obj")), orc.Mesh.load_obj(scene_path(scene + ".obj")), int(mf)


@pytest.mark.parametrize("name", ["cube:300", "dodgeColorTest:300", "bunny:300", "bunny:8", "testding:40", "soup",
                                  "ties", "same"])
def test_gpu_box_partition(rt, orc, soup, name):
    """f2: generateBoundingBoxes on the device (BoundingBox.cpp:109-161, flyscene.cpp:399-428) -- the
    oracle's boxes (bounds bit for bit), box order and in-box face order, hence the same tie-break
    ranks; and the host builder's, too."""
    mesh, omesh, mf = _box_case(rt, orc, soup, name)
    host = rt.Scene(mesh, min_faces=mf, box_builder=rt.RT_BOXES_HOST)
    dev = rt.Scene(mesh, min_faces=mf, box_builder=rt.RT_BOXES_GPU)
    ih, idv = host.info(), dev.info()
    assert ih["box_builder"] == rt.RT_BOXES_HOST and idv["box_builder"] == rt.RT_BOXES_GPU
    assert idv["boxes_gpu_ms"] > 0
    hb, db = host.ref_boxes(), dev.ref_boxes()
    ob = orc.Scene(omesh, min_faces=mf).boxes()
    assert idv["n_ref_boxes"] == len(ob[1]), (idv["n_ref_boxes"], len(ob[1]))
    for a, b, o in zip(hb, db, ob):
        assert np.asarray(b).tobytes() == np.asarray(o).tobytes(), (name, "device vs oracle")
        assert np.asarray(a).tobytes() == np.asarray(b).tobytes(), (name, "host vs device")
    if name == "same":
        assert idv["n_ref_boxes"] == 1
    if name in ("bunny:300", "ties"):
        W, H = 480, 270
        cam = rt.flycam(W, H, 0, 0, 20)
        a = host.render(cam, rt.DEFAULT_LIGHTS, W, H, mode=rt.RT_MODE_FULL, want_hits=True)
        b = dev.render(cam, rt.DEFAULT_LIGHTS, W, H, mode=rt.RT_MODE_FULL, want_hits=True)
        for x, y in zip(a[:3], b[:3]):
            assert np.asarray(x).tobytes() == np.asarray(y).tobytes()


def test_gpu_box_partition_nonfinite_uses_host(rt):
    """A referenced vertex with a non-finite coordinate: the device builder declines, the host one runs."""
    v = np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0], [np.nan, 0, 1], [1, 1, 1], [0, 1, 1]], np.float32)
    f = np.arange(6, dtype=np.uint32).reshape(-1, 3)
    mesh = rt.Mesh.from_arrays(v, f, np.array([rt.SOUP_MATERIAL], np.float32))
    try:
        sc = rt.Scene(mesh, box_builder=rt.RT_BOXES_GPU)
    except rt.RTError:
        return  # rejected later in scene creation: nothing built on the device either
    assert sc.info()["box_builder"] == rt.RT_BOXES_HOST


def test_longest_first_dispatch_order(rt):
    """The one-wave render kernels dispatch a slot's next frame of the same shape longest-first
    (k_order_lpt, from the wave costs the previous frame recorded): the dispatch order is a permutation of
    the frame's waves that keeps each wave on its chunked-XCD position class and differs from the
    default order, and every frame renders the same bits as with the default order (variant 131072)."""
    mesh = rt.Mesh.load_obj(scene_path("bunny.obj"))
    sc = rt.Scene(mesh, frames_in_flight=1)
    for W, H, mode, depth in ((1920, 1080, rt.RT_MODE_PRIMARY, 0), (1000, 563, rt.RT_MODE_FULL, 0),
                              (640, 360, rt.RT_MODE_FULL, 3)):
        cam = rt.flycam(W, H, 0, 0, 20)
        prev = rt.set_variant(131072)
        try:
            ref = sc.render(cam, rt.DEFAULT_LIGHTS, W, H, mode=mode, want_hits=True, max_depth=depth)
        finally:
            rt.set_variant(prev)
        orders = []
        for k in range(3):  # frame 0: default order (no costs yet); frames 1, 2: longest-first
            got = sc.render(cam, rt.DEFAULT_LIGHTS, W, H, mode=mode, want_hits=True, max_depth=depth,
                            flags=rt.RT_FRAME_TIMELINE)
            for a, b in zip(ref[:3], got[:3]):
                assert np.asarray(a).tobytes() == np.asarray(b).tobytes(), (W, H, mode, depth, k)
            qw = (sc.timeline()[:, 7] & 0x0FFFFFFF).astype(np.int64)
            assert np.array_equal(np.sort(qw), np.arange(len(qw))), "dispatch order is not a permutation"
            orders.append(qw)
        n = len(orders[0])
        C = 64
        full = (n // (8 * C)) * 8 * C
        pos = np.arange(n)
        cls = np.where(pos < full, (pos // C) % 8, pos % 8)  # class of logical wave j (default order's XCD)
        for o in orders[1:]:
            assert not np.array_equal(o, orders[0])          # reordered
            assert (cls[o] == pos % 8).all()                 # every wave keeps its XCD position class


def test_wave_stats_sum_to_frame_counters(rt):
    """RT_FRAME_WAVE_STATS (the per-wave breakdown's input, tools/wave_breakdown.py): each logical wave's own
    counts add up to the counting run's frame totals -- PRIMARY node steps / triangle records / hits, FULL the
    packet phases' node steps and triangle tests (rt_debug_counters ST_PS / ST_PT)."""
    mesh = rt.Mesh.load_obj(scene_path("bunny.obj"))
    sc = rt.Scene(mesh, frames_in_flight=1)
    W, H = 640, 360
    cam = rt.flycam(W, H, 0, 0, 20)
    st = sc.render(cam, rt.DEFAULT_LIGHTS, W, H, flags=rt.RT_FRAME_STATS | rt.RT_FRAME_WAVE_STATS)[1]
    ws = sc.wave_stats().astype(np.int64)
    assert len(ws) == 4 * ((W + 15) // 16) * ((H + 15) // 16)
    assert ws[:, 0].sum() == st["wave_node_fetches"] and ws[:, 1].sum() == st["wave_tri_fetches"]
    assert ws[:, 2].sum() == st["hits"] and (ws[:, 2] <= 64).all()
    sc.render(cam, rt.DEFAULT_LIGHTS, W, H, mode=rt.RT_MODE_FULL, flags=rt.RT_FRAME_STATS | rt.RT_FRAME_WAVE_STATS)
    ws = sc.wave_stats().astype(np.int64)
    c = sc.counters(80)
    ST_PS, ST_PT = 48 + 8, 48 + 12
    assert [int(ws[:, p].sum()) for p in range(4)] == c[ST_PS:ST_PS + 4]
    assert [int(ws[:, 4 + p].sum()) for p in range(4)] == c[ST_PT:ST_PT + 4]
    assert c[ST_PS] > 0 and c[ST_PS + 2] > 0  # primary and reflection walks happened
    with pytest.raises(rt.RTError):  # a frame without the flag has no per-wave record
        sc.render(cam, rt.DEFAULT_LIGHTS, W, H)
        sc.wave_stats()


def test_split_costliest_waves(rt, soup):
    """Lone FULL frames dispatched longest-first trace their costliest waves (FrameParams::split_k) as four
    16-lane sub-waves each: every frame after a slot's first (which has no wave costs yet) must still
    render the bits of the default-order frame (variant 131072: no longest-first order, hence no split),
    for frames large enough to split and for a frame too small to (fewer than 32 waves); the soup (a
    large scene) keeps whole waves, and with RT_SPLIT_K forced the library reads it once per process, so
    the soup case checks the unsplit order path."""
    mesh = rt.Mesh.load_obj(scene_path("bunny.obj"))
    cases = [(rt.Scene(mesh, frames_in_flight=1), 1000, 563), (rt.Scene(mesh, frames_in_flight=1), 24, 16),
             (soup[0], 480, 270)]
    for (sc, W, H), mode in [(c, m) for c in cases for m in (rt.RT_MODE_FULL, rt.RT_MODE_PRIMARY)]:
        cam = rt.flycam(W, H, 0, 0, 20)
        prev = rt.set_variant(131072)
        try:
            ref = sc.render(cam, rt.DEFAULT_LIGHTS, W, H, mode=mode, want_hits=True)
        finally:
            rt.set_variant(prev)
        for k in range(20):  # past the order's refresh (8 frames per slot) on one slot and on four
            got = sc.render(cam, rt.DEFAULT_LIGHTS, W, H, mode=mode, want_hits=True)
            for a, b in zip(ref[:3], got[:3]):
                assert np.asarray(a).tobytes() == np.asarray(b).tobytes(), (W, H, mode, k)


@pytest.mark.parametrize("name", ["cube", "dodgeColorTest", "bunny", "soup"])
def test_box_colors_mode(rt, orc, soup, name):
    """RT_MODE_BOX_COLORS = traceRay with RENDER_BOUNDINGBOX_COLORED_TRIANGLES set (flyscene.cpp:334-348):
    every pixel's colour bit-identical to the oracle's (sum of the colours of the boxes that hasFace() the
    hit face, in box order), with the reference's setRandomColor colours and with caller-set colours;
    the fused kernel, the trace + shade pair, a counting frame and any max_depth render the same bits."""
    if name == "soup":
        sc, osc = soup
        W, H, dz = 480, 270, 20
    else:
        sc = rt.Scene(rt.Mesh.load_obj(scene_path(name + ".obj")))
        osc = orc.Scene(orc.Mesh.load_obj(scene_path(name + ".obj")))
        W, H, dz = (320, 180, 20) if name == "bunny" else (256, 144, 0)
    nb = osc.box_count()
    assert sc.info()["n_ref_boxes"] == nb
    rng = np.random.default_rng(5)
    for colors in (None, rng.uniform(0, 1, (nb, 3)).astype(np.float32)):
        if colors is not None:
            sc.set_box_colors(colors)
        ocol = orc.box_colors_glibc(nb) if colors is None else colors
        cam = rt.flycam(W, H, 0, 0, dz)
        rgb, face, t, st = sc.render(cam, rt.DEFAULT_LIGHTS, W, H, mode=rt.RT_MODE_BOX_COLORS, want_hits=True)
        orgb, oface, ot = osc.render(orc.flycam(W, H, 0, 0, dz), orc.DEFAULT_LIGHTS, W, H, box_colors=ocol,
                                     threads=16)
        assert (face.reshape(-1) == oface).all(), name
        assert same_bits(t.reshape(-1), ot).all(), name
        assert rgb.reshape(-1, 3).tobytes() == orgb.tobytes(), f"{name}: colours differ from the oracle"
        assert (face >= 0).any()
        for kw in (dict(max_depth=3), dict(flags=rt.RT_FRAME_STATS)):
            got = sc.render(cam, rt.DEFAULT_LIGHTS, W, H, mode=rt.RT_MODE_BOX_COLORS, want_hits=True, **kw)
            assert got[0].tobytes() == rgb.tobytes() and got[1].tobytes() == face.tobytes(), kw
        prev = rt.set_variant(32768)
        try:
            got = sc.render(cam, rt.DEFAULT_LIGHTS, W, H, mode=rt.RT_MODE_BOX_COLORS, want_hits=True)
        finally:
            rt.set_variant(prev)
        assert got[0].tobytes() == rgb.tobytes()
    sc.set_box_colors()  # the shared soup scene goes back to the default colours


def _mesh_from(rt, v):
    n = len(v) // 3
    return rt.Mesh.from_arrays(v, np.arange(3 * n, dtype=np.uint32).reshape(-1, 3), np.array([rt.SOUP_MATERIAL], np.float32))


@pytest.mark.parametrize("case", ["nan-vertices", "coincident", "flat", "mixed-scale"])
def test_default_device_builder_edge_scenes(rt, case):
    """The default device SBVH builder (rt_build.hip gpu_build_sah) on scenes that stress it: non-finite
    vertices (the device builders refuse them; the host SBVH builds the tree), 4,000 coincident triangles
    (degenerate centroids: position medians down to leaves of <= 16), a flat soup (one extent 0) and a soup
    mixing 1e-4- and 1-sized triangles. Every tree passes the split-aware validator and renders the host
    SBVH scene's frames bit for bit (PRIMARY and FULL)."""
    rng = np.random.default_rng(11)
    v = rt.generate_soup(20_000, 7).astype(np.float32)
    if case == "nan-vertices":
        v[rng.integers(0, len(v), 12), rng.integers(0, 3, 12)] = np.nan
    elif case == "coincident":
        v[: 3 * 4000] = np.tile(np.float32([[0.1, 0.1, 0.3], [0.2, 0.1, 0.3], [0.1, 0.2, 0.3]]), (4000, 1))
    elif case == "flat":
        v[:, 2] = np.float32(0.25)
    else:
        c = v.reshape(-1, 3, 3).mean(1, keepdims=True)
        small = rng.random(len(c)) < 0.5
        v = v.reshape(-1, 3, 3)
        v[small] = c[small] + (v[small] - c[small]) * np.float32(1e-2)
        v = v.reshape(-1, 3).astype(np.float32)
    mesh = _mesh_from(rt, v)
    dev = rt.Scene(mesh)
    host = rt.Scene(mesh, builder=rt.RT_BUILDER_SBVH)
    want = rt.RT_BUILDER_SBVH if case == "nan-vertices" else rt.RT_BUILDER_SBVH_GPU
    assert dev.info()["builder"] == want, (case, dev.info()["builder"])
    if case != "nan-vertices":  # (the validator's containment checks are undefined for NaN triangles)
        val = dev.validate_bvh()
        assert val["ok"] and val["covered2"] >= dev.info()["n_faces"], val
    W, H = 480, 270
    cam = rt.flycam(W, H, 0, 0, 20)
    for m in (rt.RT_MODE_PRIMARY, rt.RT_MODE_FULL):
        a = host.render(cam, rt.DEFAULT_LIGHTS, W, H, mode=m, want_hits=True)
        b = dev.render(cam, rt.DEFAULT_LIGHTS, W, H, mode=m, want_hits=True)
        assert (np.asarray(a[1]) >= 0).sum() > 1000, case
        for x, y in zip(a[:3], b[:3]):
            assert np.asarray(x).tobytes() == np.asarray(y).tobytes(), (case, m)


def test_device_builders_large_scene(rt):
    """The device builders at 3M triangles (3x the BASELINE scenes: reference budget, task and bin arrays
    sized from the face count): the SBVH and binned-SAH device trees are sound by the host validator and
    render the same frame bit for bit; the SBVH tree's SAH cost is the lower one."""
    mesh, _, _ = rt.soup_mesh(3_000_000, 99)
    sb = rt.Scene(mesh, builder=rt.RT_BUILDER_SBVH_GPU)
    sa = rt.Scene(mesh, builder=rt.RT_BUILDER_SAH_GPU)
    assert sb.info()["builder"] == rt.RT_BUILDER_SBVH_GPU and sa.info()["builder"] == rt.RT_BUILDER_SAH_GPU
    for sc in (sb, sa):
        v = sc.validate_bvh()
        assert v["ok"] and v["covered2"] >= 3_000_000, v
    assert sb.tree_cost()["sah"] < sa.tree_cost()["sah"]
    W, H = 960, 540
    cam = rt.flycam(W, H, 0, 0, 20)
    a = sb.render(cam, rt.DEFAULT_LIGHTS, W, H, want_hits=True)
    b = sa.render(cam, rt.DEFAULT_LIGHTS, W, H, want_hits=True)
    assert (np.asarray(a[1]) >= 0).sum() > W * H // 2
    for x, y in zip(a[:3], b[:3]):
        assert np.asarray(x).tobytes() == np.asarray(y).tobytes()


@pytest.mark.parametrize("builder", ["sbvh", "sbvhgpu", "sahgpu"])
@pytest.mark.parametrize("leaf", [1, 2, 8, 16])
def test_leaf_sizes_render_identical_bits(rt, soup, builder, leaf):
    """Leaf bounds 1..kMaxLeaf (16) through the host and device builders: the leaf loops (and the leaf-entry
    prefetch of a leaf's remaining triangle records) give the frame of the default scene bit for bit, PRIMARY
    and FULL, binary and 4-wide trees; the bunny and the 1M soup."""
    bid = {"sbvh": rt.RT_BUILDER_SBVH, "sbvhgpu": rt.RT_BUILDER_SBVH_GPU, "sahgpu": rt.RT_BUILDER_SAH_GPU}[builder]
    bunny = rt.Mesh.load_obj(scene_path("bunny.obj"))
    ref_b = rt.Scene(bunny)
    ref_s, _ = soup
    cases = [(bunny, ref_b, (960, 540))]
    if builder != "sbvh" or leaf == 16:  # the 1M soup's host SBVH takes seconds per build: its largest leaves only
        cases.append((ref_s.mesh, ref_s, (640, 360)))
    for mesh, ref, (W, H) in cases:
        sc = rt.Scene(mesh, builder=bid, leaf_size=leaf, wide_tree=1 if leaf >= 8 else 0)
        v = sc.validate_bvh()
        assert v["ok"], v
        cam = rt.flycam(W, H, 0, 0, 20)
        for m in (rt.RT_MODE_PRIMARY, rt.RT_MODE_FULL):
            a = ref.render(cam, rt.DEFAULT_LIGHTS, W, H, mode=m, want_hits=True)
            b = sc.render(cam, rt.DEFAULT_LIGHTS, W, H, mode=m, want_hits=True)
            for x, y in zip(a[:3], b[:3]):
                assert np.asarray(x).tobytes() == np.asarray(y).tobytes(), (builder, leaf, m)
