"""Multi-GPU path on CPU: the tile partition used across ranks, the gloo-backed timing reductions
bench.py performs (world_size 2), and that per-rank renders stitch to the single-device frame
(oracle as the renderer, since the CPU container has no GPU)."""
import importlib.util
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT, scene_path

spec = importlib.util.spec_from_file_location("bench", os.path.join(ROOT, "bench.py"))
bench = importlib.util.module_from_spec(spec)
spec.loader.exec_module(bench)


@pytest.mark.parametrize("WH", [(1920, 1080), (3840, 2160), (37, 11), (8, 8)])
@pytest.mark.parametrize("n", [1, 2, 3, 4, 8])
def test_tile_partition_is_exact_cover(WH, n):
    W, H = WH
    seen = {}
    for r in range(n):
        for t in bench.shard_tiles(W, H, r, n):
            assert t not in seen
            seen[t] = r
    assert len(seen) == ((W + 15) // 16) * ((H + 15) // 16)
    counts = np.bincount(list(seen.values()), minlength=n)
    S = bench.SHARD_SUPER_TILE if n > 1 else 1
    assert counts.max() - counts.min() <= S * S  # interleaving super-tiles balances tile counts


@pytest.mark.parametrize("WH", [(1920, 1080), (3840, 2160), (1000, 600), (37, 11), (8, 8)])
@pytest.mark.parametrize("n", [1, 2, 3, 4, 8])
def test_shard_tiles_match_library(rt, WH, n):
    """bench.shard_tiles (the host-side restatement) lists exactly the library's tiles, in its slot order,
    and rt_frame_shard_bytes holds the largest shard's slots."""
    W, H = WH
    for r in range(n):
        assert bench.shard_tiles(W, H, r, n) == rt.shard_tiles(W, H, r, n), (r, n)
    S = bench.SHARD_SUPER_TILE if n > 1 else 1
    sx, sy = -(-((W + 15) // 16) // S), -(-((H + 15) // 16) // S)
    assert rt.shard_bytes(W, H, n) == -(-(sx * sy) // n) * S * S * 768
    # a smaller buffer receives only its capacity
    import ctypes
    full = rt.shard_tiles(W, H, 0, n)
    buf = (ctypes.c_int32 * 4)(*([-1] * 4))
    assert rt.lib().rt_frame_shard_tiles(W, H, 0, n, ctypes.cast(buf, ctypes.c_void_p), 1) == len(full)
    assert list(buf) == [full[0][0], full[0][1], -1, -1]


def test_default_frames_are_baseline_configs():
    """N = 1: C3's 1920x1080 frame; N > 1: C4's fixed 3840x2160 frame split over the ranks (strong
    scaling), so every multi-GPU line lands on a BASELINE config."""
    assert bench.frame_for(1, None) == (1920, 1080)
    for n in (2, 4, 8):
        assert bench.frame_for(n, None) == (3840, 2160)
    assert bench.frame_for(8, "1920x1080") == (1920, 1080)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    reduce = bench.make_reducer(dist, torch.device("cpu"))
    dist.barrier()
    q.put((rank, reduce(1.0 + rank, "MAX"), reduce(100.0 * (rank + 1), "SUM")))
    dist.destroy_process_group()


def test_gloo_two_rank_timing_reduction():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [r[1] for r in res] == [2.0, 2.0]       # max over ranks of elapsed
    assert [r[2] for r in res] == [300.0, 300.0]   # whole-job rays


def test_sharded_renders_stitch_to_full_frame(orc):
    W, H, n = 44, 30, 3
    sc = orc.Scene(orc.Mesh.load_obj(scene_path("cube.obj")))
    cam = orc.flycam(W, H)
    full, _, _ = sc.render(cam, orc.DEFAULT_LIGHTS, W, H)
    out = np.full((H, W, 3), np.nan, np.float32)
    for r in range(n):
        pix = [(x, y) for tx, ty in bench.shard_tiles(W, H, r, n)
               for y in range(ty * 16, min(H, ty * 16 + 16)) for x in range(tx * 16, min(W, tx * 16 + 16))]
        rgb, _, _ = sc.render(cam, orc.DEFAULT_LIGHTS, W, H, pixels=pix)
        for (x, y), c in zip(pix, rgb):
            out[y, x] = c
    assert out.tobytes() == full.reshape(H, W, 3).tobytes()


def _shared_worker(rank, world, port, path, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import conftest
    rt = conftest.rtamd
    mesh = rt.Mesh.load_obj(scene_path("bunny.obj"))
    sc, secs = bench.shared_scene(lambda: rt.Scene(mesh, device=rt.RT_DEVICE_NONE),
                                  lambda p: rt.Scene.load(p, device=rt.RT_DEVICE_NONE), rank, dist.barrier, path)
    info = sc.info()
    per_rank = bench.gather_all(dist, torch.device("cpu"), secs)
    q.put((rank, info["bvh_nodes"], info["n_ref_boxes"], info["builder"], sc.validate_bvh()["ok"], per_rank))
    dist.destroy_process_group()


def test_gloo_scene_built_once_per_node(tmp_path):
    """with N > 1 ranks on one node, rank 0 builds the scene and writes the f1 cache,
    the others load it (bench.shared_scene); every rank ends up with the same tree, and the cache file
    is removed afterwards."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    path = str(tmp_path / "shared.rtscene")
    procs = [ctx.Process(target=_shared_worker, args=(r, 3, port, path, q)) for r in range(3)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert len({r[1:4] for r in res}) == 1 and all(r[4] for r in res)
    assert res[0][3] == 2  # RT_BUILDER_SBVH, kept by the cache
    assert len(res[0][5]) == 3 and all(x >= 0 for x in res[0][5])
    assert not os.path.exists(path)


def test_bench_refuses_more_gpus_than_visible():
    """`python bench.py --gpus 8` without a launcher is the in-process multi-device run; with fewer visible
    devices it must fail, never print an n_gpus 1 line. Also a launcher whose
    WORLD_SIZE differs from --gpus."""
    import subprocess
    import sys
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env["CUDA_VISIBLE_DEVICES"] = env["HIP_VISIBLE_DEVICES"] = ""  # no visible GPU, whatever the host has
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--steps", "1", "--warmup", "0"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode != 0
    assert '"n_gpus"' not in r.stdout
    assert "visible" in r.stderr
    env["WORLD_SIZE"] = "2"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--steps", "1"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr


def test_timed_window_must_hold_its_frames():
    """bench.timed_frames stops its clock after the caller's device synchronise and reads the frames' event times
    afterwards; a synchronise that drains nothing (the frames still running) must fail, not report the enqueue rate."""
    import pytest

    class FakeScene:  # frames "take" 1 ms of kernel time each; render_async returns at once
        def __init__(self):
            self.n = 0

        def render_async(self, *a, **k):
            self.n += 1

        def synchronize(self):
            self.n = 0
            return {}

        def synchronize_devices(self):
            n, self.n = self.n, 0
            return {"kernel_ms": 1.0 * n, "launches": n, "primary_rays": 100}, []

    class FakeRT:
        DEFAULT_LIGHTS = []

    with pytest.raises(RuntimeError, match="not drained"):
        bench.timed_frames(FakeRT, FakeScene(), None, 8, 8, 0, (0, 1), 4, 1, lambda: None, lambda: None)
    # a window that could hold the frames only if more than the library's 4 frame slots ran at once (ADVICE r5:
    # the bound is the summed frame time / slots, not one frame's time)
    with pytest.raises(RuntimeError, match="not drained"):
        bench.timed_frames(FakeRT, FakeScene(), None, 8, 8, 0, (0, 1), 8, 1, lambda: None,
                           lambda: __import__("time").sleep(0.0015))
    el, st = bench.timed_frames(FakeRT, FakeScene(), None, 8, 8, 0, (0, 1), 4, 1, lambda: None,
                                lambda: __import__("time").sleep(0.01))
    assert st["launches"] == 4 and el >= 0.01 and st["prewarm_frames"] == 0
