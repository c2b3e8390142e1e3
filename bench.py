#!/usr/bin/env python3
"""Benchmark of the MI355X ray-traversal hot path (BASELINE.json metric).

Metric: "Mrays/s (primary) + frame ms at 1920x1080, 1M-tri BVH, 1/2/4/8 GPU".
Workload (C3): 1,000,000 random triangles (SplitMix64 seed 12345), Flycamera eye
(0,0,1) (translate(0,0,20)), fovy 60, one white light at (-0.5,2,3), PRIMARY mode (closest hit +
unshadowed Phong). A step = one frame: one launch of the render kernel over this rank's 16x16 tiles.
Scene and frame buffer are resident in HBM before the timed region; no host copies inside it.

Multi-GPU (one process per GPU, torchrun): the frame grows with N at 16:9 so that every GPU traces a
1080p-equivalent share (weak scaling; N=4 is C4's 3840x2160); tiles are interleaved over ranks, the
scene is replicated, and there is no collective on the data path (barrier + max/sum reductions of the
timing only). `--frame WxH` fixes the frame instead (strong scaling, e.g. --frame 3840x2160).

Prints ONE JSON line on rank 0 (contract in the task statement), including:
  roofline: algorithmic bytes per ray B = 64*N_node + 40*N_tri + 92*hit + 12 from a
            counting run of the same kernel on the same frame, times rays per launch, over the average
            launch duration measured with HIP events on the library's stream; peak 8 TB/s HBM3E.
  cpu_baseline: the CPU restatement of the reference algorithm (oracle/, "port") on a bounded pixel
            sample of the same frame, timed on this host's cores.
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "ray-tracing-project_amd")


def load_rtamd():
    import importlib.util
    spec = importlib.util.spec_from_file_location("rtamd", os.path.join(PKG, "rtamd.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def frame_for(n_gpus, override):
    if override:
        w, h = override.lower().split("x")
        return int(w), int(h), "strong"
    s = math.sqrt(n_gpus)
    return 8 * round(1920 * s / 8), 8 * round(1080 * s / 8), "weak"


def cpu_baseline(scene, soup_args, W, H, full, target_s, threads):
    """Oracle ("port" of the reference algorithm) on a strided pixel sample of the same frame."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    t0 = time.perf_counter()
    if scene == "soup":
        n_tris, seed, mat = soup_args
        v = O.generate_soup(n_tris, seed)
        f = np.arange(3 * n_tris, dtype=np.uint32).reshape(-1, 3)
        sc = O.Scene(O.Mesh.from_arrays(v, f, np.array([mat], np.float32)))
        what = f"{n_tris}-tri soup"
    else:
        sc = O.Scene(O.Mesh.load_obj(os.path.join(ROOT, "scenes", "bunny.obj")))
        what = "bunny"
    build_s = time.perf_counter() - t0
    cam = O.flycam(W, H, 0, 0, 20)

    def run(k):  # every k-th pixel of the frame in row-major order (a deterministic, spread sample)
        idx = np.arange(k // 2, W * H, k, dtype=np.int64)
        pix = np.stack([idx % W, idx // W], axis=1).astype(np.int32)
        t = time.perf_counter()
        sc.render(cam, O.DEFAULT_LIGHTS, W, H, full=full, pixels=pix, threads=threads)
        return len(pix), time.perf_counter() - t

    n, dt = run(509)  # calibration sample (~4k rays)
    k = 509
    for _ in range(3):
        rate = n / max(dt, 1e-6)
        k = max(1, math.ceil(W * H / max(rate * target_s, 1.0)))
        n, dt = run(k)
        if dt > 0.6 * target_s or k == 1:
            break
    return {"value": round(n / dt / 1e6, 6), "unit": "Mrays/s", "cores": threads, "kind": "port",
            "sample": f"{n} primary rays = every {k}th pixel (row-major) of the same {W}x{H} frame "
                      f"({what}, eye (0,0,1), {'FULL' if full else 'PRIMARY'}); {dt:.1f} s of CPU work on "
                      f"{threads} threads; box partition build {build_s:.1f} s excluded"}


def shard_tiles(W, H, rank, n):
    """16x16 tiles this rank renders (the kernel's assignment: tile t goes to rank t % n)."""
    tx = (W + 15) // 16
    return [(t % tx, t // tx) for t in range(rank, tx * ((H + 15) // 16), n)]


def e2e_frame_ms(rt, sc, cam, W, H, mode, rank, n, dist, iters=5):
    """End-to-end frame with the output path: render this rank's tiles, pack them as 8-bit,
    gather every rank's slice on rank 0 (RCCL all-gather over xGMI; gloo via host when rehearsing), unpack
    there and copy the 8-bit frame to the host. Not the bench value: the PCIe-inclusive latency."""
    import torch
    slice_b = rt.shard_bytes(W, H, n)
    on_gpu = dist is None or backend_is_nccl(dist)
    slc = torch.empty(slice_b, dtype=torch.uint8, device="cuda")
    gathered = torch.empty(n * slice_b, dtype=torch.uint8, device="cuda" if on_gpu else "cpu")
    frame = torch.empty(W * H * 3, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters + 1):
        if dist is not None:
            dist.barrier()
        t = time.perf_counter()
        sc.render_async(cam, rt.DEFAULT_LIGHTS, W, H, mode=mode, shard=(rank, n))
        sc.synchronize()
        if n == 1:
            host, _ = sc.download_rgb8(W, H)
        else:
            sc.pack_shard_rgb8(slc.data_ptr())
            if on_gpu:
                dist.all_gather_into_tensor(gathered, slc)
            else:
                dist.all_gather_into_tensor(gathered, slc.cpu())
            if rank == 0:
                src = gathered if on_gpu else gathered.cuda()
                torch.cuda.synchronize()
                rt.unpack_shards_rgb8(src.data_ptr(), n, W, H, frame.data_ptr(), torch.cuda.current_device())
                host = frame.cpu()
        ts.append((time.perf_counter() - t) * 1e3)
    return sorted(ts[1:])[len(ts[1:]) // 2]


def backend_is_nccl(dist):
    return dist is not None and dist.get_backend() == "nccl"


def make_reducer(dist, dev):
    import torch

    def reduce(x, op):
        if dist is None:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=getattr(dist.ReduceOp, op))
        return float(t.item())
    return reduce


def measured_traffic(W, H, n_faces, mode, kernel_ms, kernel):
    """HBM traffic of the same kernel on the same workload from the committed rocprofv3 PMC summary
    (profiles/pmc_latest.json, tools/profile.sh + tools/summarize_profile.py): 2*FETCH_SIZE + WRITE_SIZE
    bytes per launch (gfx950 correction), expressed as GB/s over this run's average launch time."""
    p = os.path.join(ROOT, "profiles", "pmc_latest.json")
    if not os.path.exists(p):
        return None, None
    d = json.load(open(p))
    cfg = d.get("bench_line_under_trace", {}).get("config", {})
    if cfg.get("frame") != f"{W}x{H}" or cfg.get("triangles") != n_faces or cfg.get("mode") != mode:
        return None, None
    if not str(d.get("kernel", "")).startswith(kernel + "<"):  # profiled with another kernel form
        return None, None
    b = d.get("hbm_bytes_per_launch")
    if not b:
        return None, None
    return round(b / (kernel_ms * 1e-3) / 1e9, 1), (f"profiles/{d.get('tag')}_pmc.json: "
                                                   f"{b / 1e6:.1f} MB per launch (2*FETCH_SIZE+WRITE_SIZE)")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--tris", type=int, default=1_000_000)
    ap.add_argument("--frame", default=None, help="WxH (strong scaling); default 1080p per GPU (weak)")
    ap.add_argument("--mode", choices=["primary", "full"], default="primary")
    ap.add_argument("--scene", default="soup", help="soup | bunny")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-stats", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the end-to-end (render + 8-bit frame to host) timing")
    ap.add_argument("--leaf", type=int, default=0, help="BVH leaf size bound (0 = library default)")
    ap.add_argument("--builder", choices=["sah", "lbvh"], default="sah",
                    help="BVH builder: host binned SAH (default) or the device LBVH (SURVEY f2)")
    ap.add_argument("--frames-in-flight", type=int, default=0,
                    help="frames that may overlap on the GPU (0 = library default, 4)")
    a = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal knob: BENCH_DEVICE pins every rank to one device (several ranks sharing one GPU, with
    # BENCH_BACKEND=gloo for the timing reductions); unset in real runs (one GPU per rank)
    if "BENCH_DEVICE" in os.environ:
        local = int(os.environ["BENCH_DEVICE"])
    if world != a.gpus and world > 1:
        print(f"warning: WORLD_SIZE {world} != --gpus {a.gpus}", file=sys.stderr)
    n = max(world, 1)

    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        backend = os.environ.get("BENCH_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
        if torch.cuda.is_available():
            torch.cuda.set_device(local)
        dist.init_process_group(backend=backend)
    elif torch.cuda.is_available():
        torch.cuda.set_device(local)
    dev = torch.device("cuda", local) if (torch.cuda.is_available() and backend_is_nccl(dist)) else torch.device("cpu")

    def barrier():
        if dist is not None:
            dist.barrier()

    reduce = make_reducer(dist, dev)

    rt = load_rtamd()
    W, H, scaling = frame_for(n, a.frame)
    t0 = time.perf_counter()
    if a.scene == "soup":
        mesh, _, _ = rt.soup_mesh(a.tris, 12345)
        scene_name = f"{a.tris} random triangles (SplitMix64 seed 12345)"
    else:
        mesh = rt.Mesh.load_obj(os.path.join(ROOT, "scenes", "bunny.obj"))
        scene_name = "Stanford bunny (69,451 triangles)"
    sc = rt.Scene(mesh, device=local, leaf_size=a.leaf, frames_in_flight=a.frames_in_flight,
                  builder=rt.RT_BUILDER_LBVH_GPU if a.builder == "lbvh" else rt.RT_BUILDER_SAH)
    info = sc.info()
    info_fif = a.frames_in_flight or 4
    setup_s = time.perf_counter() - t0
    cam = rt.flycam(W, H, 0, 0, 20)
    mode = rt.RT_MODE_FULL if a.mode == "full" else rt.RT_MODE_PRIMARY
    shard = (rank, n)

    for _ in range(a.warmup):
        sc.render_async(cam, rt.DEFAULT_LIGHTS, W, H, mode=mode, shard=shard)
    sc.synchronize()

    barrier()
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    t_start = time.perf_counter()
    for _ in range(a.steps):
        sc.render_async(cam, rt.DEFAULT_LIGHTS, W, H, mode=mode, shard=shard)
    st = sc.synchronize()
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t_start

    my_rays = st["primary_rays"] * a.steps
    elapsed_max = reduce(elapsed, "MAX")
    total_rays = reduce(float(my_rays), "SUM")
    kernel_ms_avg = st["kernel_ms"] / max(st["launches"], 1)
    kernel_ms_max = reduce(kernel_ms_avg, "MAX")

    trace_ms_avg = st["trace_kernel_ms"] / max(st["launches"], 1)
    trace_ms_max = reduce(trace_ms_avg, "MAX")
    roof = None
    stats = None
    if rank == 0 and not a.no_stats:
        # counting run of the same kernels on the same frame (RT_FRAME_STATS)
        sc.render_async(cam, rt.DEFAULT_LIGHTS, W, H, mode=mode, shard=shard, flags=rt.RT_FRAME_STATS)
        stats = sc.synchronize()
        rays = max(stats["primary_rays"], 1)
        n_node = stats["node_visits"] / rays
        n_tri = stats["tri_tests"] / rays
        hit = stats["hits"] / rays
        # B = 64 N_node + 40 N_tri + 92 hit + 12 per ray. PRIMARY runs as one kernel
        # (k_primary_fused: traversal + shading, so its share is the whole B); with RT_KERNEL_VARIANT bit
        # 32768 it runs as k_trace_primary (64 N_node + 40 N_tri + its 8-B hit record) + k_shade_primary.
        # FULL: k_render_full carries B (its secondary rays on top are not counted).
        split = mode == rt.RT_MODE_PRIMARY and (int(os.environ.get("RT_KERNEL_VARIANT", "0") or 0) & (32768 | 256 | 2048))
        b_trace = 64 * n_node + 40 * n_tri + 8
        b_ray = 64 * n_node + 40 * n_tri + 92 * hit + 12
        b_kern = b_trace if split else b_ray
        kern_ms = trace_ms_avg if mode == rt.RT_MODE_PRIMARY else kernel_ms_avg
        achieved = b_kern * st["primary_rays"] / (kern_ms * 1e-3) / 1e9
        kname = ("k_trace_primary" if split else "k_primary_fused") if mode == rt.RT_MODE_PRIMARY else "k_render_full"
        traffic, traffic_note = measured_traffic(W, H, info["n_faces"], a.mode, kern_ms, kname)
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": 8000.0, "unit": "GB/s",
                "frac": round(achieved / 8000.0, 4), "traffic": traffic, "traffic_source": traffic_note,
                "kernel": kname,
                "kernel_ms": round(kern_ms, 4), "bytes_per_ray_kernel": round(b_kern, 1),
                "bytes_per_ray_path": round(b_ray, 1), "n_node": round(n_node, 2), "n_tri": round(n_tri, 2),
                "hit": round(hit, 4),
                "path_achieved_GBps": round(b_ray * st["primary_rays"] / (kernel_ms_avg * 1e-3) / 1e9, 1),
                # the same bytes over the wall-clock interval per frame (frames overlap in flight)
                "achieved_throughput_GBps": round(b_kern * st["primary_rays"] / (elapsed / a.steps) / 1e9, 1),
                "wave_fetch_bytes_per_ray": round((64 * stats["wave_node_fetches"] + 64 * stats["wave_tri_fetches"]) / rays, 2)}

    e2e = None
    if not a.no_e2e and torch.cuda.is_available():
        e2e = reduce(e2e_frame_ms(rt, sc, cam, W, H, mode, rank, n, dist), "MAX")

    cpu = None
    if rank == 0 and n == 1 and not a.no_cpu:
        threads = min(16, os.cpu_count() or 1)
        cpu = cpu_baseline(a.scene, (a.tris, 12345, rt.SOUP_MATERIAL), W, H, a.mode == "full", a.cpu_seconds,
                           threads)

    if rank == 0:
        value = total_rays / elapsed_max / 1e6
        if a.scene == "soup":
            cname = "C3" if (W, H) == (1920, 1080) else ("C4" if (W, H) == (3840, 2160) else "C3-family")
        else:
            cname = "C5" if a.mode == "full" else "C2"
        extra = {}
        if e2e is not None:
            # one frame end to end: render + 8-bit frame assembled on rank 0 (RCCL all-gather for N>1) + D2H
            extra["e2e_frame_ms"] = round(e2e, 3)
        if stats is not None:
            extra["rays_per_frame_total"] = stats["total_rays"]  # primary + shadow + reflection (FULL)
            extra["total_mrays_per_s"] = round(stats["total_rays"] * n * a.steps / elapsed_max / 1e6, 2)
        out = {
            "metric": "Mrays/s (primary) + frame ms at 1920x1080, 1M-tri BVH, 1/2/4/8 GPU",
            "value": round(value, 2),
            "unit": "Mrays/s",
            "n_gpus": n,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(elapsed_max / a.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic",
            "config": {"workload": f"{cname}: {scene_name}, {W}x{H} {a.mode} rays, eye (0,0,1), 1 light",
                       "frame": f"{W}x{H}", "triangles": info["n_faces"], "mode": a.mode,
                       "parallelism": f"tiles/{n} (16x16 tiles interleaved over ranks, scene replicated)",
                       "frames_in_flight": info_fif,
                       # per-frame latency (first kernel start to last kernel end of one frame); with
                       # frames in flight, frames overlap and ms_per_step is the throughput interval
                       "kernel_ms_per_frame": round(kernel_ms_max, 4),
                       "trace_kernel_ms": round(trace_ms_max, 4),
                       "kernel_mrays_per_s": round(total_rays / a.steps / (kernel_ms_max * 1e-3) / 1e6, 2),
                       "bvh_nodes": info["bvh_nodes"], "bvh_depth": info["bvh_depth"],
                       "ref_boxes": info["n_ref_boxes"], "scene_setup_s": round(setup_s, 2),
                       "builder": "lbvh-gpu" if info["builder"] == 1 else "sah-host",
                       "build_ms": {"prep": round(info["prep_ms"], 1), "ref_boxes": round(info["boxes_ms"], 1),
                                    "bvh": round(info["bvh_ms"], 1), "bvh_gpu_kernels": round(info["bvh_gpu_ms"], 2),
                                    "upload": round(info["upload_ms"], 1)}, **extra},
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
