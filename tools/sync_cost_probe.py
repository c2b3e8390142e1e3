"""Where the end of bench.py's timed region goes: C3 (1M soup, 1920x1080 PRIMARY, 4 frames in flight), K frames
timed as bench.py does (A: rt_synchronize_devices -- wait + per-frame event read-out -- then device synchronise)
against B (device synchronise only; the event read-out after the clock stops), interleaved reps. Also the host
cost of the read-out alone (GPU already idle). One JSON line per rep. Usage: python tools/sync_cost_probe.py [K] [reps] [prewarm batch] [early torch init 0/1] [plain|mimic] [prewarm ms]"""
import importlib.util
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("rtamd", os.path.join(ROOT, "ray-tracing-project_amd", "rtamd.py"))
rt = importlib.util.module_from_spec(spec)
spec.loader.exec_module(rt)


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    B = int(sys.argv[3]) if len(sys.argv) > 3 else 4  # frames per synchronised batch in the 50 ms prewarm
    early = len(sys.argv) > 4 and sys.argv[4] == "1"  # torch's CUDA state initialised before the scene is built
    if early:
        torch.cuda.synchronize()
    mesh, _, _ = rt.soup_mesh(1_000_000, 12345)
    sc = rt.Scene(mesh, device=0)
    W, H = 1920, 1080
    cam = rt.flycam(W, H, 0, 0, 20)
    mode = rt.RT_MODE_PRIMARY

    def frames(n):
        for _ in range(n):
            sc.render_async(cam, rt.DEFAULT_LIGHTS, W, H, mode=mode, shard=(0, 1))

    mimic = len(sys.argv) > 5 and sys.argv[5] == "mimic"  # prewarm batches end as the timed region does
    pw = float(sys.argv[6]) / 1e3 if len(sys.argv) > 6 else 0.05  # prewarm seconds
    t = time.perf_counter()
    while time.perf_counter() - t < pw:
        frames(B)
        if mimic:
            sc.synchronize_devices()
            torch.cuda.synchronize()
        else:
            sc.synchronize()
    for rep in range(reps):
        for form in ("A", "B"):
            frames(5)
            sc.synchronize()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            frames(K)
            if form == "A":
                t_q = time.perf_counter()
                st, _ = sc.synchronize_devices()
                torch.cuda.synchronize()
                el = time.perf_counter() - t0
                readout = None
            else:
                t_q = time.perf_counter()
                torch.cuda.synchronize()
                el = time.perf_counter() - t0
                t1 = time.perf_counter()
                st, _ = sc.synchronize_devices()
                readout = (time.perf_counter() - t1) * 1e3
            print(json.dumps({"prewarm_ms": pw * 1e3, "mimic": mimic, "early_torch_init": early, "B": B, "rep": rep, "form": form, "K": K, "ms_per_frame": round(el / K * 1e3, 4),
                              "mrays_s": round(st["primary_rays"] * K / el / 1e6, 1),
                              "enqueue_ms": round((t_q - t0) * 1e3, 3),
                              "readout_ms_idle": None if readout is None else round(readout, 4),
                              "kernel_ms_per_frame": round(st["kernel_ms"] / max(st["launches"], 1), 4)}), flush=True)


if __name__ == "__main__":
    main()
