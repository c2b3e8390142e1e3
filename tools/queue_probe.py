"""Frames in flight vs the HIP runtime's hardware queues (GPU box): how far consecutive rt_render_async frames
overlap in a fresh process, for a few stream-creation situations before the scene's frame-slot streams.

  python tools/queue_probe.py <variant> <scene> <frames_in_flight>
variants: plain (the scene is the process's first), pre<K> (K extra HIP streams created -- and kept -- first),
second (a first scene of the same mesh created and destroyed before), keep2 (a first scene kept alive).
Prints one JSON line: Mrays/s, ms per frame, kernel ms per frame (first kernel start to last kernel end of a
frame: ~ms per frame x frames in flight when they overlap fully)."""
import json
import os
import sys
import time

import torch  # noqa: F401  (first, as in bench.py: the process's HIP runtime comes up with torch's)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ray-tracing-project_amd"))
import rtamd as rt  # noqa: E402


def main(variant, scene, fif, steps=60):
    fif = int(fif)
    if scene == "soup":
        mesh, _, _ = rt.soup_mesh(1_000_000, 12345)
        mode = rt.RT_MODE_PRIMARY
    else:
        mesh = rt.Mesh.load_obj(os.path.join(ROOT, "scenes", "bunny.obj"))
        mode = rt.RT_MODE_FULL
    keep = []
    if variant.startswith("pre"):
        keep = [torch.cuda.Stream() for _ in range(int(variant[3:]))]
        for s in keep:  # first use
            with torch.cuda.stream(s):
                torch.zeros(1, device="cuda")
        torch.cuda.synchronize()
    if variant == "second":
        first = rt.Scene(mesh, frames_in_flight=fif)
        del first
    if variant == "keep2":
        keep.append(rt.Scene(mesh, frames_in_flight=fif))
    sc = rt.Scene(mesh, frames_in_flight=fif)
    W, H = 1920, 1080
    cam = rt.flycam(W, H, 0, 0, 20)
    for _ in range(8):
        sc.render_async(cam, rt.DEFAULT_LIGHTS, W, H, mode=mode)
    sc.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        sc.render_async(cam, rt.DEFAULT_LIGHTS, W, H, mode=mode)
    st = sc.synchronize()
    el = time.perf_counter() - t0
    print(json.dumps({"variant": variant, "scene": scene, "fif": fif, "mrays_per_s": round(W * H * steps / el / 1e6, 1),
                      "ms_per_frame": round(el / steps * 1e3, 4),
                      "kernel_ms_per_frame": round(st["kernel_ms"] / max(st["launches"], 1), 4),
                      "hw_queues_env": os.environ.get("GPU_MAX_HW_QUEUES")}), flush=True)


if __name__ == "__main__":
    main(*sys.argv[1:4])
