#!/usr/bin/env python3
"""Lone frames under the reference's moving camera: one frame at a time (each frame
synchronised before the next is queued, as rt_render does), a static camera against rtamd.CameraPath (WASD held,
flyscene.cpp:116-127), on a 1-slot and a 4-slot scene, for the longest-first dispatch policies of this library
(RT_LPT_MOVED / RT_LPT_REFRESH debug knobs) or another build of it (RTAMD_LIB, e.g. the round-5 library whose
cost maps were per frame slot). One JSON line per measurement.

Usage: RTAMD_DEBUG_KNOBS=1 python tools/moving_ab.py <soup|bunny> <primary|full> <policy> [frames] [reps]
  policy: lib (the library as built), moved0 / moved1 (RT_LPT_MOVED), r1 (RT_LPT_REFRESH=1), nolpt (variant 131072),
          dil0 / dil1 / dil2 (RT_LPT_DILATE: a moving camera's cost map dilated over r waves), nopred (RT_LPT_PRED=0:
          the map dilated around each wave's own position, not its predicted one), exact (every pose
          rendered twice and the second render timed: its map was recorded at the same pose -- the best an order
          from wave costs can do on the moving poses), env:K=V[,K=V...] (any debug knobs)
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

scene, mode, policy = sys.argv[1], sys.argv[2], sys.argv[3]
frames = int(sys.argv[4]) if len(sys.argv) > 4 else 60
reps = int(sys.argv[5]) if len(sys.argv) > 5 else 2
env = {"moved0": {"RT_LPT_MOVED": "0"}, "moved1": {"RT_LPT_MOVED": "1"}, "r1": {"RT_LPT_REFRESH": "1"},
       "dil0": {"RT_LPT_DILATE": "0"}, "dil1": {"RT_LPT_DILATE": "1"}, "dil2": {"RT_LPT_DILATE": "2"},
       "nopred": {"RT_LPT_PRED": "0"}, "exact": {"RT_LPT_DILATE": "0", "RT_LPT_PRED": "0"}}.get(policy, {})
if policy.startswith("env:"):  # any debug knobs, e.g. env:RT_SPLIT_KP_ANY=1,RT_LPT_MOVED=1
    env = dict(kv.split("=", 1) for kv in policy[4:].split(","))
os.environ.update(env)
rt = bench.load_rtamd()
import torch  # noqa: E402

W, H = 1920, 1080
if scene == "soup":
    mesh, _, _ = rt.soup_mesh(1_000_000, 12345)
else:
    mesh = rt.Mesh.load_obj(os.path.join(ROOT, "scenes", "bunny.obj"))
m = rt.RT_MODE_FULL if mode == "full" else rt.RT_MODE_PRIMARY
if policy == "nolpt":
    rt.set_variant(131072)
lib = os.path.basename(os.environ.get("RTAMD_LIB", "librtamd.so"))
for fif in (1, 4):
    sc = rt.Scene(mesh, frames_in_flight=fif)
    static = rt.flycam(W, H, 0, 0, 20)
    for _ in range(40):  # warm the GPU and the maps
        sc.render_async(static, rt.DEFAULT_LIGHTS, W, H, mode=m)
        sc.synchronize()
    for rep in range(reps):
        for cam_kind in ("static", "moving", "stopped"):
            # stopped: 20 untimed moving frames, then the timed frames hold the path's last pose (the camera stops)
            path = rt.CameraPath(W, H) if cam_kind != "static" else None
            for _ in range(10 if cam_kind != "stopped" else 20):  # the path's first poses (untimed)
                sc.render_async(path.next() if path else static, rt.DEFAULT_LIGHTS, W, H, mode=m)
                sc.synchronize()
            if cam_kind == "stopped":
                hold = path.camera()
                cams = [hold] * frames
            else:
                cams = path.take(frames) if path else [static] * frames
            k_ms = tr_ms = el = 0.0
            torch.cuda.synchronize()
            for c in cams:
                if policy == "exact":  # record this pose's own costs first (untimed)
                    sc.render_async(c, rt.DEFAULT_LIGHTS, W, H, mode=m)
                    sc.synchronize()
                t0 = time.perf_counter()
                sc.render_async(c, rt.DEFAULT_LIGHTS, W, H, mode=m)
                st = sc.synchronize()
                el += time.perf_counter() - t0
                k_ms += st["kernel_ms"]
                tr_ms += st["trace_kernel_ms"]
            rec = {"lib": lib, "policy": policy, "scene": scene, "mode": mode, "fif": fif, "rep": rep, "camera": cam_kind,
                   "frames": frames, "mrays_per_s_one_at_a_time": round(W * H * frames / el / 1e6, 1),
                   "frame_ms_wall": round(el / frames * 1e3, 4), "kernel_ms": round(tr_ms / frames, 4),
                   "frame_ms_events": round(k_ms / frames, 4)}
            if hasattr(rt.lib(), "rt_debug_lpt_stats"):
                rec["lpt"] = sc.lpt_stats()
            print(json.dumps(rec), flush=True)
    del sc
