#!/usr/bin/env python3
"""In-kernel clock of the bench workload's render kernel (MI355X_MICROARCH.md "DVFS give-back" item 6): lone
frames rendered with RT_FRAME_TIMELINE after a second of back-to-back frames; per wave
d(s_memtime) / d(s_memrealtime) x 100 MHz, median over the waves of the frames (waves of >= 5 us only, for the
100-MHz clock's resolution). Used by tools/summarize_profile.py as the clock of the issue fractions.

Usage: python tools/kernel_clock.py out.json [--scene soup|bunny] [--mode primary|full] [other bench args ignored]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("out")
ap.add_argument("--scene", default="soup")
ap.add_argument("--mode", default="primary")
a, _ = ap.parse_known_args()
rt = bench.load_rtamd()
W, H = 1920, 1080
mesh = rt.soup_mesh(1_000_000, 12345)[0] if a.scene == "soup" else rt.Mesh.load_obj(os.path.join(ROOT, "scenes", "bunny.obj"))
m = rt.RT_MODE_FULL if a.mode == "full" else rt.RT_MODE_PRIMARY
sc = rt.Scene(mesh, frames_in_flight=4)
cam = rt.flycam(W, H, 0, 0, 20)
t0 = time.perf_counter()
while time.perf_counter() - t0 < 1.0:  # the clock the chip holds under this load
    for _ in range(8):
        sc.render_async(cam, rt.DEFAULT_LIGHTS, W, H, mode=m)
    sc.synchronize()
ghz = []
for _ in range(5):
    sc.render_async(cam, rt.DEFAULT_LIGHTS, W, H, mode=m, flags=rt.RT_FRAME_TIMELINE)
    sc.synchronize()
    tl = sc.timeline().astype(np.int64)
    dt = ((tl[:, 3] << 32) | tl[:, 2]) - ((tl[:, 1] << 32) | tl[:, 0])
    dr = (tl[:, 5] - tl[:, 4]) & 0xFFFFFFFF
    ok = (dr >= 500) & (dt > 0)
    ghz.append(dt[ok] / dr[ok] * 0.1)
g = np.concatenate(ghz)
rec = {"clock_GHz": round(float(np.median(g)), 4), "p10": round(float(np.percentile(g, 10)), 4),
       "p90": round(float(np.percentile(g, 90)), 4), "waves": int(len(g)),
       "what": f"{a.scene} {a.mode} 1920x1080, 5 timeline frames alone after 1 s of frames in flight"}
json.dump(rec, open(a.out, "w"))
print(json.dumps(rec))
