#!/usr/bin/env python3
"""Where a lone frame's wave time goes: node steps, triangle tests, the rest of a wave
(ray generation, shading, start / end) and idle wave slots.

One frame of the workload is rendered as a counting run with per-wave counts (RT_FRAME_STATS |
RT_FRAME_WAVE_STATS: each logical wave's packet node steps, triangle tests and hit lanes; for FULL the node
steps and triangle tests of each of its four packet phases), then K lone frames of the product kernel with
RT_FRAME_TIMELINE (each wave's start / end on the constant 100 MHz clock, the logical wave it traced). Per
wave, the duration is fitted as  d = a + b * node_steps + c * tri_tests (+ e * hit_lanes)  by least squares
over all waves of the K frames (FULL: node steps and triangle tests of the primary phase and of the three
secondary phases as separate terms), and the frame's summed wave time is split by the fitted terms; idle =
the frame's span x the resident-wave slots it could fill - the summed wave time. Static camera (the frame's
own cost map: the longest-first order the product uses for a frame alone); the timeline frames do not split
waves into sub-waves. One JSON line per workload, and a text summary.

Usage: python tools/wave_breakdown.py [c3|c5|c2] ...
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

rt = bench.load_rtamd()
W, H = 1920, 1080
K = 6
SLOTS = {"c3": 8 * 1024, "c2": 8 * 1024, "c5": 6 * 1024}  # waves per SIMD x 1024 SIMDs (the kernels' occupancy)


def run(cfg):
    full = cfg == "c5"
    if cfg == "c3":
        mesh, _, _ = rt.soup_mesh(1_000_000, 12345)
    else:
        mesh = rt.Mesh.load_obj(os.path.join(ROOT, "scenes", "bunny.obj"))
    m = rt.RT_MODE_FULL if full else rt.RT_MODE_PRIMARY
    sc = rt.Scene(mesh, frames_in_flight=1)
    cam = rt.flycam(W, H, 0, 0, 20)
    for _ in range(30):
        sc.render_async(cam, rt.DEFAULT_LIGHTS, W, H, mode=m)
        sc.synchronize()
    sc.render_async(cam, rt.DEFAULT_LIGHTS, W, H, mode=m, flags=rt.RT_FRAME_STATS | rt.RT_FRAME_WAVE_STATS)
    sc.synchronize()
    ws = sc.wave_stats().astype(np.float64)
    rows, spans, kern = [], [], []
    for _ in range(K):
        sc.render_async(cam, rt.DEFAULT_LIGHTS, W, H, mode=m, flags=rt.RT_FRAME_TIMELINE)
        st = sc.synchronize()
        kern.append(st["trace_kernel_ms"])
        tl = sc.timeline().astype(np.int64)
        r0, r1 = tl[:, 4], tl[:, 5]
        qw = tl[:, 7] & 0x0FFFFFFF
        ok = (r1 > 0) & (qw < len(ws))
        r0, r1, qw = r0[ok], r1[ok], qw[ok]
        dur_us = ((r1 - r0) & 0xFFFFFFFF) / 100.0  # 100 MHz
        spans.append(float(((r1.max() - r0.min()) & 0xFFFFFFFF) / 100.0))
        rows.append((qw, dur_us))
    qw = np.concatenate([r[0] for r in rows])
    d = np.concatenate([r[1] for r in rows])
    X = ws[qw]
    if full:
        names = ["primary_nodes", "secondary_nodes", "primary_tris", "secondary_tris"]
        feats = np.stack([X[:, 0], X[:, 1:4].sum(1), X[:, 4], X[:, 5:8].sum(1)], 1)
    else:
        names = ["node_steps", "tri_tests", "hit_lanes"]
        feats = np.stack([X[:, 0], X[:, 1], X[:, 2]], 1)
    A = np.concatenate([np.ones((len(d), 1)), feats], 1)
    coef, *_ = np.linalg.lstsq(A, d, rcond=None)
    pred = A @ coef
    r2 = 1.0 - ((d - pred) ** 2).sum() / max(((d - d.mean()) ** 2).sum(), 1e-12)
    per_frame = len(d) / K
    tot = d.sum() / K  # wave-us per frame
    parts = {"fixed_per_wave": coef[0] * per_frame}
    for i, n in enumerate(names):
        parts[n] = coef[i + 1] * feats[:, i].sum() / K
    span = float(np.median(spans))
    slots = SLOTS[cfg]
    cap = span * slots
    out = {"workload": cfg.upper(), "frames": K, "waves_per_frame": int(per_frame),
           "frame_span_us": round(span, 1), "kernel_ms_hip_events": round(float(np.median(kern)), 4),
           "wave_slots": slots, "wave_us_per_frame": round(tot, 0),
           "fit": {"intercept_us": round(coef[0], 3), **{f"us_per_{n}": round(c, 5) for n, c in zip(names, coef[1:])},
                   "r2": round(float(r2), 3)},
           "share_of_slot_time": {k: round(v / cap, 4) for k, v in parts.items()},
           "idle_share_of_slot_time": round(1.0 - tot / cap, 4),
           "mean_resident_waves_per_simd": round(tot / span / 1024, 2),
           "wave_us": {"p50": round(float(np.percentile(d, 50)), 1), "p99": round(float(np.percentile(d, 99)), 1),
                       "max": round(float(d.max()), 1)},
           "counts_per_wave": {n: round(float(feats[:, i].mean()), 2) for i, n in enumerate(names)}}
    print(json.dumps(out), flush=True)
    return out


if __name__ == "__main__":
    for c in sys.argv[1:] or ["c3", "c5"]:
        run(c)
