#!/usr/bin/env python3
"""Where a lone frame's tail comes from: wave start / end times of the product's lone frames with the split
(RT_TIMELINE_SPLIT=1, debug knob: timeline frames keep the longest-first split of the costliest waves into
16-lane sub-waves, as the product's lone frames do).

Per frame (RT_FRAME_TIMELINE, 100 MHz clock): the span, resident waves over time (in 10 slices of the span), and
the waves that end in the last 10% of the span -- how many, how many of them are sub-waves, when they started
(share of the span) and how long they ran. One JSON line per workload and camera.

Usage: RTAMD_DEBUG_KNOBS=1 RT_TIMELINE_SPLIT=1 python tools/tail_probe.py [c5|c2|c3] [static|moving]
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


def run(cfg, camera):
    full = cfg == "c5"
    mesh = rt.soup_mesh(1_000_000, 12345)[0] if cfg == "c3" else rt.Mesh.load_obj(os.path.join(ROOT, "scenes", "bunny.obj"))
    m = rt.RT_MODE_FULL if full else rt.RT_MODE_PRIMARY
    sc = rt.Scene(mesh, frames_in_flight=1)
    path = rt.CameraPath(W, H) if camera == "moving" else None
    static = rt.flycam(W, H, 0, 0, 20)
    for _ in range(30):
        sc.render_async(path.next() if path else static, rt.DEFAULT_LIGHTS, W, H, mode=m)
        sc.synchronize()
    recs = []
    for _ in range(K):
        sc.render_async(path.next() if path else static, rt.DEFAULT_LIGHTS, W, H, mode=m, flags=rt.RT_FRAME_TIMELINE)
        st = sc.synchronize()
        tl = sc.timeline().astype(np.int64)
        r0, r1 = tl[:, 4], tl[:, 5]
        ok = r1 > 0
        idx = np.nonzero(ok)[0]
        n_blocks = int(idx.max()) + 1  # (the buffer holds 2 x the waves under RT_TIMELINE_SPLIT; every launched block writes)
        base = r0[ok].min()
        s = ((r0[ok] - base) & 0xFFFFFFFF) / 100.0
        e = ((r1[ok] - base) & 0xFFFFFFFF) / 100.0
        span = float(e.max())
        waves = 4 * ((W + 15) // 16) * ((H + 15) // 16)  # one-wave blocks of the 16x16 tiles
        split_blocks = n_blocks - waves  # 3 x split_k extra blocks; the first 4 x split_k blocks are sub-waves
        sub = idx < 4 * (split_blocks // 3) if split_blocks > 0 else np.zeros(len(idx), bool)
        sl = np.linspace(0, span, 11)
        resident = [float(((s < sl[i + 1]) & (e > sl[i])).sum()) / 1024 for i in range(10)]  # per SIMD, slice overlap
        late = e > 0.9 * span
        d = e - s
        recs.append({"kernel_ms": st["trace_kernel_ms"], "span_us": span, "blocks": int(n_blocks),
                     "split_k": int(split_blocks // 3), "resident_per_simd_by_tenth": [round(x, 2) for x in resident],
                     "late_waves": int(late.sum()), "late_sub_waves": int((late & sub).sum()),
                     "late_start_share_p50": float(np.median(s[late]) / span) if late.any() else None,
                     "late_start_share_min": float(s[late].min() / span) if late.any() else None,
                     "late_dur_us_p50": float(np.median(d[late])) if late.any() else None,
                     "late_dur_us_max": float(d[late].max()) if late.any() else None,
                     "dur_us_p50": float(np.median(d)), "dur_us_p99": float(np.percentile(d, 99)),
                     "sub_dur_us_p50": float(np.median(d[sub])) if sub.any() else None,
                     "sub_dur_us_max": float(d[sub].max()) if sub.any() else None,
                     "last_start_us": float(s.max())})
    out = {"workload": cfg.upper(), "camera": camera, "frames": K}
    for k in recs[0]:
        v = [r[k] for r in recs]
        if isinstance(v[0], list):
            out[k] = [round(float(np.median([x[i] for x in v])), 2) for i in range(len(v[0]))]
        elif v[0] is None:
            out[k] = None
        else:
            out[k] = round(float(np.median(v)), 4)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c5"
    cams = sys.argv[2:] or ["static", "moving"]
    for c in cams:
        run(cfg, c)
