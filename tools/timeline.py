"""Wave timeline of the render kernel (diagnostics for the one-frame-at-a-time efficiency).

capture (GPU box):  python tools/timeline.py capture OUT.npz [--scene soup|bunny] [--mode primary|full]
    renders the bench frame a few times (one frame on the GPU at a time), then once with
    RT_FRAME_TIMELINE, and saves every wave's start / end clocks, CU and XCD, with its tile position.
analyse (anywhere): python tools/timeline.py analyse OUT.npz
    kernel span from the constant 100 MHz clock, shader clock from s_memtime / s_memrealtime, mean
    resident waves over the span, occupancy over time (ramp / steady / tail), wave-duration spread, and
    what the span would be if every SIMD stayed full (sum of wave time / slots).
With RTAMD_DEBUG_KNOBS=1 RT_TIMELINE_SPLIT=1 the captured frames keep the lone-frame split of their costliest
waves (one record per block: blocks 0 .. 4K-1 are 16-lane sub-waves) and the analysis reports them apart.
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def capture(out, scene, mode, frame, variant=0):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import conftest
    rt = conftest.rtamd
    rt.set_variant(variant)
    W, H = (int(x) for x in frame.split("x"))
    if scene == "soup":
        mesh, _, _ = rt.soup_mesh(1_000_000)
    else:
        mesh = rt.Mesh.load_obj(os.path.join(ROOT, "scenes", "bunny.obj"))
    sc = rt.Scene(mesh, frames_in_flight=1)
    m = rt.RT_MODE_FULL if mode == "full" else rt.RT_MODE_PRIMARY
    cam = rt.flycam(W, H, 0, 0, 20)
    recs = []
    for k in range(8):
        flags = rt.RT_FRAME_TIMELINE if k >= 5 else 0
        sc.render_async(cam, rt.DEFAULT_LIGHTS, W, H, mode=m, flags=flags)
        st = sc.synchronize()
        if flags:
            recs.append((sc.timeline(), st["kernel_ms"]))
    units = ((W + 15) // 16) * ((H + 15) // 16) * 4
    np.savez_compressed(out, tl=np.stack([r[0] for r in recs]), kernel_ms=np.array([r[1] for r in recs]),
                        units=units, W=W, H=H, mode=mode, scene=scene, identity=json.dumps(rt.build_identity()))
    print("captured", out, [r[1] for r in recs])


def analyse(path, slots_per_simd=8):
    d = np.load(path)
    res = []
    for tl, kms in zip(d["tl"], d["kernel_ms"]):
        t0 = tl[:, 0].astype(np.uint64) | (tl[:, 1].astype(np.uint64) << np.uint64(32))
        t1 = tl[:, 2].astype(np.uint64) | (tl[:, 3].astype(np.uint64) << np.uint64(32))
        r0, r1 = tl[:, 4].astype(np.int64), tl[:, 5].astype(np.int64)
        ok = (t1 > t0)
        cyc = (t1 - t0).astype(np.float64)[ok]
        rdt = ((r1 - r0) % (1 << 32)).astype(np.float64)[ok]
        clk = cyc.sum() / (rdt.sum() / 100e6) / 1e9 if rdt.sum() > 0 else float("nan")
        base = r0[ok].min()
        s = (r0[ok] - base) / 100.0  # microseconds (100 MHz)
        e = (r1[ok] - base) / 100.0
        span = e.max()
        # resident waves over time (1 us bins)
        nb = int(np.ceil(span)) + 1
        occ = np.zeros(nb)
        for a, b in zip(s, e):
            ia, ib = int(a), int(b)
            occ[ia:ib + 1] += 1
        slots = 1024 * slots_per_simd
        wave_us = (e - s)
        ideal = wave_us.sum() / slots
        q = np.percentile(wave_us, [5, 50, 95, 99])
        full = np.nonzero(occ >= 0.9 * occ.max())[0]
        hw = tl[ok, 6]
        cu = (tl[ok, 7] >> 28) * 1000 + ((hw >> 13) & 3) * 100 + ((hw >> 12) & 1) * 10 + ((hw >> 8) & 15)
        per_cu = np.bincount(np.unique(cu, return_inverse=True)[1], weights=wave_us)
        # RT_TIMELINE_SPLIT captures: blocks 0 .. 4K-1 are the 16-lane sub-waves of the K costliest waves
        units = int(d["units"]) if "units" in d.files else None
        idx = np.nonzero(ok)[0]
        k_split = (int(ok.sum()) - units) // 3 if units else 0
        sub = idx < 4 * k_split
        top = np.argsort(-(e - s))[:12]
        split_info = {"split_k": k_split} if k_split > 0 else {}
        if k_split > 0:
            split_info.update({
                "sub_wave_us_p50_p95_max": [round(float(x), 1) for x in np.percentile(wave_us[sub], [50, 95, 100])],
                "whole_wave_us_p50_p95_max": [round(float(x), 1) for x in np.percentile(wave_us[~sub], [50, 95, 100])],
                "sub_wave_time_share": round(float(wave_us[sub].sum() / wave_us.sum()), 3),
                "last_sub_wave_end_us": round(float(e[sub].max()), 1),
                "whole_waves_end_us_p50_p99_max": [round(float(x), 1) for x in np.percentile(e[~sub], [50, 99, 100])],
            })
        split_info["longest_blocks"] = [{"block": int(idx[i]), "sub": bool(sub[i]), "start_us": round(float(s[i]), 1),
                                         "us": round(float(e[i] - s[i]), 1)} for i in top]
        res.append({
            "kernel_ms_hip_events": float(kms), "span_us": round(float(span), 1), "waves": int(ok.sum()),
            "shader_clock_GHz": round(float(clk), 3),
            "mean_resident_waves_per_simd": round(float(wave_us.sum() / span / 1024), 2),
            "peak_resident_waves": int(occ.max()),
            "ramp_us_to_90pct": round(float(full[0]) if len(full) else float("nan"), 1),
            "tail_us_below_90pct": round(float(span - full[-1]) if len(full) else float("nan"), 1),
            "tail_us_below_50pct": round(float(span - np.nonzero(occ >= 0.5 * occ.max())[0][-1]), 1),
            "span_if_always_full_us": round(float(ideal), 1),
            "wave_us_p5_p50_p95_p99": [round(float(x), 1) for x in q],
            "cus_seen": int(len(per_cu)), "cu_busy_us_min_mean_max": [round(float(per_cu.min()) / 32, 1),
                                                                     round(float(per_cu.mean()) / 32, 1),
                                                                     round(float(per_cu.max()) / 32, 1)],
            "last_10pct_dispatched_wave_us_mean": round(float(wave_us[int(0.9 * len(wave_us)):].mean()), 1),
            "first_10pct_dispatched_wave_us_mean": round(float(wave_us[: int(0.1 * len(wave_us))].mean()), 1),
            **split_info,
        })
    for r in res:
        print(json.dumps(r))
    return res


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("cmd", choices=["capture", "analyse"])
    ap.add_argument("path")
    ap.add_argument("--scene", default="soup")
    ap.add_argument("--mode", default="primary")
    ap.add_argument("--frame", default="1920x1080")
    ap.add_argument("--variant", type=int, default=0, help="kernel-variant bits (131072: default dispatch order)")
    ap.add_argument("--slots", type=int, default=8, help="resident waves per SIMD the kernel is built for (FULL small: 6)")
    a = ap.parse_args()
    if a.cmd == "capture":
        capture(a.path, a.scene, a.mode, a.frame, a.variant)
    else:
        analyse(a.path, a.slots)
