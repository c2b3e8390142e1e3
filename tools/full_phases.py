#!/usr/bin/env python3
"""The FULL megakernel's packet walks by phase, from the counting run (RT_FRAME_STATS,
rt_debug_counters slots ST_PW .. ST_PH, csrc/rt_kernels.h): per phase (primary, shadows of the primary hits,
reflection, shadows of the reflection hits) the wave-level walks, the mean active lanes at a walk's entry, node
steps and triangle tests (per walk and as a share of the frame's), and the secondary phases' node steps by the
walk's active lanes (1-8, 9-16, 17-32, 33-48, 49-64). One JSON line per workload.

Usage: python tools/full_phases.py [bunny|soup] ...   (1920x1080 FULL, eye (0,0,1); bunny also at the moving pose)
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

rt = bench.load_rtamd()
ST_HLT = 45
ST_PW = ST_HLT + 3
ST_PL, ST_PS, ST_PT, ST_PH = ST_PW + 4, ST_PW + 8, ST_PW + 12, ST_PW + 16
PHASES = ["primary", "shadow0", "reflection", "shadow1"]
W, H = 1920, 1080
for scene in sys.argv[1:] or ["bunny"]:
    if scene == "soup":
        mesh, _, _ = rt.soup_mesh(1_000_000, 12345)
    else:
        mesh = rt.Mesh.load_obj(os.path.join(ROOT, "scenes", scene + ".obj"))
    sc = rt.Scene(mesh, frames_in_flight=1)
    poses = [("eye (0,0,1)", rt.flycam(W, H, 0, 0, 20))]
    if scene == "bunny":
        p = rt.CameraPath(W, H)
        p.take(bench.MOVE_POSE)
        poses.append((f"moving pose {bench.MOVE_POSE}", p.camera()))
    for name, cam in poses:
        sc.render_async(cam, rt.DEFAULT_LIGHTS, W, H, mode=rt.RT_MODE_FULL, flags=rt.RT_FRAME_STATS)
        st = sc.synchronize()
        c = sc.counters(80)
        tot_steps = sum(c[ST_PS + p] for p in range(4)) or 1
        tot_tris = sum(c[ST_PT + p] for p in range(4)) or 1
        out = {"scene": scene, "pose": name, "frame": f"{W}x{H}", "rays": st["total_rays"], "phases": {}}
        for p, ph in enumerate(PHASES):
            w = c[ST_PW + p]
            out["phases"][ph] = {"walks": w, "mean_active_lanes": round(c[ST_PL + p] / max(w, 1), 2),
                                 "node_steps": c[ST_PS + p], "node_steps_per_walk": round(c[ST_PS + p] / max(w, 1), 1),
                                 "tri_tests": c[ST_PT + p], "share_of_node_steps": round(c[ST_PS + p] / tot_steps, 4),
                                 "share_of_tri_tests": round(c[ST_PT + p] / tot_tris, 4)}
        hist = [c[ST_PH + b] for b in range(5)]
        hs = sum(hist) or 1
        out["secondary_node_steps_by_active_lanes"] = {k: round(v / hs, 4) for k, v in
                                                       zip(["1-8", "9-16", "17-32", "33-48", "49-64"], hist)}
        sec_lanes = sum(c[ST_PL + p] for p in (1, 2, 3)) / max(sum(c[ST_PW + p] for p in (1, 2, 3)), 1)
        out["secondary_mean_active_lanes"] = round(sec_lanes, 2)
        print(json.dumps(out), flush=True)
    del sc
