"""Packet -> per-lane hybrid traversal model from the counting run (C3 and C2 frames).

The counting traversal (rt_kernels.h traverse<STATS>) records, per wave:
  * how many lanes entered each node step / leaf visit (histogram: 0, 1, 2-3, 4-7, 8-15, 16-31, 32-64 lanes);
  * for thresholds k = 4, 8, 16: the node steps / triangle tests the packet spends in "switched regions"
    (subtrees entered by fewer than k lanes), and what walking those regions one ray per lane would cost
    (per region, the maximum over the wave's lanes of the steps / tests whose node that lane entered).

The hybrid's per-wave work = packet work outside the regions + the per-lane maxima inside them. Instructions
are priced with the per-step costs measured on the product kernels: a packet node step
~24 VALU + ~20 SALU + ~3.5 SMEM (C3 counters: 5,075 VALU, 2,151 SALU, 351 SMEM per wave over 100.5 steps and
19.4 triangle tests), a packet triangle test ~100 VALU + 1 SMEM; a per-lane node step pays the same 12 FMA
box tests plus the per-lane decision and stack (~34 VALU, the VGPR-stack loop's count) and four vector loads
of the 64-B record instead of one scalar load; a per-lane triangle test the same ~100 VALU plus four vector
loads. Usage (GPU box): python tools/hybrid_model.py [soup bunny bunny:full]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import conftest  # noqa: E402

rt = conftest.rtamd
ST_WNODE, ST_WTRI, ST_NODE, ST_TRI, ST_RAYS = 2, 3, 0, 1, 4
ST_HN0 = 22
ST_HL0, ST_HPN = ST_HN0 + 7, ST_HN0 + 14
ST_HPT, ST_HLN, ST_HLT = ST_HPN + 3, ST_HPN + 6, ST_HPN + 9
KS = [4, 8, 16]
BINS = ["0", "1", "2-3", "4-7", "8-15", "16-31", "32-64"]
# per-step instruction prices (see the docstring)
P_NODE_VALU, P_NODE_SALU, P_NODE_SMEM = 24.0, 20.0, 3.5
P_TRI_VALU, P_TRI_SMEM = 100.0, 1.0
L_NODE_VALU, L_NODE_VMEM = 34.0, 4.0
L_TRI_VALU, L_TRI_VMEM = 100.0, 4.0


def main(scenes):
    W, H = 1920, 1080
    out = []
    for spec in scenes:
        name, _, mode = spec.partition(":")  # e.g. bunny:full -- every phase of the FULL megakernel counted together
        if name == "soup":
            mesh, _, _ = rt.soup_mesh(1_000_000, 12345)
        else:
            mesh = rt.Mesh.load_obj(os.path.join(ROOT, "scenes", "bunny.obj"))
        sc = rt.Scene(mesh, device=0)
        cam = rt.flycam(W, H, 0, 0, 20)
        sc.render(cam, rt.DEFAULT_LIGHTS, W, H, flags=rt.RT_FRAME_STATS,
                  **({"mode": rt.RT_MODE_FULL} if mode == "full" else {}))
        c = sc.counters(64)
        waves = (W // 8) * ((H + 7) // 8)
        wn, wt = c[ST_WNODE], c[ST_WTRI]
        d = {"scene": spec, "waves": waves, "node_steps_per_wave": wn / waves, "tri_tests_per_wave": wt / waves,
             "node_visits_per_ray": c[ST_NODE] / c[ST_RAYS], "tri_tests_per_ray": c[ST_TRI] / c[ST_RAYS],
             "node_lanes_hist": {b: c[ST_HN0 + i] / max(wn, 1) for i, b in enumerate(BINS)},
             "leaf_lanes_hist": {b: c[ST_HL0 + i] / max(sum(c[ST_HL0:ST_HL0 + 7]), 1) for i, b in enumerate(BINS)}}
        base_valu = wn * P_NODE_VALU + wt * P_TRI_VALU
        base_mem = wn * P_NODE_SMEM + wt * P_TRI_SMEM
        for i, k in enumerate(KS):
            pn, pt, ln, lt = c[ST_HPN + i], c[ST_HPT + i], c[ST_HLN + i], c[ST_HLT + i]
            valu = (wn - pn) * P_NODE_VALU + (wt - pt) * P_TRI_VALU + ln * L_NODE_VALU + lt * L_TRI_VALU
            mem = (wn - pn) * P_NODE_SMEM + (wt - pt) * P_TRI_SMEM + ln * L_NODE_VMEM + lt * L_TRI_VMEM
            d[f"k{k}"] = {
                "packet_node_steps_in_regions_share": pn / max(wn, 1),
                "packet_tri_tests_in_regions_share": pt / max(wt, 1),
                "per_lane_node_steps_per_wave": ln / waves, "per_lane_tri_tests_per_wave": lt / waves,
                "hybrid_node_steps_per_wave": (wn - pn + ln) / waves,
                "hybrid_tri_tests_per_wave": (wt - pt + lt) / waves,
                "predicted_valu_change": valu / base_valu - 1.0,
                "predicted_valu_plus_mem_change": (valu + mem) / (base_valu + base_mem) - 1.0,
                "predicted_salu_change": -(pn * P_NODE_SALU) / max(wn * P_NODE_SALU, 1.0),
            }
        out.append(d)
        print(json.dumps(d), flush=True)
    return out


if __name__ == "__main__":
    main(sys.argv[1:] or ["soup", "bunny"])
