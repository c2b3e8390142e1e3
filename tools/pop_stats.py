"""Counting run (also the wave-level triangle-stage counts) of the C3 soup / bunny frames (RT_FRAME_STATS) and the raw counters of rt_debug_counters:
how many wave stack pops there are per wave, and how many of them no lane still needed (every lane that
had wanted the entry now has a closest hit nearer than its entry distance) -- the node steps that a
culling test at the pop would save. Usage: python tools/pop_stats.py [soup|bunny ...]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import conftest  # noqa: E402

rt = conftest.rtamd
NAMES = ["node_visits", "tri_tests", "wave_node_fetches", "wave_tri_fetches", "primary_rays", "hits",
         "total_rays", "wave_pops", "wave_pops_cullable", "wave_wide_fetches", "wave_tri_cand", "wave_tri_prebox",
         "wave_tri_inside", "wave_tri_exit_edge1", "wave_tri_exit_edge2",
         "wave_tri_cand_m", "wave_tri_exit_edge1_m", "wave_tri_exit_edge2_m", "wave_tri_inside_m",
         "wave_tri_desc", "wave_tri_cand_desc_m", "wave_tri_accept_outside_entry"]


def main(scenes):
    W, H = 1920, 1080
    for name in scenes:
        if name == "soup":
            mesh, _, _ = rt.soup_mesh(1_000_000, 12345)
        else:
            mesh = rt.Mesh.load_obj(os.path.join(ROOT, "scenes", "bunny.obj"))
        sc = rt.Scene(mesh, device=0)
        cam = rt.flycam(W, H, 0, 0, 20)
        _, face_s, t_s, _ = sc.render(cam, rt.DEFAULT_LIGHTS, W, H, flags=rt.RT_FRAME_STATS, want_hits=True)
        out = sc.counters(24)
        _, face_n, t_n, _ = sc.render(cam, rt.DEFAULT_LIGHTS, W, H, want_hits=True)
        d = {k: out[i] for i, k in enumerate(NAMES)}
        waves = (W // 8) * ((H + 7) // 8)
        d["scene"] = name
        d["waves"] = waves
        # the counting run's frame against the production kernel's (any traversal experiment must not change it)
        d["counting_frame_face_mismatches"] = int((face_s != face_n).sum())
        d["counting_frame_t_mismatches"] = int((t_s.view("u4") != t_n.view("u4")).sum())
        d["pops_per_wave"] = d["wave_pops"] / waves
        d["node_steps_per_wave"] = d["wave_node_fetches"] / waves
        d["cullable_share_of_pops"] = d["wave_pops_cullable"] / max(d["wave_pops"], 1)
        wt = max(d["wave_tri_fetches"], 1)
        d["tri_tests_per_wave"] = d["wave_tri_fetches"] / waves
        d["tri_share_cand"] = d["wave_tri_cand"] / wt  # some lane past the plane-distance stage
        d["tri_share_prebox"] = d["wave_tri_prebox"] / wt  # some candidate's hit point in the grown triangle box
        d["tri_share_inside"] = d["wave_tri_inside"] / wt  # some lane past the edge tests
        d["tri_share_exit_edge1"] = d["wave_tri_exit_edge1"] / wt  # staged edge tests: none left after edge 1
        d["tri_share_exit_edge2"] = d["wave_tri_exit_edge2"] / wt
        # round 4: candidates restricted to the lanes whose ray entered the leaf's box (all leaves / leaves
        # reached by descent only), and whether any lane outside the entry mask ever accepted (must be 0)
        d["tri_share_cand_masked"] = d["wave_tri_cand_m"] / wt
        d["tri_share_exit_edge1_masked"] = d["wave_tri_exit_edge1_m"] / wt
        d["tri_share_exit_edge2_masked"] = d["wave_tri_exit_edge2_m"] / wt
        d["tri_share_inside_masked"] = d["wave_tri_inside_m"] / wt
        d["tri_share_in_descent_leaves"] = d["wave_tri_desc"] / wt
        d["tri_share_cand_descent_masked"] = d["wave_tri_cand_desc_m"] / wt
        print(json.dumps(d), flush=True)


if __name__ == "__main__":
    main(sys.argv[1:] or ["soup", "bunny"])
