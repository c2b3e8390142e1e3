"""Counting-run diagnostics for the bench workload (GPU box): per-wave node / triangle fetches and
per-ray visits of the current kernel variant (RT_KERNEL_VARIANT). Prints one JSON line."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ray-tracing-project_amd"))
import rtamd as rt  # noqa: E402

W, H = 1920, 1080
n = int(os.environ.get("DIAG_TRIS", "1000000"))
mesh, _, _ = rt.soup_mesh(n)
sc = rt.Scene(mesh, leaf_size=int(os.environ.get("DIAG_LEAF", "0")))
cam = rt.flycam(W, H, 0, 0, 20)
sc.render_async(cam, rt.DEFAULT_LIGHTS, W, H, flags=rt.RT_FRAME_STATS)
st = sc.synchronize()
waves = ((W + 15) // 16) * ((H + 15) // 16) * 4
rays = st["primary_rays"]
out = {"variant": os.environ.get("RT_KERNEL_VARIANT", "0"), "waves": waves,
       "wave_node_fetches_per_wave": st["wave_node_fetches"] / waves,
       "wave_tri_fetches_per_wave": st["wave_tri_fetches"] / waves,
       "node_visits_per_ray": st["node_visits"] / rays, "tri_tests_per_ray": st["tri_tests"] / rays,
       "hit_rate": st["hits"] / rays}
print(json.dumps(out))
