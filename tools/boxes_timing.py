"""Box-partition build time, host vs device (rt_scene_opts.box_builder), on the C3 soup and the bunny."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ray-tracing-project_amd"))
import rtamd as rt  # noqa: E402

out = {}
for name in ("soup", "bunny"):
    if name == "soup":
        mesh, _, _ = rt.soup_mesh(1_000_000)
    else:
        mesh = rt.Mesh.load_obj(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "scenes", "bunny.obj"))
    for bb in (rt.RT_BOXES_HOST, rt.RT_BOXES_GPU, rt.RT_BOXES_HOST, rt.RT_BOXES_GPU):
        t0 = time.perf_counter()
        sc = rt.Scene(mesh, box_builder=bb)
        wall = (time.perf_counter() - t0) * 1e3
        i = sc.info()
        out.setdefault(name, []).append({"box_builder": i["box_builder"], "boxes_ms": round(i["boxes_ms"], 2),
                                         "boxes_gpu_ms": round(i["boxes_gpu_ms"], 2), "n_boxes": i["n_ref_boxes"],
                                         "scene_create_ms": round(wall, 1)})
        del sc
print(json.dumps(out, indent=1))
