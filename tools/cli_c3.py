#!/usr/bin/env python3
"""The drop-in CLI (ray-tracing-project_amd/host/main.cpp, the Flyscene mirror) on the C3 scene (VERDICT r5
item 4): the 1M-triangle soup written as an OBJ + MTL (the soup material), rendered by rt_render_cli at
1920x1080 PRIMARY from eye (0,0,1) with the library's default builders; reports the CLI's scene setup line
(OBJ load + rt_scene_create, and rt_scene_create alone, the builders that ran) and checks its PPM against the
library's own frame of the same OBJ (rt.Mesh.load_obj, same camera) written by rt_write_ppm.

Usage: python tools/cli_c3.py   (GPU box; writes into $TMPDIR)
"""
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

rt = bench.load_rtamd()
W, H = 1920, 1080
v = rt.generate_soup(1_000_000, 12345)
tmp = tempfile.mkdtemp(dir=os.environ.get("TMPDIR", "/tmp"))
obj, mtl = os.path.join(tmp, "soup.obj"), os.path.join(tmp, "soup.mtl")
m = rt.SOUP_MATERIAL
with open(mtl, "w") as f:
    f.write(f"newmtl soup\nKa {m[0]:.9g} {m[1]:.9g} {m[2]:.9g}\nKd {m[3]:.9g} {m[4]:.9g} {m[5]:.9g}\n"
            f"Ks {m[6]:.9g} {m[7]:.9g} {m[8]:.9g}\nNs {m[9]:.9g}\nNi {m[10]:.9g}\nd {m[11]:.9g}\n")
t0 = time.perf_counter()
with open(obj, "w") as f:
    f.write("mtllib soup.mtl\n")
    f.write("".join(f"v {x:.9g} {y:.9g} {z:.9g}\n" for x, y, z in v.tolist()))
    f.write("usemtl soup\n")
    n = len(v) // 3
    f.write("".join(f"f {3 * i + 1} {3 * i + 2} {3 * i + 3}\n" for i in range(n)))
write_s = time.perf_counter() - t0
cli = os.path.join(ROOT, "ray-tracing-project_amd", "lib", "rt_render_cli")
out = os.path.join(tmp, "cli.ppm")
res = {"obj_mb": round(os.path.getsize(obj) / 2**20, 1), "obj_write_s": round(write_s, 1)}
runs = []
for k in range(2):
    t = time.perf_counter()
    log = subprocess.run([cli, obj, str(W), str(H), "--primary", "--dz", "20", "--out", out], check=True,
                         capture_output=True, text=True).stdout
    runs.append({"wall_s": round(time.perf_counter() - t, 2),
                 "setup_line": [x for x in log.splitlines() if x.startswith("scene setup:")][0],
                 "render_line": [x for x in log.splitlines() if "Time it took" in x][0]})
res["cli_runs"] = runs
sc = rt.Scene(rt.Mesh.load_obj(obj))
rgb, _ = sc.render(rt.flycam(W, H, 0, 0, 20), rt.DEFAULT_LIGHTS, W, H)
ref = os.path.join(tmp, "ref.ppm")
rt.write_ppm(ref, rgb)
res["ppm_equal_library_frame"] = open(out, "rb").read() == open(ref, "rb").read()
res["library_builder"] = sc.info()["builder"]
print(json.dumps(res))
for p in (obj, mtl, out, ref):
    os.remove(p)
