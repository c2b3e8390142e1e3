"""Probe (GPU box): throughput of back-to-back frames on one stream vs frames alternating over two
scene handles (two streams), to size the gain of keeping two frames in flight."""
import os, sys, time, json
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ray-tracing-project_amd"))
import rtamd as rt
W, H = 1920, 1080
mesh, _, _ = rt.soup_mesh(1_000_000)
a = rt.Scene(mesh); b = rt.Scene(mesh)
cam = rt.flycam(W, H, 0, 0, 20)
def run(scs, n=40):
    for i in range(6): scs[i % len(scs)].render_async(cam, rt.DEFAULT_LIGHTS, W, H)
    for s in scs: s.synchronize()
    t = time.perf_counter()
    for i in range(n): scs[i % len(scs)].render_async(cam, rt.DEFAULT_LIGHTS, W, H)
    for s in scs: s.synchronize()
    return n * W * H / (time.perf_counter() - t) / 1e6
print(json.dumps({"one_stream": run([a]), "two_streams": run([a, b]), "one_stream_again": run([a])}))
