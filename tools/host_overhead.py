"""Host cost of queueing a frame (GPU box): rt_render_async through the Python wrapper vs a raw ctypes call
with prebuilt arguments, on a tiny frame (the GPU never limits), frames in flight 4."""
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import conftest  # noqa: E402

rt = conftest.rtamd
sc = rt.Scene(rt.Mesh.load_obj(os.path.join(ROOT, "scenes", "cube.obj")))
W, H = int(sys.argv[1]) if len(sys.argv) > 1 else 64, int(sys.argv[2]) if len(sys.argv) > 2 else 64
cam = rt.flycam(W, H)
lights = rt.DEFAULT_LIGHTS
L = rt.lib()


def run(fn, n=1024, batch=256):
    fn()
    sc.synchronize()
    t = 0.0
    for _ in range(n // batch):
        t0 = time.perf_counter()
        for _ in range(batch):
            fn()
        t += time.perf_counter() - t0
        sc.synchronize()
    return t / n * 1e6


wrapper = run(lambda: sc.render_async(cam, lights, W, H))
larr = rt.Scene._lights(lights)
fr = rt.Frame(W, H, rt.RT_MODE_PRIMARY, 0, 1, 0, 0)
cp, lp, fp = C.byref(cam), C.cast(larr, C.c_void_p), C.byref(fr)
raw = run(lambda: L.rt_render_async(sc.h, cp, lp, len(lights), fp))
print(f"{W}x{H}: us per rt_render_async: python wrapper {wrapper:.1f}, raw ctypes {raw:.1f}")
