"""CPU-baseline calibration: the oracle "port" against the reference's own rate.

The survey timed the unmodified reference's calculateMinimumFace + calculateColor loop (PRIMARY) on the
1M-triangle soup, eye z=1, single-threaded, over a 32x18 grid of the 1080p framing: 383 primary rays/s
(survey container: 8-vCPU Intel Xeon, g++ 11.4 -O2). This script times the
oracle (oracle/rt_oracle.c: the same flat boxes, loops and float expressions, with the per-call matrix
work hoisted and the boxes swept by a vectorised intersectBox) on the same grid in this container, one
thread, and writes profiles/cpu_calibration.json. bench.py reports the ratio next to its cpu_baseline.
"""
import json
import os
import platform
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402

REFERENCE_RAYS_PER_S_PER_CORE = 383.0  # BASELINE.md section 2 (survey measurement of the reference)
SOUP_MATERIAL = [0.1, 0.1, 0.1, 0.7, 0.7, 0.7, 0.2, 0.2, 0.2, 16.0, 1.0, 1.0]


def cpu_model():
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True).stdout
        for line in out.splitlines():
            if line.startswith("Model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def main():
    v = O.generate_soup(1_000_000, 12345)
    f = np.arange(3_000_000, dtype=np.uint32).reshape(-1, 3)
    sc = O.Scene(O.Mesh.from_arrays(v, f, np.array([SOUP_MATERIAL], np.float32)))
    W, H = 1920, 1080
    pix = np.array([(i, j) for j in range(0, H, 60) for i in range(0, W, 60)], np.int32)  # 32 x 18
    best = 0.0
    for _ in range(3):
        t0 = time.perf_counter()
        sc.render(O.flycam(W, H, 0, 0, 20), O.DEFAULT_LIGHTS, W, H, pixels=pix, threads=1)
        best = max(best, len(pix) / (time.perf_counter() - t0))
    out = {"port_rays_per_s_per_thread": round(best, 1), "reference_rays_per_s_per_core": REFERENCE_RAYS_PER_S_PER_CORE,
           "port_over_reference": round(best / REFERENCE_RAYS_PER_S_PER_CORE, 2),
           "sample": "32x18 grid (every 60th row and column) of the 1920x1080 framing, 1M-triangle soup, eye z=1, "
                     "PRIMARY, one thread (the survey's reference measurement, BASELINE.md section 2)",
           "host": cpu_model(), "note": "same container image as the survey's reference run; the reference itself "
                                        "cannot be rebuilt here without GL/GLEW/GLFW stand-ins (DESIGN.md section 2)"}
    path = os.path.join(ROOT, "profiles", "cpu_calibration.json")
    json.dump(out, open(path, "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
