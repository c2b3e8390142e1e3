"""Regenerates tests/golden/images.npz from the pinned CPU oracle (oracle/build/liboracle.so).

Golden images (float32 RGB + per-pixel face index + t) at the C1 size for the small scenes and a
reduced 320x180 frame of the reference's default scene. Each key is <scene>__<mode>__<W>__<H>_{rgb,face,t}.
Default Flycamera (eye (0,0,2)), default light (-0.5,2,3) white (flyscene.cpp:37).
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402

CASES = [("cube", 256, 256), ("cornell", 256, 256), ("dodgeColorTest", 320, 180)]


def main():
    out = {}
    for name, W, H in CASES:
        mesh = O.Mesh.load_obj(os.path.join(ROOT, "scenes", name + ".obj"))
        sc = O.Scene(mesh)
        cam = O.flycam(W, H)
        for mode in ("primary", "full"):
            rgb, face, t = sc.render(cam, O.DEFAULT_LIGHTS, W, H, full=(mode == "full"), threads=8)
            key = f"{name}__{mode}__{W}__{H}"
            out[key + "_rgb"] = rgb.reshape(H, W, 3)
            out[key + "_face"] = face.reshape(H, W)
            out[key + "_t"] = t.reshape(H, W)
            print(key, "hit %.3f" % (face >= 0).mean())
    np.savez_compressed(os.path.join(ROOT, "tests", "golden", "images.npz"), **out)


if __name__ == "__main__":
    main()
