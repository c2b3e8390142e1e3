"""Full-frame oracle fixtures for the benchmark configurations.

For each configuration the pinned CPU oracle (oracle/build/liboracle.so, the restatement of the
reference's traceRay loop, src/flyscene.cpp:299-371) renders EVERY pixel; the fixture keeps
  * SHA-256 of the per-pixel face index (int32), t (float32 bits) and colour (float32 bits) arrays,
  * hit count, the colour sum, and
  * a strided sample of the actual values (every 257th pixel, row-major) for diagnosing a mismatch.
Output: tests/golden/fullframe_digests.json + tests/golden/fullframe_samples.npz.

The GPU tests compare the device frame's digests with these (C4's 8.3 M pixels are checked on the
box this way, without re-running the oracle there); tests/test_oracle_pinning.py recomputes the C2
entry on the CPU so the fixture itself stays tied to the oracle build.

Usage: python tools/gen_fullframe_digests.py [--threads N] [--only C2,C3]
"""
import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402

SOUP_MATERIAL = [0.1, 0.1, 0.1, 0.7, 0.7, 0.7, 0.2, 0.2, 0.2, 16.0, 1.0, 1.0]
SAMPLE_STRIDE = 257

# name: (scene, W, H, mode, max_depth)   eye (0,0,1) = Flycamera translate(0,0,20), default light
CASES = {
    "C2": ("bunny", 1920, 1080, "primary", None),
    "C3": ("soup", 1920, 1080, "primary", None),
    "C5": ("bunny", 1920, 1080, "full", None),
    "C3-full": ("soup", 1920, 1080, "full", None),
    "C4": ("soup", 3840, 2160, "primary", None),
    "bunny-depth3": ("bunny", 1920, 1080, "full", 3),
    # the moving camera (round 6): the pose MOVE_POSE frames along rtamd.CameraPath (the
    # reference's WASD translate per frame, flyscene.cpp:116-127), the pose bench.py's moving_camera checks
    "C3-moving": ("soup", 1920, 1080, "primary", None),
    "C5-moving": ("bunny", 1920, 1080, "full", None),
}
MOVE_POSE = 37  # bench.py MOVE_POSE


def case_camera(key, W, H):
    """The oracle camera of a case: Flycamera translate(0, 0, 20), or for *-moving the path pose, built by the
    product's host-side path helper (pure float32 arithmetic, no device) and copied into the oracle's struct."""
    if not key.endswith("-moving"):
        return O.flycam(W, H, 0, 0, 20), None
    import importlib.util
    spec = importlib.util.spec_from_file_location("rtamd", os.path.join(ROOT, "ray-tracing-project_amd", "rtamd.py"))
    rt = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(rt)
    p = rt.CameraPath(W, H)
    p.take(MOVE_POSE)
    c = p.camera()
    oc = O.Camera()
    for k in range(16):
        oc.view[k] = c.view_matrix[k]
    oc.viewport[:] = list(c.viewport)
    oc.fovy, oc.aspect = c.fovy, c.aspect_ratio
    return oc, [c.view_matrix[12], c.view_matrix[13], c.view_matrix[14]]


def digest(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def frame_record(rgb, face, t):
    face = np.asarray(face, np.int32).reshape(-1)
    t = np.asarray(t, np.float32).reshape(-1)
    rgb = np.asarray(rgb, np.float32).reshape(-1, 3)
    return {"face_sha256": digest(face), "t_sha256": digest(t), "rgb_sha256": digest(rgb),
            "hits": int((face >= 0).sum()), "rgb_sum": float(np.asarray(rgb, np.float64).sum())}


def oracle_scene(name):
    if name == "soup":
        v = O.generate_soup(1_000_000, 12345)
        f = np.arange(3 * 1_000_000, dtype=np.uint32).reshape(-1, 3)
        return O.Scene(O.Mesh.from_arrays(v, f, np.array([SOUP_MATERIAL], np.float32)))
    return O.Scene(O.Mesh.load_obj(os.path.join(ROOT, "scenes", name + ".obj")))


def render_case(sc, cam, W, H, mode, max_depth, threads):
    return sc.render(cam, O.DEFAULT_LIGHTS, W, H, full=(mode == "full"), threads=threads, max_depth=max_depth)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=len(os.sched_getaffinity(0)))
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    only = [x for x in a.only.split(",") if x]
    jpath = os.path.join(ROOT, "tests", "golden", "fullframe_digests.json")
    spath = os.path.join(ROOT, "tests", "golden", "fullframe_samples.npz")
    out = json.load(open(jpath)) if os.path.exists(jpath) else {}
    samples = dict(np.load(spath)) if os.path.exists(spath) else {}
    scenes = {}
    for key, (scene, W, H, mode, depth) in CASES.items():
        if only and key not in only:
            continue
        if scene not in scenes:
            scenes[scene] = oracle_scene(scene)
        t0 = time.time()
        cam, view_t = case_camera(key, W, H)
        rgb, face, t = render_case(scenes[scene], cam, W, H, mode, depth, a.threads)
        dt = time.time() - t0
        rec = frame_record(rgb, face, t)
        rec.update({"scene": scene, "W": W, "H": H, "mode": mode, "max_depth": depth, "eye_dz": 20,
                    "oracle_s": round(dt, 1), "threads": a.threads})
        if view_t is not None:
            rec.update({"camera_path_pose": MOVE_POSE, "view_translation": view_t})
        out[key] = rec
        idx = np.arange(0, W * H, SAMPLE_STRIDE)
        samples[key + "_idx"] = idx.astype(np.int32)
        samples[key + "_face"] = face.reshape(-1)[idx]
        samples[key + "_t"] = t.reshape(-1)[idx]
        samples[key + "_rgb"] = rgb.reshape(-1, 3)[idx]
        print(key, rec, flush=True)
        json.dump(out, open(jpath, "w"), indent=1, sort_keys=True)
        np.savez_compressed(spath, **samples)


if __name__ == "__main__":
    main()
