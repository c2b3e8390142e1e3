"""Child process of test_variants_library_renders_identical_bits (tests/test_gpu_parity.py): loads the
library named by RTAMD_LIB (lib/librtamd_variants.so: the product kernels plus the A/B kernels of
rt_variants.hip) and renders, for every A/B variant, bunny (PRIMARY + FULL, 1080p) and the 1M soup (FULL
640x360, PRIMARY 1000x563) with the default kernels and with the variant. Prints one JSON line:
{variant name: [differing cases]}. Not a test module (no test_ functions); needs a GPU."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import conftest  # noqa: E402  (loads ray-tracing-project_amd/rtamd.py, honouring RTAMD_LIB)
from conftest import scene_path  # noqa: E402
from test_gpu_parity import VARIANTS_LIB, variant_frames_identical  # noqa: E402


def main():
    rt = conftest.rtamd
    assert os.path.basename(rt.LIB_PATH).startswith("librtamd_variants"), rt.LIB_PATH
    # host SBVH scenes: they also carry the quantised 4-wide tree the W4 variant walks (the device builders
    # build the binary tree only, and a variant without its tree would render with the default kernels)
    bunny = rt.Scene(rt.Mesh.load_obj(scene_path("bunny.obj")), builder=rt.RT_BUILDER_SBVH)
    mesh, _, _ = rt.soup_mesh(1_000_000)
    soup = rt.Scene(mesh, builder=rt.RT_BUILDER_SBVH)
    out = {}
    for name, bits in sorted(VARIANTS_LIB.items()):
        out[name] = [list(map(int, c)) for c in variant_frames_identical(rt, (bunny, soup), bits)]
        print(f"{name}: {'identical' if not out[name] else out[name]}", file=sys.stderr, flush=True)
    # the FULL stage pipeline (variant 16) sizes its ray lists for whole frames: a sharded frame is refused
    # with an error, never rendered wrong
    prev = rt.set_variant(16)
    try:
        cam = rt.flycam(256, 256, 0, 0, 20)
        try:
            bunny.render(cam, rt.DEFAULT_LIGHTS, 256, 256, mode=rt.RT_MODE_FULL, shard=(0, 2))
            out["_pipeline_shard_refused"] = [[0]]
        except rt.RTError as e:
            out["_pipeline_shard_refused"] = [] if "whole frames only" in str(e) else [[1]]
    finally:
        rt.set_variant(prev)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
