"""Register / scratch / occupancy report of the device kernels (compile-only, no GPU).

python tools/kernel_resources.py [-D...] [filter ...]
Compiles csrc/rt_device.hip for gfx950 with the Makefile's flags plus any -D options, and prints
VGPRs, SGPRs, private scratch bytes per lane and occupancy of every kernel whose mangled name contains
one of the filters (default: the render kernels). A scratch size > 0 on a hot kernel is a regression to
look at before measuring anything (the FULL megakernel's allocation is fragile).
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FLAGS = ["-O3", "--offload-arch=gfx950", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math",
         "-fno-slp-vectorize", "-munsafe-fp-atomics", "-w"]


def report(defines, filters):
    src = os.path.join(ROOT, "ray-tracing-project_amd", "csrc", "rt_device.hip")
    cmd = ["/opt/rocm/bin/hipcc"] + FLAGS + defines + ["--cuda-device-only", "-c",
                                                       "-Rpass-analysis=kernel-resource-usage", "-o", os.devnull, src]
    txt = subprocess.run(cmd, capture_output=True, text=True).stderr
    rows, cur = {}, None
    for line in txt.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            rows[cur] = {}
            continue
        for key, pat in (("vgpr", r"VGPRs: (\d+)"), ("sgpr", r"TotalSGPRs: (\d+)"),
                         ("scratch", r"ScratchSize \[bytes/lane\]: (\d+)"), ("occ", r"Occupancy \[waves/SIMD\]: (\d+)")):
            m = re.search(pat, line)
            if m and cur:
                rows[cur][key] = int(m.group(1))
    out = {k: v for k, v in rows.items() if any(f in k for f in filters)}
    for k, v in out.items():
        print(f"{k[:72]:72s} vgpr {v.get('vgpr')} sgpr {v.get('sgpr')} scratch {v.get('scratch')} occ {v.get('occ')}")
    return out


if __name__ == "__main__":
    defs = [a for a in sys.argv[1:] if a.startswith("-D")]
    flt = [a for a in sys.argv[1:] if not a.startswith("-D")] or ["k_render_full", "k_primary_fused", "k_render_depth"]
    report(defs, flt)
