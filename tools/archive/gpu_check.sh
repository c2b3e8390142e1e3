#!/bin/bash
# One GPU-box session: parity tests, then a short bench, then a rocprofv3 kernel-trace of the bench.
# Every GPU step has its own time limit; stop at the first crash/timeout (exit 124/134/137/139).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rocm-smi --showproductname > gpurun_out/gpu_info.txt 2>&1 || true
lscpu | grep -E "Model name|^CPU\(s\)" >> gpurun_out/gpu_info.txt 2>&1 || true
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 600 > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
case $rc in 124|134|137|139) echo "GPU step failed hard ($rc)"; exit $rc;; esac
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?
echo "bench rc=$rc"; cat gpurun_out/bench.json
exit $rc
