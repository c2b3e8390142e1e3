#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/dual
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "variants or box_colors or soup_1m" > gpurun_out/dual/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/dual/pytest.log; [ $rc -ne 0 ] && exit $rc
TAG=dual LIBS="default dual6" VARS="0 1048576" CFGS="soup:primary:1 soup:primary:4 bunny:primary:4" REPS=2 bash tools/ab_variants_env.sh
