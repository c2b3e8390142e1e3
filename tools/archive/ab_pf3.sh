#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pf3
RTAMD_LIB=$PWD/ray-tracing-project_amd/lib/librtamd_pf3.so timeout -k 10 300 python -u -m pytest tests/test_gpu_fullframe.py -m gpu -x -q \
    -p no:cacheprovider --timeout 200 --timeout-method thread -k "matches_oracle and (C2 or C3 or C5) or digests" > gpurun_out/pf3/pytest.log 2>&1
rc=$?; echo "pf3 parity rc=$rc"; tail -1 gpurun_out/pf3/pytest.log; [ $rc -ne 0 ] && exit $rc
TAG=pf3 LIBS="default pf3" CFGS="soup:primary:1 soup:primary:4 bunny:primary:4 bunny:full:4" REPS=3 bash tools/ablibs.sh
