#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/fw6
RTAMD_LIB=$PWD/ray-tracing-project_amd/lib/librtamd_fw6.so timeout -k 10 300 python -u -m pytest tests/test_gpu_fullframe.py -m gpu -x -q \
    -p no:cacheprovider --timeout 200 --timeout-method thread -k "matches_oracle and C5 or digests" > gpurun_out/fw6/pytest.log 2>&1
rc=$?; echo "fw6 parity rc=$rc"; tail -1 gpurun_out/fw6/pytest.log; [ $rc -ne 0 ] && exit $rc
TAG=fw6 LIBS="default fw6" CFGS="bunny:full:4 bunny:full:1" REPS=3 bash tools/ablibs.sh
