#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/fw7
RTAMD_LIB=$PWD/ray-tracing-project_amd/lib/librtamd_fw7.so timeout -k 10 300 python -u -m pytest tests/test_gpu_fullframe.py -m gpu -x -q \
    -p no:cacheprovider --timeout 200 --timeout-method thread -k "matches_oracle and C5" > gpurun_out/fw7/pytest.log 2>&1
rc=$?; echo "fw7 parity rc=$rc"; tail -1 gpurun_out/fw7/pytest.log; [ $rc -ne 0 ] && exit $rc
TAG=fw7 LIBS="fw6 fw7" CFGS="bunny:full:4" REPS=3 bash tools/ablibs.sh
