#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/osh2
RTAMD_LIB=$PWD/ray-tracing-project_amd/lib/librtamd_osh2.so timeout -k 10 300 python -u -m pytest tests/test_gpu_fullframe.py -m gpu -x -q \
    -p no:cacheprovider --timeout 200 --timeout-method thread -k "matches_oracle and C5 or digests or depth" > gpurun_out/osh2/pytest.log 2>&1
rc=$?; echo "osh2 parity rc=$rc"; tail -1 gpurun_out/osh2/pytest.log; [ $rc -ne 0 ] && exit $rc
TAG=osh2 LIBS="default osh2" CFGS="bunny:full:4 bunny:full:1 soup:full:4" REPS=3 bash tools/ablibs.sh
