#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ml
RTAMD_LIB=$PWD/ray-tracing-project_amd/lib/librtamd_ml.so timeout -k 10 300 python -u -m pytest tests/test_gpu_fullframe.py -m gpu -x -q \
    -p no:cacheprovider --timeout 200 --timeout-method thread -k "matches_oracle and C5 or digests or depth" > gpurun_out/ml/pytest.log 2>&1
rc=$?; echo "ml parity rc=$rc"; tail -1 gpurun_out/ml/pytest.log; [ $rc -ne 0 ] && exit $rc
TAG=ml LIBS="default ml" CFGS="bunny:full:4 bunny:full:1 soup:full:4" REPS=3 bash tools/ablibs.sh
