#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/cert
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/cert/pytest.log 2>&1
rc=$?; tail -12 gpurun_out/cert/pytest.log; [ $rc -ne 0 ] && exit $rc
TAG=cert LIBS="default nocert" CFGS="soup:primary:1 soup:primary:4 bunny:primary:4 bunny:full:4 soup:full:4" REPS=2 bash tools/ablibs.sh
