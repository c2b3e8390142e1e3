#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pf45
for tag in pf4 pf5; do
  RTAMD_LIB=$PWD/ray-tracing-project_amd/lib/librtamd_$tag.so timeout -k 10 300 python -u -m pytest tests/test_gpu_fullframe.py -m gpu -x -q \
      -p no:cacheprovider --timeout 200 --timeout-method thread -k "matches_oracle and (C2 or C3 or C5)" > gpurun_out/pf45/pytest_$tag.log 2>&1
  rc=$?; echo "$tag parity rc=$rc"; tail -1 gpurun_out/pf45/pytest_$tag.log; [ $rc -ne 0 ] && exit $rc
done
TAG=pf45 LIBS="default pf4 pf5" CFGS="soup:primary:1 soup:primary:4 bunny:full:4" REPS=2 bash tools/ablibs.sh
