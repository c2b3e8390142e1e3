#!/bin/bash
# Prefetch modes (RT_PF_MODE builds): parity of each build on the full-frame C2/C3/C5 + digest tests, then
# the interleaved A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pfm
for tag in pf1 pf2; do
  RTAMD_LIB=$PWD/ray-tracing-project_amd/lib/librtamd_$tag.so timeout -k 10 300 python -u -m pytest tests/test_gpu_fullframe.py -m gpu -x -q \
      -p no:cacheprovider --timeout 200 --timeout-method thread -k "matches_oracle and (C2 or C3 or C5) or digests" > gpurun_out/pfm/pytest_$tag.log 2>&1
  rc=$?; echo "$tag parity rc=$rc"; tail -2 gpurun_out/pfm/pytest_$tag.log; [ $rc -ne 0 ] && exit $rc
done
TAG=pfm LIBS="default pf1 pf2" CFGS="soup:primary:1 soup:primary:4 bunny:primary:4 bunny:full:4 soup:full:4" REPS=2 bash tools/ablibs.sh
