#!/bin/bash
# A/B of the packed-fma octant slab test (RT_PK_SLAB=1) against the default build: parity first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pk
RTAMD_LIB=$PWD/ray-tracing-project_amd/lib/librtamd_pkslab.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullframe.py \
    -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pk/pytest.log 2>&1
rc=$?; echo "pk parity rc=$rc"; tail -1 gpurun_out/pk/pytest.log; [ $rc -ne 0 ] && exit $rc
TAG=pk LIBS="default pkslab" CFGS="soup:primary:4 bunny:primary:4 soup:primary:1 bunny:full:4 soup:full:4" REPS=3 bash tools/ablibs.sh
