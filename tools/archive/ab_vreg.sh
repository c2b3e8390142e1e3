#!/bin/bash
# A/B of the VGPR-copy knobs (RT_TRI_VREG: triangle edge differences; RT_EYE_VREG: primary eye) against the
# default build: parity of the combined build first, then interleaved bench runs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/vreg
RTAMD_LIB=$PWD/ray-tracing-project_amd/lib/librtamd_bothvreg.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullframe.py \
    -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/vreg/pytest.log 2>&1
rc=$?; echo "vreg parity rc=$rc"; tail -1 gpurun_out/vreg/pytest.log; [ $rc -ne 0 ] && exit $rc
TAG=vreg LIBS="default trivreg eyevreg bothvreg" CFGS="soup:primary:4 bunny:primary:4 soup:primary:1 bunny:full:4" REPS=2 bash tools/ablibs.sh
