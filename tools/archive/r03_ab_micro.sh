#!/bin/bash
# Round 3: GPU suite on the default build, then A/B of the node-step / triangle micro-optimisations
# (librtamd_base = all off; noclip0 / inreg0 = one off) on C3 and C2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r03_micro}
mkdir -p $OUT
export TMPDIR=/tmp
hard() { case $1 in 124|134|137|139) echo "hard failure ($1): stopping"; exit $1;; esac; }
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
  rc=$?; echo "suite rc=$rc"; tail -4 $OUT/pytest_gpu.log; hard $rc; [ $rc -ne 0 ] && exit $rc
fi
TAG=${TAG:-r03_micro} REPS=${REPS:-2} LIBS="${LIBS:-default base noclip0 inreg0}" CFGS="${CFGS:-soup:primary:4 soup:primary:1 bunny:primary:4}" \
    STEPS=${STEPS:-50} bash tools/ablibs.sh
