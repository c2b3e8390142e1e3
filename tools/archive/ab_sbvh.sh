#!/bin/bash
export RTAMD_DEBUG_KNOBS=1  # the library reads RT_* knobs only when asked (rt_debug_env_knobs)
# A/B of the spatial-split BVH (RT_SBVH=<alpha>) against the binned-SAH tree: GPU parity suite with the
# SBVH scenes first, then interleaved bench runs (the scene is built inside each bench process).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sbvh
RT_SBVH=${ALPHA:-1e-5} timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullframe.py \
    -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/sbvh/pytest.log 2>&1
rc=$?; echo "sbvh parity rc=$rc"; tail -3 gpurun_out/sbvh/pytest.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
for cfg in ${CFGS:-soup:primary:4 soup:primary:1 bunny:primary:4 bunny:full:4}; do
  IFS=: read scene mode fif <<< "$cfg"
  for a in 0 ${ALPHA:-1e-5}; do
    out=gpurun_out/sbvh/a${a}_${scene}_${mode}_f${fif}_r$rep.json
    RT_SBVH=$a timeout -k 10 300 python bench.py --scene $scene --mode $mode --frames-in-flight $fif --steps 50 \
        --warmup 5 --no-cpu --no-e2e --no-extra > $out 2> ${out%.json}.err
    rc=$?
    python3 -c "import json; d=json.load(open('$out')); c=d['config']; print('sbvh=$a $scene $mode fif$fif r$rep', d['value'], d['ms_per_step'], c['kernel_ms_one_frame_alone'], d['roofline'].get('n_node'), d['roofline'].get('n_tri'))" 2>/dev/null || echo "a$a rc=$rc"
    case $rc in 0) ;; *) exit $rc;; esac
  done
done
done
