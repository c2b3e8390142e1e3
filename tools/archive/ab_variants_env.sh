#!/bin/bash
export RTAMD_DEBUG_KNOBS=1  # the library reads RT_* knobs only when asked (rt_debug_env_knobs)
# A/B of kernel variants (RT_KERNEL_VARIANT values) and library builds on bench workloads, interleaved
# over REPS rounds. VARS="0 1048576"; LIBS="default dual6"; CFGS="soup:primary:1 ..." (scene:mode:fif).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-abv}
mkdir -p gpurun_out/$TAG
for rep in $(seq 1 ${REPS:-2}); do
for cfg in ${CFGS:-soup:primary:1 soup:primary:4}; do
  IFS=: read scene mode fif <<< "$cfg"
  for tag in ${LIBS:-default}; do
  for var in ${VARS:-0}; do
    if [ "$tag" = default ]; then lib=""; else lib="$PWD/ray-tracing-project_amd/lib/librtamd_$tag.so"; fi
    out=gpurun_out/$TAG/${tag}_v${var}_${scene}_${mode}_f${fif}_r$rep.json
    RT_KERNEL_VARIANT=$var RTAMD_LIB=$lib timeout -k 10 300 python bench.py --scene $scene --mode $mode --frames-in-flight $fif \
        --steps ${STEPS:-50} --warmup 5 --no-cpu --no-stats --no-e2e --no-extra > $out 2> ${out%.json}.err
    rc=$?
    python3 -c "import json; d=json.load(open('$out')); print('$tag v$var $scene $mode fif$fif r$rep', d['value'], d['ms_per_step'], d['config']['kernel_ms_one_frame_alone'])" 2>/dev/null || echo "$tag v$var rc=$rc"
    case $rc in 0) ;; *) exit $rc;; esac
  done
  done
done
done
