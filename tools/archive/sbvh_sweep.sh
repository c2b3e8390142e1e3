#!/bin/bash
export RTAMD_DEBUG_KNOBS=1  # the library reads RT_* knobs only when asked (rt_debug_env_knobs)
# SBVH parameter sweep on the C3 soup (bench.py builds the scene in-process): combos of
# RT_SBVH (alpha) / RT_SBVH_BUDGET / RT_SAH_TRAV given as "alpha:budget:trav" in COMBOS.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sbsw
for rep in 1 2; do
for combo in ${COMBOS:-0:0.5:0.7 1e-5:0.5:0.7 1e-6:1.0:0.7 1e-7:1.0:0.7 1e-6:1.0:0.5 1e-6:1.0:1.0}; do
  IFS=: read a b tr <<< "$combo"
  for fif in ${FIFS:-4}; do
    out=gpurun_out/sbsw/a${a}_b${b}_t${tr}_f${fif}_r$rep.json
    RT_SBVH=$a RT_SBVH_BUDGET=$b RT_SAH_TRAV=$tr timeout -k 10 300 python bench.py --scene soup --mode primary --frames-in-flight $fif --steps 50 \
        --warmup 5 --no-cpu --no-e2e --no-extra > $out 2> ${out%.json}.err
    rc=$?
    python3 -c "import json; d=json.load(open('$out')); c=d['config']; print('$combo fif$fif r$rep', d['value'], d['ms_per_step'], c['kernel_ms_one_frame_alone'], d['roofline'].get('n_node'), d['roofline'].get('n_tri'))" 2>/dev/null || echo "$combo rc=$rc"
    case $rc in 0) ;; *) exit $rc;; esac
  done
done
done
