#!/bin/bash
export RTAMD_DEBUG_KNOBS=1  # the library reads RT_* knobs only when asked (rt_debug_env_knobs)
# Strong-scaling rehearsal on one GPU: the C4 frame's shard 0 of K (K = 1, 2, 4, 8), i.e. the per-GPU work
# of a K-GPU run without the collective; efficiency = K x shard rate / the whole frame's rate.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/rehearse
for K in ${KS:-1 2 4 8}; do
  for fif in ${FIFS:-4}; do
  for var in ${VARS:-0}; do
  for st in ${STS:-0}; do
    if [ $K = 1 ]; then extra="--frame 3840x2160"; else extra="--rehearse-shards $K"; fi
    o=gpurun_out/rehearse/k${K}_f${fif}_v${var}_s$st
    RT_SUPER_TILE=$st RT_KERNEL_VARIANT=$var timeout -k 10 300 python bench.py $extra --frames-in-flight $fif --steps 100 --warmup 5 --no-cpu --no-stats --no-e2e --no-extra \
        > $o.json 2> $o.err
    rc=$?
    python3 -c "import json; d=json.load(open('$o.json')); c=d['config']; print('K=$K fif=$fif var=$var super=$st', d['value'], d['ms_per_step'], c['kernel_ms_one_frame_alone'], c['host_enqueue_ms_per_frame'])" || echo "K=$K rc=$rc"
    case $rc in 0) ;; *) exit $rc;; esac
  done
  done
  done
done
