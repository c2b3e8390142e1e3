#!/bin/bash
export RTAMD_DEBUG_KNOBS=1  # the library reads RT_* knobs only when asked (rt_debug_env_knobs)
# A/B of the longest-first dispatch order (variant bit 131072 = default order) on the bench configs,
# one frame at a time and 4 in flight; plus wave timelines with LPT on. Output: gpurun_out/<tag>/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-ab_lpt}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -12 $OUT/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for cfg in "soup primary" "bunny primary" "bunny full" "soup full"; do
  set -- $cfg
  for fif in 1 4; do
    for v in ${VARIANTS:-0 131072}; do
      RT_KERNEL_VARIANT=$v timeout -k 10 300 python bench.py --scene $1 --mode $2 --frames-in-flight $fif --steps 50 --warmup 5 \
          --no-cpu --no-e2e --no-extra > $OUT/b_$1_$2_f${fif}_v$v.json 2> $OUT/b_$1_$2_f${fif}_v$v.err || exit $?
      python3 -c "import json; d=json.load(open('$OUT/b_$1_$2_f${fif}_v$v.json')); print('$1 $2 fif$fif v$v', d['value'], d['ms_per_step'], d['config']['kernel_ms_one_frame_alone'])"
    done
  done
done
for sv in "soup primary" "bunny full"; do
  set -- $sv
  timeout -k 10 120 python tools/timeline.py capture $OUT/tl_$1_$2.npz --scene $1 --mode $2 || exit $?
done
# the same configurations with an older build kept under ab_*/ (its own bench.py + library), same box
for old in ${OLD_BUILDS:-}; do
  for cfg in "soup primary" "bunny primary" "bunny full" "soup full"; do
    set -- $cfg
    for fif in 1 4; do
      timeout -k 10 300 python $old/bench.py --scene $1 --mode $2 --frames-in-flight $fif --steps 50 --warmup 5 \
          --no-cpu --no-e2e > $OUT/old_${old}_$1_$2_f${fif}.json 2> $OUT/old_${old}_$1_$2_f${fif}.err || exit $?
      python3 -c "import json; d=json.load(open('$OUT/old_${old}_$1_$2_f${fif}.json')); print('$old $1 $2 fif$fif', d['value'], d['ms_per_step'])"
    done
  done
done
