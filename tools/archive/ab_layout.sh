#!/bin/bash
export RTAMD_DEBUG_KNOBS=1  # the library reads RT_* knobs only when asked (rt_debug_env_knobs)
# Node layout A/B: depth-first (default) vs sibling pairs in one 128-B line (RT_NODE_LAYOUT=pairs).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/layout
RT_NODE_LAYOUT=pairs timeout -k 10 300 python -u -m pytest tests/test_gpu_fullframe.py -m gpu -x -q \
    -p no:cacheprovider --timeout 200 --timeout-method thread -k "matches_oracle and (C2 or C3 or C5)" > gpurun_out/layout/pytest.log 2>&1
rc=$?; echo "pairs parity rc=$rc"; tail -1 gpurun_out/layout/pytest.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2 3; do
  for cfg in soup:primary:1 soup:primary:4 bunny:full:4 soup:full:4; do
    IFS=: read scene mode fif <<< "$cfg"
    for lay in dfs pairs; do
      out=gpurun_out/layout/${lay}_${scene}_${mode}_f${fif}_r$rep.json
      RT_NODE_LAYOUT=$lay timeout -k 10 300 python bench.py --scene $scene --mode $mode --frames-in-flight $fif --steps 50 --warmup 5 \
          --no-cpu --no-stats --no-e2e --no-extra > $out 2> ${out%.json}.err
      rc=$?
      python3 -c "import json; d=json.load(open('$out')); print('$lay $scene $mode fif$fif r$rep', d['value'], d['ms_per_step'], d['config']['kernel_ms_one_frame_alone'])" 2>/dev/null || echo "$lay rc=$rc"
      case $rc in 0) ;; *) exit $rc;; esac
    done
  done
done
