#!/bin/bash
export RTAMD_DEBUG_KNOBS=1  # the library reads RT_* knobs only when asked (rt_debug_env_knobs)
# SAH cost ratio on the bunny configurations (GPU box): TRAVS="1 0.7" bash tools/sah_bunny.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sahb
for rep in 1 2; do for t in ${TRAVS:-1 0.7}; do for m in primary full; do
  out=gpurun_out/sahb/t${t}_${m}_r${rep}.json
  RT_SAH_TRAV=$t timeout -k 10 300 python bench.py --scene bunny --mode $m --steps 30 --warmup 5 --no-cpu --no-e2e \
      > $out 2> ${out%.json}.err
  rc=$?
  python3 -c "import json; d=json.load(open('$out')); r=d['roofline']; print('trav $t $m rep$rep', d['value'], d['config']['kernel_ms_per_frame'], 'ms n_node', r.get('n_node'), 'n_tri', r.get('n_tri'))" 2>/dev/null || echo "trav $t $m rc=$rc"
  case $rc in 124|134|137|139) exit $rc;; esac
done; done; done
