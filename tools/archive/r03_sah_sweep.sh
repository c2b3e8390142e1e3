#!/bin/bash
export RTAMD_DEBUG_KNOBS=1  # the library reads RT_* knobs only when asked (rt_debug_env_knobs)
# Round 3: SBVH traversal-cost constant (RT_SAH_TRAV) and leaf bound (--leaf) re-swept after the triangle
# test got cheaper (staged edge tests, box certificates). One JSON line per run under gpurun_out/<TAG>/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r03_sah}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
for rep in 1 2; do
for scene in soup bunny; do
  for tv in 0.5 0.7 1.0 1.4; do
    for leaf in 0 2 6; do
      [ "$leaf" != 0 ] && [ "$tv" != 0.7 ] && continue
      out=gpurun_out/$TAG/${scene}_t${tv}_l${leaf}_r$rep.json
      RT_SAH_TRAV=$tv timeout -k 10 300 python bench.py --scene $scene --mode primary --leaf $leaf --steps 50 --warmup 5 \
          --no-cpu --no-stats --no-e2e --no-extra > $out 2> ${out%.json}.err
      rc=$?
      python3 -c "import json; d=json.load(open('$out')); print('$scene trav $tv leaf $leaf r$rep', d['value'], d['ms_per_step'], d['config']['kernel_ms_one_frame_alone'], d['config']['bvh_nodes'])" 2>/dev/null || echo "$scene $tv $leaf rc=$rc"
      case $rc in 0) ;; *) exit $rc;; esac
    done
  done
done
done
