#!/bin/bash
export RTAMD_DEBUG_KNOBS=1  # the library reads RT_* knobs only when asked (rt_debug_env_knobs)
# SAH cost-ratio sweep (RT_SAH_TRAV) x leaf cap on the bench workload (GPU box). SAH="trav:leaf ..."
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sah
for cfg in ${SAH:-1:4}; do
  t=${cfg%%:*}; leaf=${cfg##*:}
  RT_SAH_TRAV=$t timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu --leaf $leaf \
      > gpurun_out/sah/t${t}_l${leaf}.json 2> gpurun_out/sah/t${t}_l${leaf}.err
  rc=$?
  python3 -c "import json; d=json.load(open('gpurun_out/sah/t${t}_l${leaf}.json')); r=d['roofline']; print('trav $t leaf $leaf', d['value'], d['config']['kernel_ms_per_frame'], 'ms nodes', d['config']['bvh_nodes'], 'n_node', r.get('n_node'), 'n_tri', r.get('n_tri'), 'wfetch', r.get('wave_fetch_bytes_per_ray'))" 2>/dev/null || echo "trav $t leaf $leaf rc=$rc"
  case $rc in 124|134|137|139) exit $rc;; esac
done
