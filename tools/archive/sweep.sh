#!/bin/bash
export RTAMD_DEBUG_KNOBS=1  # the library reads RT_* knobs only when asked (rt_debug_env_knobs)
# A/B sweep of kernel variants and BVH leaf sizes on the bench workload (GPU box).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sweep
if [ "${RUN_TESTS:-1}" = "1" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 600 > gpurun_out/sweep/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/sweep/pytest_gpu.log
  case $rc in 124|134|137|139) exit $rc;; esac
fi
for cfg in ${SWEEP:-0:4 1:4 2:4 3:4 6:4 7:4 2:2 2:8}; do
  v=${cfg%%:*}; leaf=${cfg##*:}
  RT_KERNEL_VARIANT=$v timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu --leaf $leaf ${BENCH_EXTRA:-} \
      > gpurun_out/sweep/v${v}_l${leaf}.json 2> gpurun_out/sweep/v${v}_l${leaf}.err
  rc=$?
  python3 -c "import json,sys; d=json.load(open('gpurun_out/sweep/v${v}_l${leaf}.json')); r=d['roofline'] or {}; print('variant $v leaf $leaf', d['value'], 'Mrays/s', d['config']['kernel_ms_per_frame'], 'ms', 'nodes', d['config']['bvh_nodes'], 'n_node', r.get('n_node'), 'n_tri', r.get('n_tri'), 'wfetch', r.get('wave_fetch_bytes_per_ray'))" 2>/dev/null || echo "variant $v leaf $leaf rc=$rc"
  case $rc in 124|134|137|139) exit $rc;; esac
done
