#!/bin/bash
export RTAMD_DEBUG_KNOBS=1  # the library reads RT_* knobs only when asked (rt_debug_env_knobs)
# A/B matrix on the bench workload (GPU box): library builds x RT_KERNEL_VARIANT values, one frame in
# flight (isolated kernels) with the counting run, so node/triangle counts come with each time.
#   RUNS="default:0 default:512 order:0" FIF=1 bash tools/ab_matrix.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/abm
for rep in 1 2; do for run in ${RUNS:-default:0}; do
  tag=${run%%:*}; v=${run#*:}
  if [ "$tag" = default ]; then lib=""; else lib="$PWD/ray-tracing-project_amd/lib/librtamd_$tag.so"; fi
  out=gpurun_out/abm/${tag}_v${v}_r${rep}.json
  RTAMD_LIB=$lib RT_KERNEL_VARIANT=$v timeout -k 10 300 python bench.py --steps 40 --warmup 5 --no-cpu --no-e2e \
      --frames-in-flight ${FIF:-1} ${BENCH_EXTRA:-} > $out 2> ${out%.json}.err
  rc=$?
  python3 -c "
import json; d=json.load(open('$out')); c=d['config']; r=d['roofline']
print('%-8s v%-5s rep$rep %8.1f Mrays/s  frame %.4f ms  trace %.4f ms  nodes %.2f tris %.2f wfetchB %.1f' % ('$tag', '$v', d['value'], c['kernel_ms_per_frame'], c['trace_kernel_ms'], r['n_node'], r['n_tri'], r['wave_fetch_bytes_per_ray']))" 2>/dev/null || echo "$tag v$v rc=$rc"
  case $rc in 124|134|137|139) exit $rc;; esac
done; done
