#!/bin/bash
export RTAMD_DEBUG_KNOBS=1  # the library reads RT_* knobs only when asked (rt_debug_env_knobs)
# A/B of kernel variants (RT_KERNEL_VARIANT) x library builds, one frame in flight (isolated kernels)
# and the default frames in flight: VARIANTS="0 256" LIBS="default x2w8"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/abv
for rep in 1 2; do for tag in ${LIBS:-default}; do for v in ${VARIANTS:-0}; do for fif in ${FIFS:-1 3}; do
  if [ "$tag" = default ]; then lib=""; else lib="$PWD/ray-tracing-project_amd/lib/librtamd_$tag.so"; fi
  out=gpurun_out/abv/${tag}_v${v}_f${fif}.json
  RTAMD_LIB=$lib RT_KERNEL_VARIANT=$v timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu --no-stats --no-e2e \
      --frames-in-flight $fif ${BENCH_EXTRA:-} > $out 2> ${out%.json}.err
  rc=$?
  python3 -c "import json; d=json.load(open('$out')); print('$tag v$v fif$fif', d['value'], 'Mrays/s', d['config']['kernel_ms_per_frame'], d['config']['trace_kernel_ms'])" 2>/dev/null || echo "$tag v$v rc=$rc"
  case $rc in 124|134|137|139) exit $rc;; esac
done; done; done; done
