#!/bin/bash
# A/B of library builds with one frame in flight (isolated kernel timing): LIBS="default prev ..."
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab1
for rep in 1 2; do for tag in ${LIBS:-default}; do
  if [ "$tag" = default ]; then lib=""; else lib="$PWD/ray-tracing-project_amd/lib/librtamd_$tag.so"; fi
  RTAMD_LIB=$lib timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu --no-stats --no-e2e --frames-in-flight 1 ${BENCH_EXTRA:-} \
      > gpurun_out/ab1/$tag.json 2> gpurun_out/ab1/$tag.err
  rc=$?
  python3 -c "import json; d=json.load(open('gpurun_out/ab1/$tag.json')); print('$tag', d['value'], 'Mrays/s', d['config']['kernel_ms_per_frame'], d['config']['trace_kernel_ms'])" 2>/dev/null || echo "$tag rc=$rc"
  case $rc in 124|134|137|139) exit $rc;; esac
done; done
