#!/bin/bash
# A/B of library builds (make ablib TAG=...) on the bench workload (GPU box). LIBS="default noslp ..."
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
for rep in 1 2; do
for tag in ${LIBS:-default}; do
  if [ "$tag" = default ]; then lib=""; else lib="$PWD/ray-tracing-project_amd/lib/librtamd_$tag.so"; fi
  RTAMD_LIB=$lib timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu --no-stats ${BENCH_EXTRA:-} \
      > gpurun_out/ab/$tag.json 2> gpurun_out/ab/$tag.err
  rc=$?
  python3 -c "import json; d=json.load(open('gpurun_out/ab/$tag.json')); print('$tag', d['value'], 'Mrays/s', d['config']['kernel_ms_per_frame'], 'ms', d['config'].get('trace_kernel_ms'))" 2>/dev/null || echo "$tag rc=$rc"
  case $rc in 124|134|137|139) exit $rc;; esac
done
done
