#!/bin/bash
export RTAMD_DEBUG_KNOBS=1  # the library reads RT_* knobs only when asked (rt_debug_env_knobs)
# A/B of library builds on the FULL configurations (GPU box): LIBS="default fw4 ...", VARIANT env
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/abf
for tag in ${LIBS:-default}; do for sc in ${SCENES:-bunny soup}; do
  if [ "$tag" = default ]; then lib=""; else lib="$PWD/ray-tracing-project_amd/lib/librtamd_$tag.so"; fi
  RTAMD_LIB=$lib RT_KERNEL_VARIANT=${VARIANT:-0} timeout -k 10 300 python bench.py --scene $sc --mode full --steps 20 --warmup 5 --no-cpu --no-stats \
      > gpurun_out/abf/${tag}_$sc.json 2> gpurun_out/abf/${tag}_$sc.err
  rc=$?
  python3 -c "import json; d=json.load(open('gpurun_out/abf/${tag}_$sc.json')); print('$tag $sc', d['value'], 'Mrays/s', d['config']['kernel_ms_per_frame'], 'ms')" 2>/dev/null || echo "$tag $sc rc=$rc"
  case $rc in 124|134|137|139) exit $rc;; esac
done; done
