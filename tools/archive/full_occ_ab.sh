#!/bin/bash
export RTAMD_DEBUG_KNOBS=1  # the library reads RT_* knobs only when asked (rt_debug_env_knobs)
# FULL megakernel occupancy A/B (GPU box): library builds x RT_KERNEL_VARIANT on bunny (C5) and the soup.
#   RUNS="bunny:default:0 bunny:small7:0 bunny:default:8192 soup:default:0 soup:big6:0" bash tools/full_occ_ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/focc
for rep in 1 2; do for run in ${RUNS:-bunny:default:0}; do
  IFS=: read -r scene tag v <<< "$run"
  if [ "$tag" = default ]; then lib=""; else lib="$PWD/ray-tracing-project_amd/lib/librtamd_$tag.so"; fi
  out=gpurun_out/focc/${scene}_${tag}_v${v}_r${rep}.json
  RTAMD_LIB=$lib RT_KERNEL_VARIANT=$v timeout -k 10 300 python bench.py --scene $scene --mode full --steps 20 \
      --warmup 5 --no-cpu --no-stats --no-e2e > $out 2> ${out%.json}.err
  rc=$?
  python3 -c "
import json; d=json.load(open('$out')); c=d['config']
print('%-6s %-8s v%-6s rep$rep %8.1f Mrays/s  kernel %.4f ms/frame' % ('$scene', '$tag', '$v', d['value'], c['kernel_ms_per_frame']))" 2>/dev/null || echo "$scene $tag v$v rc=$rc"
  case $rc in 124|134|137|139) exit $rc;; esac
done; done
