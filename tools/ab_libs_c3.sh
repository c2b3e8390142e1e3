#!/bin/bash
# C3 bench line per library build (lib/librtamd_<tag>.so; "default" = lib/librtamd.so), interleaved reps:
# value, ms per step, kernel ms per frame with frames in flight, one frame alone.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-ab_libs}; mkdir -p $OUT
for rep in $(seq 1 ${REPS:-2}); do
  for tag in ${LIBS:-default}; do
    if [ "$tag" = default ]; then lib=""; else lib="$PWD/ray-tracing-project_amd/lib/librtamd_$tag.so"; fi
    RTAMD_LIB=$lib timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu --no-side --no-extra ${BENCH_EXTRA:-} \
        > $OUT/${tag}_r$rep.json 2> $OUT/${tag}_r$rep.err
    rc=$?
    python3 -c "
import json;d=json.loads(open('$OUT/${tag}_r$rep.json').read().strip().splitlines()[-1]);c=d['config']
print('$tag r$rep', d['value'], d['ms_per_step'], c['kernel_ms_per_frame'], c['kernel_ms_one_frame_alone'])" || echo "$tag r$rep rc=$rc"
    case $rc in 0) ;; *) exit $rc;; esac
  done
done
