#!/bin/bash
# C3 / C5 lines per BVH leaf bound (bench.py --leaf), interleaved reps: value, ms/step, kernel ms/frame, one frame alone.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/leaf_sweep; mkdir -p $OUT
for rep in 1 2; do
  for cfg in ${CFGS:-c3:3 c3:4 c3:6 c3:8 c5:3 c5:4 c5:6 c5:8}; do
    IFS=: read w leaf <<< "$cfg"
    extra=""; [ "$w" = c5 ] && extra="--scene bunny --mode full"
    timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu --no-side --no-extra --leaf $leaf $extra \
        > $OUT/${w}_${leaf}_r$rep.json 2> $OUT/${w}_${leaf}_r$rep.err || exit $?
    python3 -c "
import json;d=json.loads(open('$OUT/${w}_${leaf}_r$rep.json').read().strip().splitlines()[-1]);c=d['config']
print('$w leaf$leaf r$rep', d['value'], d['ms_per_step'], c['kernel_ms_per_frame'], c['kernel_ms_one_frame_alone'], c.get('bvh_sah_cost',{}).get('sah'))"
  done
done
