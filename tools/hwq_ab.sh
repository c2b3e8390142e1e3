#!/bin/bash
# C3 line with the HIP runtime's hardware-queue count per process (GPU_MAX_HW_QUEUES) and frames in flight, interleaved reps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/hwq; mkdir -p $OUT
for rep in 1 2; do
  for cfg in ${CFGS:-4:4 8:4 8:3 8:2 16:4}; do
    IFS=: read q f <<< "$cfg"
    GPU_MAX_HW_QUEUES=$q timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu --no-side --no-extra --frames-in-flight $f \
        > $OUT/q${q}_f${f}_r$rep.json 2> $OUT/q${q}_f${f}_r$rep.err || exit $?
    python3 -c "
import json;d=json.loads(open('$OUT/q${q}_f${f}_r$rep.json').read().strip().splitlines()[-1]);c=d['config']
print('hwq$q fif$f r$rep', d['value'], d['ms_per_step'], c['kernel_ms_per_frame'], c['kernel_ms_one_frame_alone'])"
  done
done
