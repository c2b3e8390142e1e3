#!/bin/bash
# C3 with the chunked XCD order at band-sized runs (RT_XCD_RUN blocks per run; 4080 = one contiguous eighth of the
# 32,640 one-wave blocks per XCD, 2040 = two bands, ...): rate with frames in flight and alone, then the L2 hit rate.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp RTAMD_DEBUG_KNOBS=1
OUT=gpurun_out/xcdbands; mkdir -p $OUT
for rep in 1 2; do
  for c in ${RUNS:-64 510 1020 2040 4080}; do
    for f in 4 1; do
      RT_XCD_RUN=$c timeout -k 10 120 python bench.py --steps 40 --warmup 5 --no-cpu --no-side --no-extra --no-e2e --no-stats \
          --frames-in-flight $f > $OUT/c${c}_f${f}_r$rep.json 2> $OUT/c${c}_f${f}_r$rep.err || exit 1
      python3 -c "import json;d=json.loads(open('$OUT/c${c}_f${f}_r$rep.json').read().strip().splitlines()[-1]);c=d['config'];print('run $c fif $f r$rep', d['value'], d['ms_per_step'], c['kernel_ms_one_frame_alone'])"
    done
  done
done
for c in ${PMC_RUNS:-64 4080}; do
  RT_XCD_RUN=$c timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $OUT/pmc_c$c -o run --output-format csv -- \
      python bench.py --steps 10 --warmup 2 --no-cpu --no-side --no-extra --no-e2e --no-stats > $OUT/pmc_c$c.log 2>&1 || exit 1
done
