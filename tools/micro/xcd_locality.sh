#!/bin/bash
# C3 with the default chunked XCD order vs one contiguous tile range per XCD (variant bit 4): rate with frames in
# flight, then the L2 hit rate and memory waits of k_primary_fused under each order (rocprofv3 --pmc passes).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp RTAMD_DEBUG_KNOBS=1
OUT=gpurun_out/xcdloc; mkdir -p $OUT
for rep in 1 2; do
  for v in 0 4; do
    RT_KERNEL_VARIANT=$v timeout -k 10 120 python bench.py --steps 40 --warmup 5 --no-cpu --no-side --no-extra --no-e2e --no-stats \
        > $OUT/v${v}_r$rep.json 2> $OUT/v${v}_r$rep.err || exit 1
    python3 -c "import json;d=json.loads(open('$OUT/v${v}_r$rep.json').read().strip().splitlines()[-1]);c=d['config'];print('variant $v r$rep', d['value'], d['ms_per_step'], c['kernel_ms_one_frame_alone'])"
  done
done
for v in 0 4; do
  for pmc in "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"; do
    tag=$(echo $pmc | cut -d' ' -f1)
    RT_KERNEL_VARIANT=$v timeout -s KILL 120 rocprofv3 --pmc $pmc -d $OUT/pmc_v${v}_$tag -o run --output-format csv -- \
        python bench.py --steps 10 --warmup 2 --no-cpu --no-side --no-extra --no-e2e --no-stats > $OUT/pmc_v${v}_$tag.log 2>&1 || exit 1
  done
done
