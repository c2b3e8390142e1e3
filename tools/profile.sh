#!/bin/bash
# rocprofv3 evidence for the bench kernel (run on the GPU box): kernel-trace + stats, then separate
# --pmc passes (never combined with tracing domains). Output under gpurun_out/prof/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUTDIR:-gpurun_out/prof}
mkdir -p $OUT
# one frame on the GPU at a time, so that each dispatch's duration is the duration its counters saw
# (clock = GRBM_GUI_ACTIVE / 8 / duration); only the bench frame's launches (no second frame size)
ARGS="${BENCH_ARGS:---steps 20 --warmup 5 --no-cpu --no-extra --no-e2e --no-side --frames-in-flight 1}"
timeout -k 10 120 rocprofv3 -L > $OUT/counters_avail.txt 2>&1 || true
# the in-kernel clock of the same workload (timeline frames: s_memtime / s_memrealtime), the issue fractions' clock
timeout -k 10 120 python3 tools/kernel_clock.py $OUT/kernel_clock.json $ARGS > $OUT/kernel_clock.log 2>&1
rc=$?; echo "kernel clock rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
    python3 bench.py $ARGS > $OUT/trace_bench.json 2> $OUT/trace.err
rc=$?; echo "trace rc=$rc"; [ $rc -ne 0 ] && exit $rc
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD" "TCC_HIT_sum TCC_MISS_sum" \
           ${EXTRA_PMC:-}; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set -d $OUT/pmc$i -o run --output-format csv -- \
      python3 bench.py ${PMC_ARGS:---steps 5 --warmup 1 --no-cpu --no-stats --no-extra --no-e2e --no-side --frames-in-flight 1} > $OUT/pmc$i.json 2> $OUT/pmc$i.err
  rc=$?; echo "pmc$i ($set) rc=$rc"
  case $rc in 124|134|137|139) exit $rc;; esac
done
exit 0
