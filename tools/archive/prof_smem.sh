#!/bin/bash
export RTAMD_DEBUG_KNOBS=1  # the library reads RT_* knobs only when asked (rt_debug_env_knobs)
# Scalar-memory latency and scalar-cache pressure of the fused PRIMARY kernel (C3, one frame in flight):
# SQ_INST_LEVEL_SMEM / SQ_INSTS_SMEM = mean SMEM latency in cycles; SQC busy / stall counters.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/profsmem
mkdir -p $OUT
i=0
for set in "SQ_INST_LEVEL_SMEM SQ_INSTS_SMEM SQ_INSTS_SMEM_NORM SQ_INST_CYCLES_SMEM SQ_INST_CYCLES_SALU SQ_WAVES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" \
           "SQC_DCACHE_BUSY_CYCLES SQC_TC_STALL SQC_DCACHE_INPUT_VALID_READYB SQC_TC_DATA_READ_REQ SQC_DCACHE_MISSES_DUPLICATE SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_DCACHE_REQ" \
           "SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_LEVEL_WAVES SQ_INSTS_BRANCH"; do
  i=$((i+1))
  for var in ${VARS:-0}; do
    RT_KERNEL_VARIANT=$var timeout -s KILL 90 rocprofv3 --pmc $set -d $OUT/p${i}_v$var -o run --output-format csv -- \
        python3 bench.py --steps 5 --warmup 1 --no-cpu --no-stats --no-extra --no-e2e --frames-in-flight 1 ${BENCH_ARGS:-} > $OUT/p${i}_v$var.json 2> $OUT/p${i}_v$var.err
    rc=$?; echo "pass $i var $var rc=$rc"
    case $rc in 0) ;; *) exit $rc;; esac
  done
done
