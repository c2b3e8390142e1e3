#!/bin/bash
export RTAMD_DEBUG_KNOBS=1  # the library reads RT_* knobs only when asked (rt_debug_env_knobs)
# Counter comparison of the single-chain fused PRIMARY kernel and the dual-chain variant (C3, one frame
# in flight): issue / wait split, instruction and scalar-cache counts.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/profdual
mkdir -p $OUT
timeout -k 10 120 rocprofv3 -L > $OUT/counters_avail.txt 2>&1 || true
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC" \
           "SQC_ICACHE_REQ SQC_ICACHE_MISSES SQC_DCACHE_REQ SQC_DCACHE_MISSES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_IFETCH SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  for var in 0 1048576; do
    RT_KERNEL_VARIANT=$var timeout -s KILL 90 rocprofv3 --pmc $set -d $OUT/p${i}_v$var -o run --output-format csv -- \
        python3 bench.py --steps 5 --warmup 1 --no-cpu --no-stats --no-extra --no-e2e --frames-in-flight 1 > $OUT/p${i}_v$var.json 2> $OUT/p${i}_v$var.err
    rc=$?; echo "pass $i var $var rc=$rc"
    case $rc in 0) ;; *) exit $rc;; esac
  done
done
