#!/bin/bash
export RTAMD_DEBUG_KNOBS=1  # the library reads RT_* knobs only when asked (rt_debug_env_knobs)
# Occupancy experiment (diagnostics): the C3 bench with the fused PRIMARY kernel capped at fewer resident
# waves per CU by padding its LDS (RT_LDS_PAD bytes per one-wave block: 160 KiB / (pad + ~1 KiB) blocks
# per CU). Answers how much throughput the kernel gains per extra resident traversal chain.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/occ
mkdir -p $OUT
for pad in 0 4700 5600 9000 12400 19200; do
  for fif in 1 4; do
    RT_LDS_PAD=$pad timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu --no-extra --no-e2e --no-stats \
        --frames-in-flight $fif > $OUT/pad${pad}_fif$fif.json 2> $OUT/pad${pad}_fif$fif.err
    rc=$?
    echo "pad $pad fif $fif rc=$rc $(python3 -c "import json;d=json.load(open('$OUT/pad${pad}_fif$fif.json'));print(d['value'], d['config']['kernel_ms_one_frame_alone'])" 2>/dev/null)"
    case $rc in 0) ;; *) exit $rc;; esac
  done
done
