#!/bin/bash
# A/B of one debug knob of the product library on bench workloads (GPU box), interleaved over REPS rounds:
# KNOB=<env name> VALS="<values>" (the literal value "none" leaves the knob unset = the product's behaviour)
# CFGS="scene:mode:frames-in-flight ...". One JSON line per run under gpurun_out/<TAG>/, a summary line each:
# Mrays/s, ms per step, kernel ms of one frame alone.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-knob_ab}
mkdir -p gpurun_out/$TAG
export RTAMD_DEBUG_KNOBS=1
for rep in $(seq 1 ${REPS:-2}); do
for cfg in ${CFGS:-soup:primary:1 soup:primary:4}; do
  IFS=: read scene mode fif <<< "$cfg"
  for v in $VALS; do
    out=gpurun_out/$TAG/${v}_${scene}_${mode}_f${fif}_r$rep.json
    if [ "$v" = none ]; then envs=""; else envs="$KNOB=$v"; fi
    env $envs timeout -k 10 300 python bench.py --scene $scene --mode $mode --frames-in-flight $fif --steps ${STEPS:-40} \
        --warmup 5 --no-cpu --no-stats --no-e2e --no-extra --no-side ${BENCH_EXTRA:-} > $out 2> ${out%.json}.err
    rc=$?
    python3 -c "import json; d=json.loads(open('$out').read().strip().splitlines()[-1]); print('$KNOB=$v $scene $mode fif$fif r$rep', d['value'], d['ms_per_step'], d['config']['kernel_ms_one_frame_alone'])" 2>/dev/null || echo "$v rc=$rc"
    case $rc in 0) ;; *) exit $rc;; esac
  done
done
done
