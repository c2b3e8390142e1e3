#!/bin/bash
# Full measurement pass (GPU box): default bench line (with CPU baseline), rocprofv3 trace + PMC
# passes of the bench kernel, and the C2/C5 bunny configurations. Output under gpurun_out/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/meas
timeout -k 10 600 python bench.py > gpurun_out/meas/bench_default.json 2> gpurun_out/meas/bench_default.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/meas/bench_default.json; case $rc in 0) ;; *) exit $rc;; esac
for cfg in "bunny primary" "bunny full" "soup full"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --scene $1 --mode $2 --no-cpu --steps 20 --warmup 5 \
      > gpurun_out/meas/bench_$1_$2.json 2> gpurun_out/meas/bench_$1_$2.err
  rc=$?; echo "$1 $2 rc=$rc"; python3 -c "import json; d=json.load(open('gpurun_out/meas/bench_$1_$2.json')); print(d['value'], d['unit'], d['ms_per_step'], d['config'].get('kernel_ms_per_frame'))" || true
  case $rc in 124|134|137|139) exit $rc;; esac
done
EXTRA_PMC="SQ_INSTS_LDS SQ_INSTS_BRANCH SQC_DCACHE_REQ SQC_DCACHE_MISSES SQC_DCACHE_BUSY_CYCLES" bash tools/profile.sh
