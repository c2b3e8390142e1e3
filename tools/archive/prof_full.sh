#!/bin/bash
# rocprofv3 kernel-trace stats of the FULL configurations (GPU box): gpurun_out/pfull/<scene>/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for sc in ${SCENES:-bunny soup}; do
  mkdir -p gpurun_out/pfull/$sc
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pfull/$sc -o run --output-format csv -- \
      python3 bench.py --scene $sc --mode full --no-cpu --no-stats --steps 10 --warmup 3 > gpurun_out/pfull/$sc/bench.json 2> gpurun_out/pfull/$sc/err.txt
  rc=$?; echo "$sc rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
  f=$(ls gpurun_out/pfull/$sc/*/run_kernel_stats.csv 2>/dev/null | head -1); [ -z "$f" ] && f=$(find gpurun_out/pfull/$sc -name "*kernel_stats.csv" | head -1)
  python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')): print('  %-60s calls %5s avg %9.1f us' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e3))"
done
