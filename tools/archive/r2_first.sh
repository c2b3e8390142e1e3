#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r2a
export TMPDIR=/tmp
( lscpu; python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'cpu_count', os.cpu_count())"; nproc; echo OMP=$OMP_NUM_THREADS ) > gpurun_out/r2a/host.txt 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r2a/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r2a/pytest_gpu.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python bench.py --steps 100 --warmup 5 > gpurun_out/r2a/bench.json 2> gpurun_out/r2a/bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/r2a/bench.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 100 --warmup 5 --frames-in-flight 1 --no-cpu > gpurun_out/r2a/bench_fif1.json 2> gpurun_out/r2a/bench_fif1.err
rc=$?; echo "bench fif1 rc=$rc"; cat gpurun_out/r2a/bench_fif1.json
exit $rc
