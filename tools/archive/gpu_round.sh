#!/bin/bash
# One GPU-box pass: GPU tests (parity), the default bench line, then the rocprofv3 profile of the bench
# kernel (tools/profile.sh). Every GPU step has its own time limit; stop at the first hard failure.
# Usage: bash tools/gpu_round.sh <tag> [tests|bench|prof ...]   (default: all three)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-run}; shift || true
STEPS=${*:-tests bench prof}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
hard() { case $1 in 124|134|137|139) echo "hard failure ($1): stopping"; exit $1;; esac; }
for s in $STEPS; do
  case $s in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
          > $OUT/pytest_gpu.log 2>&1
      rc=$?; echo "pytest rc=$rc"; tail -15 $OUT/pytest_gpu.log; hard $rc; [ $rc -ne 0 ] && exit $rc ;;
    bench)
      timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err
      rc=$?; echo "bench rc=$rc"; cat $OUT/bench.json; hard $rc; [ $rc -ne 0 ] && exit $rc ;;
    bench20)
      timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench20.json 2> $OUT/bench20.err
      rc=$?; echo "bench20 rc=$rc"; cat $OUT/bench20.json; hard $rc; [ $rc -ne 0 ] && exit $rc ;;
    fif1)
      timeout -k 10 300 python bench.py --frames-in-flight 1 --no-cpu > $OUT/bench_fif1.json 2> $OUT/bench_fif1.err
      rc=$?; echo "fif1 rc=$rc"; cat $OUT/bench_fif1.json; hard $rc; [ $rc -ne 0 ] && exit $rc ;;
    c2c5)
      for cfg in "bunny primary" "bunny full" "soup full"; do
        set -- $cfg
        timeout -k 10 300 python bench.py --scene $1 --mode $2 --no-cpu --steps 100 --warmup 5 \
            > $OUT/bench_$1_$2.json 2> $OUT/bench_$1_$2.err
        rc=$?; echo "$1 $2 rc=$rc"; hard $rc
      done ;;
    prof)
      OUTDIR=$OUT/prof bash tools/profile.sh > $OUT/profile.log 2>&1
      rc=$?; echo "profile rc=$rc"; tail -12 $OUT/profile.log; hard $rc ;;
  esac
done
exit 0
