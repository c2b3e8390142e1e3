#!/bin/bash
# Round-5 GPU pass: GPU tests (product library, and the RT_CHECK_PREFETCH debug build), the default bench
# line, the in-process multi-device line rehearsed on one GPU, then rocprofv3 profiles of the headline kernel
# (C3) and of the C5 FULL kernel. Every GPU step has its own time limit; stop at the first hard failure.
# Usage: bash tools/gpu_round5.sh <tag> [tests pftests bench multi prof profc5 profc2 ...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-run}; shift || true
STEPS=${*:-tests bench prof profc5}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
hard() { case $1 in 124|134|137|139) echo "hard failure ($1): stopping"; exit $1;; esac; }
for s in $STEPS; do
  case $s in
    tests)
      timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread \
          --durations=15 > $OUT/pytest_gpu.log 2>&1
      rc=$?; echo "pytest rc=$rc"; tail -25 $OUT/pytest_gpu.log; hard $rc ;;
    pftests)
      # the whole GPU suite against the debug build whose kernels check every scalar prefetch offset
      RTAMD_LIB=$PWD/ray-tracing-project_amd/lib/librtamd_pfcheck.so timeout -k 10 600 python -u -m pytest tests -m gpu -q \
          -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu_pfcheck.log 2>&1
      rc=$?; echo "pfcheck pytest rc=$rc"; tail -8 $OUT/pytest_gpu_pfcheck.log; hard $rc ;;
    multi)
      # the in-process multi-device path (no launcher) with two replicas sharing the box's GPU
      timeout -k 10 300 python bench.py --gpus 2 --devices 0,0 --steps 20 --warmup 5 > $OUT/bench_multi.json 2> $OUT/bench_multi.err
      rc=$?; echo "multi rc=$rc"; cat $OUT/bench_multi.json; hard $rc ;;
    bench)
      timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
      rc=$?; echo "bench rc=$rc"; cat $OUT/bench.json; hard $rc; [ $rc -ne 0 ] && exit $rc ;;
    ploc)
      timeout -k 10 300 python bench.py --steps 20 --warmup 5 --builder ploc --no-cpu --no-side > $OUT/bench_ploc.json 2> $OUT/bench_ploc.err
      rc=$?; echo "ploc rc=$rc"; cat $OUT/bench_ploc.json; hard $rc ;;
    profc2)
      OUTDIR=$OUT/profc2 \
      BENCH_ARGS="--scene bunny --mode primary --steps 20 --warmup 3 --no-cpu --no-extra --no-e2e --no-side --frames-in-flight 1" \
      PMC_ARGS="--scene bunny --mode primary --steps 5 --warmup 1 --no-cpu --no-stats --no-extra --no-e2e --no-side --frames-in-flight 1" \
      bash tools/profile.sh > $OUT/profile_c2.log 2>&1
      rc=$?; echo "profile c2 rc=$rc"; tail -12 $OUT/profile_c2.log; hard $rc ;;
    plocsweep)
      # PLOC A/B: neighbour radius x collapse node cost x leaf rule (C3, --builder ploc), then the SBVH line
      export RTAMD_DEBUG_KNOBS=1
      for cfg in 24:0.7:0 32:0.7:0 16:0.7:0 24:0.5:0 24:1.0:0 24:0.7:1 32:0.5:1 24:1.0:1; do
        IFS=: read r tr ru <<< "$cfg"
        RT_PLOC_RADIUS=$r RT_PLOC_TRAV=$tr RT_PLOC_RULE=$ru timeout -k 10 120 python bench.py --steps 20 --warmup 5 \
            --builder ploc --no-cpu --no-side --no-extra > $OUT/ploc_$cfg.json 2> $OUT/ploc_$cfg.err
        rc=$?; echo "ploc $cfg rc=$rc $(python3 tools/ploc_line.py $OUT/ploc_$cfg.json)"; hard $rc
      done ;;
    builders)
      # the same C3 line per builder (SBVH default, host binned SAH, device LBVH) and PLOC radii
      export RTAMD_DEBUG_KNOBS=1
      for cfg in ${BUILDERS:-sbvh sah sahgpu sbvhgpu lbvh ploc:4}; do
        IFS=: read b r <<< "$cfg"
        RT_PLOC_RADIUS=${r:-24} timeout -k 10 120 python bench.py --steps 20 --warmup 5 --builder $b --no-cpu --no-side \
            --no-extra > $OUT/builder_$cfg.json 2> $OUT/builder_$cfg.err
        rc=$?; echo "builder $cfg rc=$rc $(python3 tools/ploc_line.py $OUT/builder_$cfg.json)"; hard $rc
      done ;;
    prof)
      OUTDIR=$OUT/prof bash tools/profile.sh > $OUT/profile.log 2>&1
      rc=$?; echo "profile rc=$rc"; tail -12 $OUT/profile.log; hard $rc ;;
    profc5)
      OUTDIR=$OUT/profc5 \
      BENCH_ARGS="--scene bunny --mode full --steps 20 --warmup 3 --no-cpu --no-extra --no-e2e --no-side --frames-in-flight 1" \
      PMC_ARGS="--scene bunny --mode full --steps 5 --warmup 1 --no-cpu --no-stats --no-extra --no-e2e --no-side --frames-in-flight 1" \
      bash tools/profile.sh > $OUT/profile_c5.log 2>&1
      rc=$?; echo "profile c5 rc=$rc"; tail -12 $OUT/profile_c5.log; hard $rc ;;
  esac
done
exit 0
