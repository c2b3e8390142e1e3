#!/bin/bash
# rocprofv3 evidence for k_render_full (FULL mode: shadow + one reflection bounce) on the 1M soup and
# the bunny (C5), same passes as tools/profile.sh; summarise each with
#   RT_PROFILE_LATEST=0 python tools/summarize_profile.py <tag> gpurun_out/r02f_full_<scene>/prof
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for sc in soup bunny; do
  OUTDIR=gpurun_out/r02f_full_$sc/prof \
  BENCH_ARGS="--scene $sc --mode full --steps 20 --warmup 3 --no-cpu --no-extra --no-e2e --frames-in-flight 1" \
  PMC_ARGS="--scene $sc --mode full --steps 5 --warmup 1 --no-cpu --no-stats --no-extra --no-e2e --frames-in-flight 1" \
  bash tools/profile.sh > gpurun_out/r02f_full_$sc.log 2>&1
  rc=$?; echo "$sc profile rc=$rc"; tail -9 gpurun_out/r02f_full_$sc.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
