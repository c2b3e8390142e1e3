#!/bin/bash
# Kernel-trace stats of soup FULL: the megakernel (product library) and the FULL stage pipeline
# (variants library, RT_KERNEL_VARIANT 16): per-stage time of the pipeline's kernels.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp RTAMD_DEBUG_KNOBS=1
OUT=gpurun_out/${TAG:-prof_pipe}; mkdir -p $OUT
ARGS="--scene soup --mode full --steps 10 --warmup 2 --no-cpu --no-extra --no-e2e --no-side --no-stats --frames-in-flight 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/mega -o run --output-format csv -- python3 bench.py $ARGS \
    > $OUT/mega.json 2> $OUT/mega.err
rc=$?; echo "mega rc=$rc"; [ $rc -ne 0 ] && exit $rc
for v in ${VARIANTS:-16}; do
  RTAMD_LIB=$PWD/ray-tracing-project_amd/lib/librtamd_variants.so RT_KERNEL_VARIANT=$v timeout -k 10 300 \
      rocprofv3 --kernel-trace --stats -d $OUT/v$v -o run --output-format csv -- python3 bench.py $ARGS \
      > $OUT/v$v.json 2> $OUT/v$v.err
  rc=$?; echo "variant $v rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
