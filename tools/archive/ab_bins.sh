#!/bin/bash
# A/B of the device SBVH builder's bin count (make-time kSahBins, lib/librtamd_bins*.so) on C3: the line,
# the tree's SAH cost and node / triangle steps per ray. Interleaved reps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-ab_bins}; mkdir -p $OUT
for rep in 1 2; do
  for tag in default ${LIBS:-bins64 bins128}; do
    if [ "$tag" = default ]; then lib=""; else lib="$PWD/ray-tracing-project_amd/lib/librtamd_$tag.so"; fi
    RTAMD_LIB=$lib timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu --no-side --no-extra \
        > $OUT/${tag}_r$rep.json 2> $OUT/${tag}_r$rep.err
    rc=$?; echo "$tag r$rep rc=$rc $(python3 tools/ploc_line.py $OUT/${tag}_r$rep.json)"
    case $rc in 0) ;; *) exit $rc;; esac
  done
done
