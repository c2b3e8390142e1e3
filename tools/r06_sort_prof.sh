#!/bin/bash
# Round 6: rocprofv3 kernel trace of lone moving frames (C5 bunny FULL, C2 bunny PRIMARY): the longest-first sort's
# own duration beside the render kernel's
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-sortprof}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp MNOR05=1 RTAMD_DEBUG_KNOBS=1
for sc in bunny:full bunny:primary; do
  IFS=: read scn md <<< "$sc"
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/prof_${scn}_${md} -o run -- python3 tools/moving_ab.py $scn $md lib 60 1 \
      > $OUT/sortprof_${scn}_${md}.jsonl 2> $OUT/sortprof_${scn}_${md}.err
  rc=$?; echo "sortprof $sc rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/sortprof_${scn}_${md}.err; exit $rc; }
done
find $OUT -name "*kernel_stats.csv" | while read f; do echo "== $f"; cut -d, -f1-8 "$f" | head -12; done
