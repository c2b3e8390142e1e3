#!/bin/bash
# Round 6: k_order_lpt with register-resident items (this build) against the loop form (lib/librtamd_r06f1.so),
# lone frames one at a time under the moving camera, interleaved; the soup also re-sorting every moving frame
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-sortfast}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export RTAMD_DEBUG_KNOBS=1
for rep in 1 2; do
  for lib in cur r06f1; do
    if [ $lib = cur ]; then L=$PWD/ray-tracing-project_amd/lib/librtamd.so; else L=$PWD/ray-tracing-project_amd/lib/librtamd_$lib.so; fi
    for sc in bunny:full bunny:primary soup:primary; do
      IFS=: read scn md <<< "$sc"
      for pol in lib env:RT_LPT_MOVED=1; do
        [ $scn != soup ] && [ $pol != lib ] && continue
        RTAMD_LIB=$L timeout -k 10 180 python tools/moving_ab.py $scn $md $pol 60 1 | sed "s/\"lib\": \"[^\"]*\"/\"lib\": \"$lib\"/" >> $OUT/moving.jsonl 2>> $OUT/moving.err
        rc=$?; [ $rc -ne 0 ] && { echo "sortfast $lib $sc $pol rc=$rc"; exit $rc; }
      done
    done
  done
done
python3 tools/moving_summary.py $OUT/moving.jsonl
