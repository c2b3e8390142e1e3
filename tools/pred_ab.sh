#!/bin/bash
# Round 6: a moving camera's cost map placed by the predicted next-frame position of each wave's content
# (RT_LPT_PRED, FrameParams::pred) -- lone moving frames per policy (tools/moving_ab.py), then the static bench lines
# of this build against the r06v build (lib/librtamd_r06v.so) on the same box, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-pred}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export MNOR05=1
P="env:RT_LPT_MOVED=1,RT_LPT_PRED=1"
MSCENES=${MSCENES:-"bunny:full bunny:primary soup:primary"} MPOLICIES=${MPOLICIES:-"lib $P $P,RT_LPT_DILATE=1 $P,RT_LPT_DILW=1 $P,RT_LPT_DILATE=1,RT_LPT_DILW=1 $P,RT_LPT_DILATE=0"} \
  bash tools/gpu_round6.sh $TAG moving || exit $?
[ -n "${NOSTATIC:-}" ] && exit 0
for rep in 1 2; do
  for lib in r06v cur; do
    if [ $lib = cur ]; then L=$PWD/ray-tracing-project_amd/lib/librtamd.so; else L=$PWD/ray-tracing-project_amd/lib/librtamd_$lib.so; fi
    for sc in soup:primary bunny:full; do
      IFS=: read scn md <<< "$sc"
      RTAMD_LIB=$L timeout -k 10 120 python bench.py --scene $scn --mode $md --steps 40 --warmup 5 --no-cpu --no-side --no-extra \
          --no-e2e --no-stats --no-cold --no-moving > $OUT/static_${lib}_${scn}_r$rep.json 2> $OUT/static_${lib}_${scn}_r$rep.err
      rc=$?; [ $rc -ne 0 ] && { echo "static $lib $scn rc=$rc"; tail -3 $OUT/static_${lib}_${scn}_r$rep.err; exit $rc; }
      python3 -c "import json;d=json.loads(open('$OUT/static_${lib}_${scn}_r$rep.json').read().strip().splitlines()[-1]);c=d['config'];print('static $lib $scn r$rep', d['value'], d['ms_per_step'], c['kernel_ms_one_frame_alone'], d['roofline']['kernel_ms_isolated'])"
    done
  done
done
