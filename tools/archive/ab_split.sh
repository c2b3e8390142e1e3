#!/bin/bash
export RTAMD_DEBUG_KNOBS=1  # the library reads RT_* knobs only when asked (rt_debug_env_knobs)
# A/B of FrameParams::split_k (RT_SPLIT_K: the costliest waves of lone FULL frames as 16-lane sub-waves):
# parity tests first, then C5 (bunny FULL) and the soup FULL one frame at a time, and C5 at 4 in flight.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/ab_split
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 240 --timeout-method thread \
    -k "split_costliest or longest_first or bunny_1080p or golden_images or ragged" > $OUT/pytest.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for K in ${KS:-0 512 1024 2048}; do
    for cfg in ${CFGS:-bunny:full:1 soup:full:1 bunny:full:4}; do
      IFS=: read sc mode fif <<< "$cfg"
      env ${VAR:-RT_SPLIT_K}=$K timeout -k 10 200 python bench.py --scene $sc --mode $mode --frames-in-flight $fif --no-cpu --no-extra \
          --no-e2e --no-stats --steps 50 --warmup 5 > $OUT/b.json 2> $OUT/b.err
      rc=$?; [ $rc -ne 0 ] && { echo "bench rc=$rc"; tail -5 $OUT/b.err; exit $rc; }
      python -c "import json; d=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); c=d['config']; print('${VAR:-RT_SPLIT_K}=$K $sc $mode fif$fif r$rep', d['value'], d['ms_per_step'], c.get('kernel_ms_one_frame_alone'))" | tee -a $OUT/ab.txt
    done
  done
done
exit 0
