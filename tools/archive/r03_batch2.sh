#!/bin/bash
# Round 3 batch 2: GPU suite; default bench line (C3 + C4 frame + C2/C5 side lines); FULL split-octant A/B
# (librtamd_nosplit.so = RT_FULL_SPLIT_OCT 0) on C5 and the soup FULL; N = 2 / 4 rehearsal on one GPU.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r03_b2}
mkdir -p $OUT
export TMPDIR=/tmp
L=$PWD/ray-tracing-project_amd/lib
hard() { case $1 in 124|134|137|139) echo "hard failure ($1): stopping"; exit $1;; esac; }
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
  rc=$?; echo "suite rc=$rc"; tail -28 $OUT/pytest_gpu.log; hard $rc; [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err; rc=$?; echo "bench rc=$rc"; hard $rc; cat $OUT/bench.json
for rep in 1 2; do
  for lib in librtamd librtamd_nosplit; do
    for cfg in "bunny full 4" "bunny full 1" "soup full 4"; do
      set -- $cfg
      n=${lib}_$1_$2_fif$3_r$rep
      RTAMD_LIB=$L/$lib.so timeout -k 10 200 python bench.py --scene $1 --mode $2 --frames-in-flight $3 --no-cpu --no-extra --no-e2e --no-side --steps 50 > $OUT/$n.json 2> $OUT/$n.err
      rc=$?; hard $rc
      python3 -c "import json;d=json.load(open('$OUT/$n.json'));print('$n', d['value'], d['ms_per_step'], d['config']['kernel_ms_one_frame_alone'], d['config'].get('total_mrays_per_s'))"
    done
  done
done
for n in 2 4; do
  BENCH_DEVICE=0 BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
      --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --steps 10 --warmup 3 --no-cpu \
      > $OUT/rehearse_n$n.json 2> $OUT/rehearse_n$n.err
  rc=$?; echo "rehearse n=$n rc=$rc"; hard $rc
  python3 -c "import json;d=json.load(open('$OUT/rehearse_n$n.json'));c=d['config'];print('n=$n', d['value'], c['scene_setup_s_per_rank'], c['scene_shared_build'])"
done
exit 0
