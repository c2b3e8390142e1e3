set -u
mkdir -p gpurun_out/lpt
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "longest_first or variants or frames_in_flight" > gpurun_out/lpt/pytest.log 2>&1
rc=$?; tail -5 gpurun_out/lpt/pytest.log; [ $rc -ne 0 ] && exit $rc
for sv in "soup primary 0" "soup primary 131072" "bunny full 0" "bunny full 131072" "bunny primary 0"; do
  set -- $sv
  timeout -k 10 120 python tools/timeline.py capture gpurun_out/lpt/$1_$2_$3.npz --scene $1 --mode $2 --variant $3 || exit $?
done
timeout -k 10 300 python bench.py --frames-in-flight 1 --no-cpu --no-extra > gpurun_out/lpt/bench_fif1.json 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/lpt/bench.json 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu --no-extra > gpurun_out/lpt/bench20.json 2>&1 || exit $?
for cfg in "bunny primary" "bunny full" "soup full"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --scene $1 --mode $2 --no-cpu --steps 20 --warmup 5 > gpurun_out/lpt/bench_$1_$2.json 2>&1 || exit $?
  timeout -k 10 300 python bench.py --scene $1 --mode $2 --no-cpu --steps 20 --warmup 5 --frames-in-flight 1 > gpurun_out/lpt/bench_$1_$2_fif1.json 2>&1 || exit $?
done
