mkdir -p gpurun_out
L=$PWD/ray-tracing-project_amd/lib
for tag in fast fastbits; do
  RTAMD_LIB=$L/librtamd_$tag.so RT_KERNEL_VARIANT=1536 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pyt_$tag.txt 2>&1; rc=$?
  echo "$tag rc=$rc $(tail -1 gpurun_out/pyt_$tag.txt)"; case $rc in 0|1) ;; *) exit $rc;; esac
done
RUNS="dvote:1536 fast:0 fast:1536 fastbits:0 fastbits:1536" FIF=1 bash tools/ab_matrix.sh
for tag in dvote fast fastbits; do for sc in "--scene bunny --mode full" "--scene bunny" "--mode full"; do
  RTAMD_LIB=$L/librtamd_$tag.so RT_KERNEL_VARIANT=1536 timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu --no-e2e --no-stats $sc > gpurun_out/b.json 2>/dev/null; rc=$?
  python3 -c "import json; d=json.load(open('gpurun_out/b.json')); print('$tag', '$sc', d['value'], d['config']['kernel_ms_per_frame'])" || echo "rc=$rc"; case $rc in 0|1) ;; *) exit $rc;; esac
done; done
