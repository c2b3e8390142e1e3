#!/bin/bash
export RTAMD_DEBUG_KNOBS=1  # the library reads RT_* knobs only when asked (rt_debug_env_knobs)
# Round 3: far-origin exactness tests with the per-ray culling pad (default build) and with the static pad
# only (librtamd_nopad.so, RT_DYN_PAD=0), then the whole GPU suite and the C3 / C5 bench lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r03_far}
mkdir -p $OUT
export TMPDIR=/tmp
hard() { case $1 in 124|134|137|139) echo "hard failure ($1): stopping"; exit $1;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_far.py -m gpu -v -p no:cacheprovider --timeout 240 --timeout-method thread > $OUT/far_default.log 2>&1
rc=$?; echo "far default rc=$rc"; tail -15 $OUT/far_default.log; hard $rc
RTAMD_LIB=$PWD/ray-tracing-project_amd/lib/librtamd_nopad.so timeout -k 10 300 python -u -m pytest tests/test_gpu_far.py -m gpu -v -p no:cacheprovider --timeout 240 --timeout-method thread > $OUT/far_nopad.log 2>&1
rc=$?; echo "far nopad rc=$rc"; grep -E "PASS|FAIL|far eye|far-origin|grazing" $OUT/far_nopad.log | tail -20; hard $rc
[ "${SUITE:-1}" = 1 ] || exit 0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -25 $OUT/pytest_gpu.log; hard $rc; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu > $OUT/bench.json 2> $OUT/bench.err; rc=$?; echo "bench rc=$rc"; hard $rc
RT_KERNEL_VARIANT=2097152 timeout -k 10 300 python bench.py --no-cpu > $OUT/bench_binary.json 2> $OUT/bench_binary.err; rc=$?; echo "bench binary rc=$rc"; hard $rc
timeout -k 10 300 python bench.py --no-cpu --frames-in-flight 1 --no-extra > $OUT/bench_fif1.json 2> $OUT/bench_fif1.err; rc=$?; echo "bench fif1 rc=$rc"; hard $rc
RT_KERNEL_VARIANT=2097152 timeout -k 10 300 python bench.py --no-cpu --frames-in-flight 1 --no-extra > $OUT/bench_binary_fif1.json 2> $OUT/bench_binary_fif1.err; rc=$?; echo "bench binary fif1 rc=$rc"; hard $rc
timeout -k 10 300 python bench.py --scene bunny --no-cpu --steps 100 > $OUT/bench_c2.json 2> $OUT/bench_c2.err; rc=$?; echo "c2 rc=$rc"; hard $rc
RT_KERNEL_VARIANT=2097152 timeout -k 10 300 python bench.py --scene bunny --no-cpu --steps 100 > $OUT/bench_c2_binary.json 2> $OUT/bench_c2_binary.err; rc=$?; echo "c2 binary rc=$rc"; hard $rc
timeout -k 10 300 python bench.py --scene bunny --mode full --no-cpu --steps 100 > $OUT/bench_c5.json 2> $OUT/bench_c5.err; rc=$?; echo "c5 rc=$rc"; hard $rc
exit 0
