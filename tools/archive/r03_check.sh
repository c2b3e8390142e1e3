#!/bin/bash
# Round 3: GPU suite, then bench lines: C3 default (binary tree), C3 with the fp32 4-wide tree (prefetch
# forms: default 4 = nearest child, librtamd_wpf0 none, librtamd_wpf2 all children), C2, C5.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r03_check}
mkdir -p $OUT
export TMPDIR=/tmp
L=$PWD/ray-tracing-project_amd/lib
hard() { case $1 in 124|134|137|139) echo "hard failure ($1): stopping"; exit $1;; esac; }
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
  rc=$?; echo "suite rc=$rc"; tail -32 $OUT/pytest_gpu.log; hard $rc; [ $rc -ne 0 ] && exit $rc
fi
b() {  # name, env, args
  local name=$1; shift
  env "$@" > $OUT/$name.json 2> $OUT/$name.err; local rc=$?; hard $rc
  python3 -c "import json;d=json.load(open('$OUT/$name.json'));r=d.get('roofline') or {};c=d['config'];print('$name', d['value'], d['ms_per_step'], c['kernel_ms_one_frame_alone'], r.get('n_node'), r.get('frac'))"
}
for rep in 1 2; do
  b c3_r$rep timeout -k 10 200 python bench.py --no-cpu --no-extra --no-e2e --steps 50
  b c3_wide_r$rep timeout -k 10 200 python bench.py --no-cpu --no-extra --no-e2e --steps 50 --wide
  b c3_wide_pf0_r$rep RTAMD_LIB=$L/librtamd_wpf0.so timeout -k 10 200 python bench.py --no-cpu --no-extra --no-e2e --steps 50 --wide
  b c3_wide_pf2_r$rep RTAMD_LIB=$L/librtamd_wpf2.so timeout -k 10 200 python bench.py --no-cpu --no-extra --no-e2e --steps 50 --wide
  b c3_fif1_r$rep timeout -k 10 200 python bench.py --no-cpu --no-extra --no-e2e --steps 50 --frames-in-flight 1
  b c3_wide_fif1_r$rep timeout -k 10 200 python bench.py --no-cpu --no-extra --no-e2e --steps 50 --frames-in-flight 1 --wide
done
b c2 timeout -k 10 200 python bench.py --scene bunny --no-cpu --no-e2e --steps 100
b c2_wide timeout -k 10 200 python bench.py --scene bunny --no-cpu --no-e2e --steps 100 --wide
b c5 timeout -k 10 200 python bench.py --scene bunny --mode full --no-cpu --no-e2e --steps 100
exit 0
