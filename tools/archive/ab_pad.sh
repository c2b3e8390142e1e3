#!/bin/bash
# Round 3: cost of the per-ray culling pad: default build vs librtamd_nopad.so (static pad only), C3 / C2 / C5.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r03_abpad}
mkdir -p $OUT
L=$PWD/ray-tracing-project_amd/lib
hard() { case $1 in 124|134|137|139) echo "hard failure ($1): stopping"; exit $1;; esac; }
for rep in 1 2; do
  for lib in librtamd ${LIBS:-librtamd_nopad}; do
    for cfg in "soup primary 4" "soup primary 1" "bunny primary 4" "bunny full 4" "bunny full 1"; do
      set -- $cfg
      n=${lib}_$1_$2_fif$3_r$rep
      RTAMD_LIB=$L/$lib.so timeout -k 10 200 python bench.py --scene $1 --mode $2 --frames-in-flight $3 --no-cpu --no-extra --no-e2e --steps 50 > $OUT/$n.json 2> $OUT/$n.err
      rc=$?; hard $rc
      python3 -c "import json;d=json.load(open('$OUT/$n.json'));print('$n', d['value'], d['ms_per_step'], d['config']['kernel_ms_one_frame_alone'])"
    done
  done
done
exit 0
