#!/bin/bash
export RTAMD_DEBUG_KNOBS=1  # the library reads RT_* knobs only when asked (rt_debug_env_knobs)
# Round 3 A/B: fp32 4-wide tree prefetch forms (librtamd_wpf*.so) vs the default build and the binary tree
# (RT_KERNEL_VARIANT=2097152); C3 at 4 frames in flight and one frame at a time; then one SQ counter pass
# each for the wide default and the binary tree (one frame in flight).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r03_abwide}
mkdir -p $OUT
export TMPDIR=/tmp
L=$PWD/ray-tracing-project_amd/lib
hard() { case $1 in 124|134|137|139) echo "hard failure ($1): stopping"; exit $1;; esac; }
for rep in 1 2; do
for cfg in "default::0" "binary::2097152" ${LIBS:-wpf0 wpf1 wpf3 wpf4}; do
  name=${cfg%%::*}; var=${cfg##*::}; [ "$var" = "$cfg" ] && var=0
  lib=$L/librtamd.so; [ -f $L/librtamd_$name.so ] && lib=$L/librtamd_$name.so
  for fif in 4 1; do
    RTAMD_LIB=$lib RT_KERNEL_VARIANT=$var timeout -k 10 200 python bench.py --no-cpu --no-extra --no-e2e --steps 50 \
        --frames-in-flight $fif > $OUT/${name}_fif${fif}_r$rep.json 2> $OUT/${name}_fif${fif}_r$rep.err
    rc=$?; hard $rc
    python3 -c "import json;d=json.load(open('$OUT/${name}_fif${fif}_r$rep.json'));print('$name fif$fif r$rep', d['value'], d['ms_per_step'], d['config']['kernel_ms_one_frame_alone'], d['roofline']['n_node'])"
  done
done
done
[ "${PMC:-1}" = 1 ] || exit 0
for cfg in ${PMCCFG:-default::0 binary::2097152}; do
  name=${cfg%%::*}; var=${cfg##*::}
  lib=$L/librtamd.so; [ -f $L/librtamd_$name.so ] && lib=$L/librtamd_$name.so
  RTAMD_LIB=$lib RT_KERNEL_VARIANT=$var timeout -s KILL 120 rocprofv3 --pmc ${PMCSET:-SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM} \
      -d $OUT/pmc_$name -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-stats --no-extra --no-e2e --frames-in-flight 1 \
      > $OUT/pmc_$name.json 2> $OUT/pmc_$name.err
  rc=$?; echo "pmc $name rc=$rc"; hard $rc
done
exit 0
