#!/bin/bash
# C3 soup PRIMARY with the default (SBVH) builder: leaf-size bounds and frames-in-flight counts,
# interleaved, 2 reps. Output under gpurun_out/lfsw/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/lfsw
for rep in 1 2; do
for cfg in ${CFGS:-4:4 2:4 3:4 6:4 8:4 4:6 4:8}; do
  IFS=: read leaf fif <<< "$cfg"
  out=gpurun_out/lfsw/l${leaf}_f${fif}_r$rep.json
  timeout -k 10 300 python bench.py --scene soup --mode primary --leaf $leaf --frames-in-flight $fif --steps 50 \
      --warmup 5 --no-cpu --no-e2e --no-extra > $out 2> ${out%.json}.err
  rc=$?
  python3 -c "import json; d=json.load(open('$out')); c=d['config']; print('leaf $leaf fif$fif r$rep', d['value'], d['ms_per_step'], c['kernel_ms_one_frame_alone'], d['roofline'].get('n_node'), d['roofline'].get('n_tri'))" 2>/dev/null || echo "$cfg rc=$rc"
  case $rc in 0) ;; *) exit $rc;; esac
done
done
