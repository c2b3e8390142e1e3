#!/bin/bash
# Super-tile order at one shard (C3 / C4 frames, bench defaults), RT_SUPER_TILE = 0 (default) / 2 / 4 / 8
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/supern1
for rep in 1 2; do
for cfg in "1920x1080 4" "1920x1080 1" "3840x2160 4"; do
  set -- $cfg
  for st in 0 2 4 8; do
    o=gpurun_out/supern1/${1}_f$2_s${st}_r$rep
    RT_SUPER_TILE=$st timeout -k 10 300 python bench.py --frame $1 --frames-in-flight $2 --steps 50 --warmup 5 --no-cpu --no-stats --no-e2e --no-extra > $o.json 2> $o.err
    rc=$?
    python3 -c "import json; d=json.load(open('$o.json')); print('$1 fif$2 super=$st r$rep', d['value'], d['ms_per_step'], d['config']['kernel_ms_one_frame_alone'])" || echo "rc=$rc"
    case $rc in 0) ;; *) exit $rc;; esac
  done
done
done
