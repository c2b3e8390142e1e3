set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/fifab
for rep in 1 2; do
  for bx in gpu host; do
    timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu --no-side --no-extra --boxes $bx > gpurun_out/fifab/${bx}_r$rep.json 2>/dev/null
    rc=$?; python3 -c "
import json;d=json.loads(open('gpurun_out/fifab/${bx}_r$rep.json').read().strip().splitlines()[-1]);c=d['config']
print('$bx r$rep', d['value'], d['ms_per_step'], c['kernel_ms_per_frame'], c['kernel_ms_one_frame_alone'])"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
