cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/fif
for rep in 1 2; do for f in 2 3 4 6 8; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu --no-side --no-extra --frames-in-flight $f > gpurun_out/fif/f${f}_r$rep.json 2> gpurun_out/fif/f${f}_r$rep.err || exit $?
  python3 -c "
import json;d=json.loads(open('gpurun_out/fif/f${f}_r$rep.json').read().strip().splitlines()[-1]);c=d['config']
print('fif$f r$rep', d['value'], d['ms_per_step'], c['kernel_ms_per_frame'], c['kernel_ms_one_frame_alone'])"
done; done
