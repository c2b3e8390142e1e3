cd $GRAFT_REPO_ROOT
for f in 1 2 3 4; do
 timeout -k 10 200 python bench.py --steps 40 --warmup 5 --no-cpu --no-stats --frames-in-flight $f > gpurun_out/fif$f.json 2>/dev/null || exit 1
 python3 -c "import json; d=json.load(open('gpurun_out/fif$f.json')); print('fif $f', d['value'], d['ms_per_step'], d['config']['kernel_ms_per_frame'])"
 timeout -k 10 200 python bench.py --steps 40 --warmup 5 --no-cpu --no-stats --frames-in-flight $f --scene bunny --mode full > gpurun_out/fifb$f.json 2>/dev/null || exit 1
 python3 -c "import json; d=json.load(open('gpurun_out/fifb$f.json')); print('bunny full fif $f', d['value'], d['ms_per_step'], d['config']['kernel_ms_per_frame'])"
done
