set -u
mkdir -p gpurun_out/fullab
for v in 0 16 240 16432; do
  RT_KERNEL_VARIANT=$v timeout -k 10 300 python bench.py --scene soup --mode full --frames-in-flight 1 --steps 10 --warmup 2 --no-cpu --no-e2e --no-extra > gpurun_out/fullab/v$v.json 2> gpurun_out/fullab/v$v.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/fullab/v$v.json')); r=d['roofline']; print('v$v', d['value'], d['ms_per_step'], d['config']['kernel_ms_one_frame_alone'], 'total rays', d['config'].get('rays_per_frame_total'), 'n_node', r['n_node'], 'n_tri', r['n_tri'], 'alg B/ray', r['algorithmic_bytes_per_ray'])"
done
