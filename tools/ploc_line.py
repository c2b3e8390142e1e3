"""One summary line of a bench.py JSON record (PLOC sweep): Mrays/s, one-frame kernel ms, tree size, setup."""
import json
import sys

try:
    d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
    c = d["config"]
    print(f"{d['value']:.1f} Mrays/s one_frame_ms {c['kernel_ms_one_frame_alone']} nodes {c['bvh_nodes']} "
          f"depth {c['bvh_depth']} setup_s {c['scene_setup_s']} bvh_ms {c['build_ms']['bvh']} "
          f"gpu_ms {c['build_ms'].get('bvh_gpu_kernels')} n_node {d['roofline'].get('n_node')} "
          f"n_tri {d['roofline'].get('n_tri')} sah {c.get('bvh_sah_cost')} parity {d.get('parity', {}).get('face_t_digest_equal')}")
except Exception as e:  # a failed run: say so on the sweep's line
    print(f"(no record: {e})")
