#!/bin/bash
export RTAMD_DEBUG_KNOBS=1  # the library reads RT_* knobs only when asked (rt_debug_env_knobs)
# FULL-mode A/B (GPU box): parity tests, then bench of bunny/soup FULL per RT_KERNEL_VARIANT in VARIANTS
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/fab
if [ "${RUN_TESTS:-1}" = "1" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 600 > gpurun_out/fab/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/fab/pytest.log; case $rc in 0) ;; *) exit $rc;; esac
fi
for v in ${VARIANTS:-0 16}; do for sc in ${SCENES:-bunny soup}; do
  RT_KERNEL_VARIANT=$v timeout -k 10 300 python bench.py --scene $sc --mode full --no-cpu --steps 20 --warmup 5 > gpurun_out/fab/v${v}_$sc.json 2> gpurun_out/fab/v${v}_$sc.err
  rc=$?; python3 -c "import json; d=json.load(open('gpurun_out/fab/v${v}_$sc.json')); c=d['config']; print('v$v $sc', d['value'], c['kernel_ms_per_frame'], c.get('total_mrays_per_s'))" || echo "rc=$rc"
  case $rc in 0) ;; *) exit $rc;; esac
done; done
