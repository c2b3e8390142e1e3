#!/bin/bash
# GPU tests with super-tile shards, the one-GPU shard rehearsal (super-tiles vs single tiles) and a
# two-rank rehearsal of bench.py (pack / gather / unpack through the e2e path).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/super
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/super/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/super/pytest.log; [ $rc -ne 0 ] && exit $rc
KS="2 4 8" FIFS="4" STS="1 0" bash tools/rehearse_shards.sh || exit $?
NS="2" bash tools/rehearse_multi.sh
