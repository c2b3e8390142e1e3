#!/bin/bash
# Round 6: the lone-frame split size under the moving camera (predicted map): RT_SPLIT_K (FULL) / RT_SPLIT_KP (PRIMARY)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-splitk}
export MNOR05=1
MSCENES="bunny:full" MPOLICIES="lib env:RT_SPLIT_K=2048 env:RT_SPLIT_K=3072 env:RT_SPLIT_K=4096 env:RT_SPLIT_K=1024" \
  bash tools/gpu_round6.sh $TAG moving || exit $?
mv gpurun_out/$TAG/moving.jsonl gpurun_out/$TAG/moving_full.jsonl
MSCENES="bunny:primary" MPOLICIES="lib env:RT_SPLIT_KP=2048 env:RT_SPLIT_KP=3072 env:RT_SPLIT_KP=512" \
  bash tools/gpu_round6.sh $TAG moving
