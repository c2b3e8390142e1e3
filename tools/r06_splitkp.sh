#!/bin/bash
# Round 6: k_primary_fused's lone-frame split size on the L2-resident bunny (RT_SPLIT_KP), static / moving / stopped
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-splitkp}
export MNOR05=1
MSCENES="bunny:primary" MPOLICIES="lib env:RT_SPLIT_KP=0 env:RT_SPLIT_KP=256 env:RT_SPLIT_KP=512 env:RT_SPLIT_KP=768 lib env:RT_SPLIT_KP=512" \
  bash tools/gpu_round6.sh $TAG moving
