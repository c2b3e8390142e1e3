#!/bin/bash
# Round 6: the longest-first sort on a stream of its own (default) vs on the frame's stream (RT_LPT_SORT_INLINE=1),
# lone frames one at a time under the moving camera; the soup also with a re-sort on every moving frame (RT_LPT_MOVED=1)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-sortside}
export MNOR05=1
MSCENES="bunny:full bunny:primary" MPOLICIES="lib env:RT_LPT_SORT_INLINE=1 lib env:RT_LPT_SORT_INLINE=1" \
  bash tools/gpu_round6.sh $TAG moving || exit $?
mv gpurun_out/$TAG/moving.jsonl gpurun_out/$TAG/moving_bunny.jsonl
MSCENES="soup:primary" MPOLICIES="lib env:RT_LPT_SORT_INLINE=1 env:RT_LPT_MOVED=1 env:RT_LPT_MOVED=1,RT_LPT_SORT_INLINE=1 lib env:RT_LPT_MOVED=1" \
  bash tools/gpu_round6.sh $TAG moving
