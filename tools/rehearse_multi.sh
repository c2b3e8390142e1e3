#!/bin/bash
# Multi-rank rehearsal on a one-GPU box: N ranks share device 0 (gloo for the timing reductions).
# Exercises the torchrun launch, shard assignment, barrier and MAX/SUM reductions of bench.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/multi
for n in ${NS:-2 4}; do
  BENCH_DEVICE=0 BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
      --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --steps 10 --warmup 3 --no-cpu \
      > gpurun_out/multi/n$n.json 2> gpurun_out/multi/n$n.err
  rc=$?; echo "n=$n rc=$rc"; cat gpurun_out/multi/n$n.json; case $rc in 0) ;; *) tail -5 gpurun_out/multi/n$n.err; exit $rc;; esac
done
