#!/bin/bash
# N > 1 bench path rehearsed on a one-GPU box: 2 ranks on the same GPU, gloo for the collectives
# (the reduce through host memory).  Checks the multi-rank timing / JSON path with real HIP work.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
export PT_BENCH_BACKEND=gloo
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 \
  bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/dist2.log 2>&1
rc=$?; grep '^{' gpurun_out/dist2.log | cut -c1-400; tail -3 gpurun_out/dist2.log; exit $rc
