#!/bin/bash
# Rehearse bench.py's N > 1 path on a 1-GPU box: 2 ranks wrap onto device 0.
# Backend gloo (host): exercises barrier, max-over-ranks timing, u0 gather, JSON line.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
MPCQP_BENCH_BACKEND=gloo timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 10 --warmup 2 --no-callers \
  > gpurun_out/dist_gloo.json 2> gpurun_out/dist_gloo.err || { tail -20 gpurun_out/dist_gloo.err; exit 1; }
cat gpurun_out/dist_gloo.json
# (RCCL itself refuses two ranks on one device -- 'Duplicate GPU detected' -- so the
# nccl leg needs a multi-GPU node: the driver's scaling run.)
