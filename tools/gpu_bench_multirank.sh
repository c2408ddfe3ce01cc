#!/bin/bash
# bench.py's multi-rank path (rendezvous, barriers, max over ranks, sharded run) with 2 ranks
# on the box's single GPU; records go through the host exchange since RCCL refuses two ranks
# on one device.
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29611 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline --exchange host --same-device \
  --shard-mode ${SHARD_MODE:-island} > gpurun_out/bench_mr.json 2> gpurun_out/bench_mr.err || { tail -30 gpurun_out/bench_mr.err; exit 1; }
cat gpurun_out/bench_mr.json
