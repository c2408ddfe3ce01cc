#!/bin/bash
# gpu_quick.sh + bench.py's multi-rank path in strong scaling (2 ranks on the box's GPU, host exchange)
set -o pipefail
bash tools/gpu_quick.sh || exit 1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29613 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline --exchange host --same-device \
  --global-particles 1000001 > gpurun_out/q/bench_strong.json 2> gpurun_out/q/bench_strong.err || { tail -30 gpurun_out/q/bench_strong.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/q/bench_strong.json'));print('strong x2', d['scaling'], d['config']['global_particles'], d['config']['n_particles_per_gpu'], round(d['value']/1e9,2))"
