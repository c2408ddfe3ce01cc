#!/bin/bash
# C3/C5 with 1 vs 2 particles per Move thread (WSMC_DIAG_MOVE_K)
set -o pipefail
mkdir -p gpurun_out/mvk
for k in 1 2; do
  WSMC_DIAG_MOVE_K=$k timeout -k 10 300 python tools/bench_moves.py > gpurun_out/mvk/k$k.json 2> gpurun_out/mvk/k$k.err || { tail gpurun_out/mvk/k$k.err; exit 1; }
  python -c "import json; [print('K=$k', json.loads(l)['config'][:3], round(json.loads(l)['seconds_per_run']*1e3,3), 'ms') for l in open('gpurun_out/mvk/k$k.json')]"
done
