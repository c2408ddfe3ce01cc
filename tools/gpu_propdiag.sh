#!/bin/bash
# propagate-kernel ablations through the bench's own instrumented timing (diagnostics only)
set -e
mkdir -p gpurun_out
for m in ${MODES:-0 1 2 3}; do
  WSMC_DIAG_PROP_MODE=$m timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/pd$m.json 2> gpurun_out/pd.err || { tail -20 gpurun_out/pd.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/pd$m.json')); print('prop mode $m', d['roofline']['avg_launch_us'], 'us')"
done
