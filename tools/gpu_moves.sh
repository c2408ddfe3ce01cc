#!/bin/bash
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python tools/bench_moves.py > gpurun_out/moves.json 2> gpurun_out/moves.err || { tail -20 gpurun_out/moves.err; exit 1; }
cat gpurun_out/moves.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profmv -o run -- python tools/bench_moves.py c3 > gpurun_out/profmv.log 2>&1
python - <<'PY'
import csv
for x in csv.DictReader(open('gpurun_out/profmv/run_kernel_stats.csv')): print(x['Name'][:40], x['Calls'], round(float(x['AverageNs'])/1e3,2), round(float(x['TotalDurationNs'])/1e6,2), 'ms total')
PY
