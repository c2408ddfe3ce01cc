#!/bin/bash
# C3 (linear regression + autoRW pair every step, 1M, T=10): rate + per-kernel profile
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/c3
rm -rf $O; mkdir -p $O
timeout -k 10 300 python tools/bench_moves.py c3 c3async > $O/c3.json 2> $O/c3.err || { tail -20 $O/c3.err; exit 1; }
cat $O/c3.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python tools/bench_moves.py c3async > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python - <<'PY'
import csv
rows = list(csv.DictReader(open('gpurun_out/c3/prof/run_kernel_stats.csv')))
for x in rows: print(x['Name'][:50], x['Calls'], round(float(x['AverageNs'])/1e3,2), 'us', round(float(x['TotalDurationNs'])/1e6,2), 'ms total')
PY
