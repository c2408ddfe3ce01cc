#!/bin/bash
# C2 through the generic statement operators: lazy genealogy vs the eager ColumnStore gathers
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/stmt
mkdir -p $O
summ() { python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], round(d['value']/1e9,3), 'G/s', round(d['ms_per_run'],2), 'ms/run', 'frac', round(d['roofline']['frac'],3))" $1 $2; }
timeout -k 10 300 python bench.py --no-cpu-baseline --statements --steps 5 --warmup 1 > $O/lazy.json 2> $O/lazy.err || { tail $O/lazy.err; exit 1; }
summ $O/lazy.json statements-lazy
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 1 > $O/fused.json 2> $O/fused.err || { tail $O/fused.err; exit 1; }
summ $O/fused.json fused
timeout -k 10 300 python bench.py --no-cpu-baseline --statements --eager-store --steps 1 --warmup 1 > $O/eager.json 2> $O/eager.err || { tail $O/eager.err; exit 1; }
summ $O/eager.json statements-eager
rm -rf $O/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --no-cpu-baseline --statements --steps 2 --warmup 1 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python - <<'PY'
import csv
for x in csv.DictReader(open('gpurun_out/stmt/prof/run_kernel_stats.csv')):
    print(x['Name'][:60], x['Calls'], round(float(x['AverageNs']) / 1e3, 2), 'us', round(float(x['TotalDurationNs'])/1e6, 2), 'ms')
PY
