#!/bin/bash
# Generic statement path after a change: parity of every -m gpu test, then C2 through the
# statements (fused resample vs the reduce-kernel sequence), C3 and its kernel statistics.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/st2
rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $O/pytest.log | head -80; exit $rc; }
summ() { python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], round(d['value']/1e9,3), 'G/s', round(d['ms_per_run'],3), 'ms/run')" $1 $2; }
timeout -k 10 300 python bench.py --no-cpu-baseline --statements > $O/st.json 2> $O/st.err || { tail $O/st.err; exit 1; }
summ $O/st.json statements
WSMC_DIAG_RESAMPLE_REDUCE=1 timeout -k 10 300 python bench.py --no-cpu-baseline --statements > $O/st_red.json 2> $O/st_red.err || { tail $O/st_red.err; exit 1; }
summ $O/st_red.json statements-reduce-seq
timeout -k 10 300 python tools/bench_moves.py c3 c3async > $O/c3.jsonl 2> $O/c3.err || { tail $O/c3.err; exit 1; }
cut -c1-200 $O/c3.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --no-cpu-baseline --statements --steps 2 --warmup 1 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python - <<'PY'
import csv
for x in list(csv.DictReader(open('gpurun_out/st2/prof/run_kernel_stats.csv')))[:12]:
    print(x['Name'][:56], x['Calls'], round(float(x['AverageNs'])/1e3, 2), 'us', round(float(x['TotalDurationNs'])/1e6, 2), 'ms')
PY
