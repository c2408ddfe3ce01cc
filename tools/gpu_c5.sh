#!/bin/bash
# C5 move program: parity of every -m gpu test, the C5 rate, and the kernel statistics of the
# same command.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/c5r
rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $O/pytest.log | head -80; exit $rc; }
timeout -k 10 300 python tools/bench_moves.py c5 c3 c3async > $O/moves.json 2> $O/moves.err || { tail $O/moves.err; exit 1; }
cat $O/moves.json | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python tools/bench_moves.py c5 > $O/stats.log 2>&1 || { tail -20 $O/stats.log; exit 1; }
python - <<'PY'
import csv
for x in list(csv.DictReader(open('gpurun_out/c5r/stats/run_kernel_stats.csv')))[:6]:
    print(x['Name'][:60], x['Calls'], round(float(x['AverageNs'])/1e3, 2), 'us')
PY
