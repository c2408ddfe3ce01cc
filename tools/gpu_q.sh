#!/bin/bash
# parity (pytest -m gpu) + the default 1M bench line + an 8M (beyond-MALL) bench line +
# rocprofv3 kernel stats of the 1M bench. Usage: tools/gpu_q.sh [pytest -k expr]
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/q
mkdir -p $O
K=${1:+-k "$1"}
eval timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread $K > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $O/pytest.log | head -100; exit $rc; }
summ() { python -c "import json,sys;d=json.load(open(sys.argv[1]));b=d['breakdown_ms_per_run'];T=d['config']['T'];print(sys.argv[2], round(d['value']/1e9,2), 'G/s', round(d['ms_per_step'],3), 'ms/run; prop/stats/fill us', round(b['propagate']*1e3/T,2), round(b['weight_stats']*1e3/T,2), round(b['scan_ancestors']*1e3/T,2), 'final ms', round(b['finalize_traceback'],3))" $1 $2; }
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
summ $O/bench.json 1M
timeout -k 10 300 python bench.py --no-cpu-baseline --particles 8000000 --steps 3 --warmup 1 > $O/bench8m.json 2> $O/bench8m.err || { tail $O/bench8m.err; exit 1; }
summ $O/bench8m.json 8M
rm -rf $O/stats
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python bench.py --no-cpu-baseline --steps 5 > $O/stats.log 2>&1 || { tail -20 $O/stats.log; exit 1; }
python - <<'PY'
import csv
for x in csv.DictReader(open('gpurun_out/q/stats/run_kernel_stats.csv')):
    if 'rocclr' in x['Name'] or 'delay' in x['Name']: continue
    print(x['Name'][:50], x['Calls'], round(float(x['AverageNs']) / 1e3, 2), 'us')
PY
