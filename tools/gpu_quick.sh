#!/bin/bash
# parity (pytest -m gpu) + the default bench line + rocprofv3 kernel stats of the bench
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/q
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/q/pytest.log 2>&1; rc=$?
tail -2 gpurun_out/q/pytest.log
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" gpurun_out/q/pytest.log | head -100; exit $rc; }
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/q/bench.json 2> gpurun_out/q/bench.err || { tail gpurun_out/q/bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/q/bench.json'));b=d['breakdown_ms_per_run'];print('bench', round(d['value']/1e9,2), 'G/s', round(d['ms_per_step'],3), 'ms/run; prop/stats/fill us', round(b['propagate']*10,2), round(b['weight_stats']*10,2), round(b['scan_ancestors']*10,2))"
rm -rf gpurun_out/q/stats
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/q/stats -o run -- python bench.py --no-cpu-baseline --steps 5 > gpurun_out/q/stats.log 2>&1 || { tail -20 gpurun_out/q/stats.log; exit 1; }
python - <<'PY'
import csv
for x in csv.DictReader(open('gpurun_out/q/stats/run_kernel_stats.csv')):
    if 'rocclr' in x['Name'] or 'delay' in x['Name']: continue
    print(x['Name'][:50], x['Calls'], round(float(x['AverageNs']) / 1e3, 2), 'us')
PY
