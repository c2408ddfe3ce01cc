#!/bin/bash
# GPU round-trip used during development: parity tests, kernel ablations, bench, rocprof
# kernel stats. Stops at the first failing step (no further GPU work after a fault).
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -m gpu -x > gpurun_out/pytest.log 2>&1 || { tail -30 gpurun_out/pytest.log; exit 1; }
tail -2 gpurun_out/pytest.log
timeout -k 10 300 python tools/ablate.py > gpurun_out/ablate.log 2>&1 || { tail -20 gpurun_out/ablate.log; exit 1; }
cat gpurun_out/ablate.log
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['achieved'], d['breakdown_ms_per_run'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof.log 2>&1
python - <<'PY'
import csv
for x in csv.DictReader(open('gpurun_out/prof/run_kernel_stats.csv')): print(x['Name'][:40], x['Calls'], round(float(x['AverageNs'])/1e3,2))
PY
