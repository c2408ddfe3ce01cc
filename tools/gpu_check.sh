#!/bin/bash
# GPU round-trip used during development: parity tests, bench, rocprof kernel stats.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -m gpu -x > gpurun_out/pytest.log 2>&1; echo PYTEST=$? >> gpurun_out/pytest.log; tail -3 gpurun_out/pytest.log
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err; echo BENCH=$?; cat gpurun_out/bench.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['achieved'], d['breakdown_ms_per_run'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof.log 2>&1; echo PROF=$?
python - <<'PY'
import csv
for x in csv.DictReader(open('gpurun_out/prof/run_kernel_stats.csv')): print(x['Name'][:40], x['Calls'], round(float(x['AverageNs'])/1e3,2))
PY
