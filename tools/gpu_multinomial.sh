#!/bin/bash
# Multinomial resampling on the GPU: the whole -m gpu suite, the fused bench with
# multinomial draws, and its rocprofv3 kernel statistics. Stops at the first failure.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -q -m gpu -x > gpurun_out/pytest_all.log 2>&1 || { tail -40 gpurun_out/pytest_all.log; exit 1; }
tail -2 gpurun_out/pytest_all.log
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --scheme multinomial > gpurun_out/bench_multi.json 2> gpurun_out/bench_multi.err || { tail -20 gpurun_out/bench_multi.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_multi.json')); print(d['value'], d['ms_per_step'], d['breakdown_ms_per_run'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_multi -o run -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline --scheme multinomial > gpurun_out/prof_multi.log 2>&1
python - <<'PY'
import csv
for x in csv.DictReader(open('gpurun_out/prof_multi/run_kernel_stats.csv')): print(x['Name'][:40], x['Calls'], round(float(x['AverageNs'])/1e3,2))
PY
