#!/bin/bash
# Parity, then bench under a few launch-shape variants (diagnostics env vars), then a rocprof
# kernel-stats pass of the default. Stops at the first failure.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py tests/test_golden.py -q -m gpu -x > gpurun_out/pytest.log 2>&1 || { tail -30 gpurun_out/pytest.log; exit 1; }
tail -1 gpurun_out/pytest.log
for ppt in 1 2 4; do
  WSMC_PROP_PPT=$ppt timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_ppt$ppt.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bench_ppt$ppt.json')); print('ppt $ppt', round(d['value']/1e10,3), 'e10', round(d['ms_per_step'],3), 'ms', d['roofline']['avg_launch_us'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof.log 2>&1
python - <<'PY'
import csv
for x in csv.DictReader(open('gpurun_out/prof/run_kernel_stats.csv')): print(x['Name'][:40], x['Calls'], round(float(x['AverageNs'])/1e3,2))
PY
