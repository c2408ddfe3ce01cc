#!/bin/bash
# Round evidence in one call: pytest -m gpu, smoke(), the default bench line, the rocprofv3
# kernel statistics of the same bench command, and the FETCH_SIZE / WRITE_SIZE passes
# (separate invocations) summarised per kernel. Stops at the first failing GPU step.
set -e
mkdir -p gpurun_out/round
export TMPDIR=/tmp
O=gpurun_out/round
timeout -k 10 1100 python -u -m pytest tests -q -m gpu -x --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 400 python bench.py --no-cpu-baseline --statements > $O/bench_statements.json 2> $O/bench_statements.err || { tail -20 $O/bench_statements.err; exit 1; }
cat $O/bench_statements.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python bench.py --no-cpu-baseline > $O/stats.log 2>&1 || { tail -20 $O/stats.log; exit 1; }
ARGS="--steps 2 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python bench.py $ARGS > $O/fetch.log 2>&1 || { tail -20 $O/fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python bench.py $ARGS > $O/write.log 2>&1 || { tail -20 $O/write.log; exit 1; }
python tools/summarize_pmc.py $O/pmc_summary.json $O/fetch $O/write > /dev/null
python tools/pmc_step_bytes.py $O/pmc_summary.json 1000000 100 $O/pmc_step_bytes.json
python - <<'PY'
import csv, json
for x in csv.DictReader(open('gpurun_out/round/stats/run_kernel_stats.csv')):
    print(x['Name'][:48], x['Calls'], round(float(x['AverageNs']) / 1e3, 2), 'us')
d = json.load(open('gpurun_out/round/pmc_summary.json'))
for k, r in d.items():
    if 'prop' in k:
        print(k[:40], 'read', round(r.get('hbm_read_bytes_corrected', 0) / 1e6, 2), 'MB  write', round(r.get('hbm_write_bytes', 0) / 1e6, 2), 'MB per dispatch')
PY
