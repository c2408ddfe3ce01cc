#!/bin/bash
# The C2 run at N = 8M and 16M per GPU (working set beyond the 256 MB MALL),
# with rocprofv3 kernel statistics and HBM traffic of the same command.
set -e
mkdir -p gpurun_out/bign
export TMPDIR=/tmp
O=gpurun_out/bign
for n in 8000000 16000000; do
  timeout -k 10 400 python bench.py --particles $n --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_$n.json 2> $O/bench_$n.err || { tail -20 $O/bench_$n.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$n.json')); r=d['roofline']; b=d['breakdown_ms_per_run']; print($n, '%.3g' % d['value'], 'prop us', round(r['avg_launch_us'],2), 'GB/s', round(r['achieved']), 'frac', round(r['frac'],3), b)"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python bench.py --particles 8000000 --steps 3 --warmup 1 --no-cpu-baseline > $O/stats.log 2>&1 || { tail -20 $O/stats.log; exit 1; }
ARGS="--particles 8000000 --steps 1 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python bench.py $ARGS > $O/fetch.log 2>&1 || { tail -20 $O/fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python bench.py $ARGS > $O/write.log 2>&1 || { tail -20 $O/write.log; exit 1; }
python tools/summarize_pmc.py $O/pmc_summary.json $O/fetch $O/write > /dev/null
python - <<'PY'
import csv, json
for x in csv.DictReader(open('gpurun_out/bign/stats/run_kernel_stats.csv')):
    print(x['Name'][:48], x['Calls'], round(float(x['AverageNs']) / 1e3, 2), 'us')
d = json.load(open('gpurun_out/bign/pmc_summary.json'))
for k, r in d.items():
    print(k[:40], 'read', round(r.get('hbm_read_bytes_corrected', 0) / 1e6, 2), 'MB  write', round(r.get('hbm_write_bytes', 0) / 1e6, 2), 'MB per dispatch')
PY
