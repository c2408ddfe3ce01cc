#!/bin/bash
# kernel timeline of the LGSSM statement path (one steady step)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/lp
mkdir -p $O
rm -rf $O/stats
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/stats -o run -- python tools/bench_lgssm.py gpu > $O/stats.log 2>&1 || { tail -20 $O/stats.log; exit 1; }
python - <<'PY'
import csv
for x in csv.DictReader(open('gpurun_out/lp/stats/run_kernel_stats.csv')):
    print(x['Name'][:60], x['Calls'], round(float(x['AverageNs']) / 1e3, 2), 'us')
rows = list(csv.DictReader(open('gpurun_out/lp/stats/run_kernel_trace.csv')))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
mid = len(rows) - 300
t0 = int(rows[mid]['Start_Timestamp'])
for r in rows[mid:mid + 20]:
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    print(f"{(s - t0) / 1e3:9.2f} {(e - s) / 1e3:7.2f}  {r['Kernel_Name'][:50]}")
PY
