#!/bin/bash
# kernel statistics of the sharded (one-rank RCCL) fused run
set -o pipefail
export TMPDIR=/tmp NCCL_SOCKET_IFNAME=lo
O=gpurun_out/rp
mkdir -p $O
rm -rf $O/stats
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python bench.py --no-cpu-baseline --rccl-one-rank --steps 5 > $O/stats.log 2>&1 || { tail -20 $O/stats.log; exit 1; }
python - <<'PY'
import csv
for x in csv.DictReader(open('gpurun_out/rp/stats/run_kernel_stats.csv')):
    print(x['Name'][:60], x['Calls'], round(float(x['AverageNs']) / 1e3, 2), 'us')
rows = list(csv.DictReader(open('gpurun_out/rp/stats/run_kernel_trace.csv')))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
# one steady step in the middle of the last run: print start offsets/durations of ~14 consecutive dispatches
mid = len(rows) - 400
t0 = int(rows[mid]['Start_Timestamp'])
for r in rows[mid:mid + 16]:
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    print(f"{(s - t0) / 1e3:9.2f} {(e - s) / 1e3:7.2f}  q{r.get('Queue_Id', r.get('Stream_Id', '?'))} {r['Kernel_Name'][:50]}")
PY
