#!/bin/bash
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/profab -o run -- python tools/ablate.py > gpurun_out/profab.log 2>&1
python - <<'PY'
import csv, collections, numpy as np, glob
f = glob.glob('gpurun_out/profab/**/run_kernel_trace.csv', recursive=True) + glob.glob('gpurun_out/profab/run_kernel_trace.csv')
rows = list(csv.DictReader(open(f[0])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
# consecutive runs of the same kernel name: report median duration and median start-to-start
groups = []
for r in rows:
    n = r['Kernel_Name'].split('(')[0].split('::')[-1]
    if groups and groups[-1][0] == n: groups[-1][1].append(r)
    else: groups.append((n, [r]))
for n, g in groups:
    if len(g) < 50: continue
    d = np.array([(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3 for r in g])
    st = np.array([int(r['Start_Timestamp']) for r in g]) / 1e3
    print(f"{n:22s} n={len(g)} dur med {np.median(d):.2f} us, start-to-start med {np.median(np.diff(st)):.2f} us")
PY
