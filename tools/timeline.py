"""One step's kernel sequence from a rocprofv3 kernel trace: durations and the gaps between
consecutive kernels. Usage: python tools/timeline.py <run_kernel_trace.csv> <marker kernel> [k]
(the k-th occurrence of the marker starts the step, the next one ends it)."""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
mark = sys.argv[2]
k = int(sys.argv[3]) if len(sys.argv) > 3 else 5
idx = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith(mark)]
i0, i1 = idx[k], idx[k + 1]
prev = None
busy = 0.0
for r in rows[i0:i1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1e3 if prev is not None else 0.0
    busy += (e - s) / 1e3
    print(f"{r['Kernel_Name'][:60]:60s} dur {(e - s) / 1e3:7.1f} gap {gap:6.1f}")
    prev = e
span = (int(rows[i1]["Start_Timestamp"]) - int(rows[i0]["Start_Timestamp"])) / 1e3
print(f"step span {span:.1f} us, kernels {busy:.1f} us")
