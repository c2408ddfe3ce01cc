"""C5 FP64 roofline: FLOP per dispatch from the SQ_INSTS_VALU_*_F64 counters
(64 lanes x (2 FMA + MUL + ADD + TRANS)) of one rocprofv3 --pmc pass, against the average
duration of the same kernels from a separate --kernel-trace --stats pass.
    python tools/c5_flops.py gpurun_out/<tag>      (written by tools/gpu.sh c5flops)"""
import csv
import json
import sys

O = sys.argv[1]
stats = {x['Name']: x for x in csv.DictReader(open(f'{O}/stats/run_kernel_stats.csv'))}
d = json.load(open(f'{O}/pmc_summary.json'))
out = {}
for k, r in d.items():
    fl = 64 * (2 * r.get('SQ_INSTS_VALU_FMA_F64', 0) + r.get('SQ_INSTS_VALU_MUL_F64', 0)
               + r.get('SQ_INSTS_VALU_ADD_F64', 0) + r.get('SQ_INSTS_VALU_TRANS_F64', 0))
    st = stats.get(k)
    if not st or fl == 0:
        continue
    us = float(st['AverageNs']) / 1e3
    tf = fl / (us * 1e-6) / 1e12
    out[k] = {"flop_per_dispatch": fl, "avg_us": us, "tflops": tf, "frac_of_78.6": tf / 78.6,
              "dispatches": int(st['Calls'])}
    print(k.split('(')[0][-24:], 'GFLOP/dispatch %.3f' % (fl / 1e9), 'us %.1f' % us, 'TFLOP/s %.2f' % tf,
          'frac %.3f' % (tf / 78.6), 'calls', st['Calls'])
json.dump(out, open(f'{O}/c5_flops.json', 'w'), indent=1)
