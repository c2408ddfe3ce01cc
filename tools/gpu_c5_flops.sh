#!/bin/bash
# C5 (damped oscillator, 5 sweeps, 4M) FP64 work from the SQ_INSTS_VALU_*_F64 counters
# (one pass), against the kernel durations of a separate --kernel-trace --stats pass:
# the FP64-VALU roofline of the score fold.
set -e
mkdir -p gpurun_out/c5
export TMPDIR=/tmp
O=gpurun_out/c5
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python tools/bench_moves.py c5 > $O/stats.log 2>&1 || { tail -20 $O/stats.log; exit 1; }
timeout -k 10 900 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 --output-format csv -d $O/pmc -o run -- python tools/bench_moves.py c5 > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
python tools/summarize_pmc.py $O/pmc_summary.json $O/pmc > /dev/null
python - <<'PY'
import csv, json
stats = {x['Name']: x for x in csv.DictReader(open('gpurun_out/c5/stats/run_kernel_stats.csv'))}
d = json.load(open('gpurun_out/c5/pmc_summary.json'))
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
    print(k.split('(')[0][-24:], 'GFLOP/dispatch %.3f' % (fl / 1e9), 'us %.1f' % us, 'TFLOP/s %.2f' % tf, 'frac %.3f' % (tf / 78.6), 'calls', st['Calls'])
json.dump(out, open('gpurun_out/c5/c5_flops.json', 'w'), indent=1)
PY
