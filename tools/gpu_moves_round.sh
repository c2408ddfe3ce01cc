#!/bin/bash
# Move-program evidence: C3 / C5 rates, C3 kernel statistics, C5 FP64 work (SQ_INSTS_VALU_*_F64)
# against its kernel durations. Run after pytest -m gpu is green.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/mv
rm -rf $O gpurun_out/c5; mkdir -p $O
timeout -k 10 400 python tools/bench_moves.py c3 c3async c5 > $O/moves.jsonl 2> $O/moves.err || { tail $O/moves.err; exit 1; }
cut -c1-330 $O/moves.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c3 -o run -- python tools/bench_moves.py c3async > $O/c3.log 2>&1 || { tail -20 $O/c3.log; exit 1; }
python - <<'PY'
import csv
for x in list(csv.DictReader(open('gpurun_out/mv/c3/run_kernel_stats.csv')))[:8]:
    print(x['Name'][:56], x['Calls'], round(float(x['AverageNs'])/1e3, 2), 'us')
PY
bash tools/gpu_c5_flops.sh
