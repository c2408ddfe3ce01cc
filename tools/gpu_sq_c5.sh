#!/bin/bash
# SQ cycle split of the C5 move program's kernels
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/sqc5
rm -rf $O; mkdir -p $O
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES --output-format csv -d $O/p -o run -- python tools/bench_moves.py c5 > $O/p.log 2>&1 || { tail -20 $O/p.log; exit 1; }
python tools/summarize_pmc.py $O/p.json $O/p > /dev/null
python - $O/p.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k, r in d.items():
    wc = r['SQ_WAVE_CYCLES']
    if not r.get('SQ_WAVES'): continue
    print(k[:34], 'waves', int(r['SQ_WAVES']), 'cyc/wave', int(wc / r['SQ_WAVES']),
          'active %.2f wait %.2f stall %.2f valu-active %.2f' % (r['SQ_ACTIVE_INST_ANY'] / wc, r['SQ_WAIT_ANY'] / wc,
          r['SQ_WAIT_INST_ANY'] / wc, r['SQ_ACTIVE_INST_VALU'] / wc),
          'valu/wave', int(r['SQ_INSTS_VALU'] / r['SQ_WAVES']), 'salu/wave', int(r['SQ_INSTS_SALU'] / r['SQ_WAVES']))
PY
