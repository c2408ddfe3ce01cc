#!/bin/bash
# SQ cycle split (issue vs parked vs stalled) and instruction mix of the fused run's kernels,
# at 1M and 8M particles (one pass each; counters per dispatch, summed over the XCDs)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/sq
rm -rf $O; mkdir -p $O
for n in 1000000 8000000; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES --output-format csv -d $O/n$n -o run -- python bench.py --particles $n --steps 1 --warmup 1 --no-cpu-baseline > $O/n$n.log 2>&1 || { tail -20 $O/n$n.log; exit 1; }
  python tools/summarize_pmc.py $O/n$n.json $O/n$n > /dev/null
  python - $O/n$n.json $n <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k, r in d.items():
    if not any(x in k for x in ('prop', 'fill', 'sums', 'final')): continue
    wc = r['SQ_WAVE_CYCLES']
    print(sys.argv[2], k[:34], 'waves', int(r['SQ_WAVES']), 'cyc/wave', int(wc / r['SQ_WAVES']),
          'active %.2f wait %.2f stall %.2f valu-active %.2f' % (r['SQ_ACTIVE_INST_ANY'] / wc, r['SQ_WAIT_ANY'] / wc,
          r['SQ_WAIT_INST_ANY'] / wc, r['SQ_ACTIVE_INST_VALU'] / wc),
          'valu/wave', int(r['SQ_INSTS_VALU'] / r['SQ_WAVES']), 'salu/wave', int(r['SQ_INSTS_SALU'] / r['SQ_WAVES']))
PY
done
