#!/bin/bash
# one SQ-counter pass over the bench (per-kernel instruction mix, wave cycles, waits)
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d gpurun_out/sq -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/sq.log 2>&1
python tools/summarize_pmc.py gpurun_out/sq_summary.json gpurun_out/sq > /dev/null
python - <<'PY'
import json
d = json.load(open('gpurun_out/sq_summary.json'))
for k, r in d.items():
    if r.get('dispatches', 0) < 50: continue
    w = r['SQ_WAVES']
    print(k.split('(')[0][-28:], 'waves', int(w), 'valu/wave %.0f' % (r['SQ_INSTS_VALU'] / w), 'salu/wave %.0f' % (r['SQ_INSTS_SALU'] / w),
          'lds/wave %.0f' % (r['SQ_INSTS_LDS'] / w), 'wave_cyc/wave %.0f' % (r['SQ_WAVE_CYCLES'] / w),
          'wait_inst %.2f' % (r['SQ_WAIT_INST_ANY'] / r['SQ_WAVE_CYCLES']), 'valu_active %.2f' % (r['SQ_ACTIVE_INST_VALU'] / r['SQ_WAVE_CYCLES']),
          'busy_cyc', int(r['SQ_BUSY_CYCLES']))
PY
