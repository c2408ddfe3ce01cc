#!/bin/bash
# SQ counters over the C3 move program (per-kernel instruction mix, wave cycles, waits)
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d gpurun_out/sqm -o run -- python tools/bench_moves.py ${WHICH:-c3} > gpurun_out/sqm.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_FLAT SQ_INSTS_LDS --output-format csv -d gpurun_out/sqm2 -o run -- python tools/bench_moves.py ${WHICH:-c3} > gpurun_out/sqm2.log 2>&1
python tools/summarize_pmc.py gpurun_out/sqm_summary.json gpurun_out/sqm > /dev/null
python tools/summarize_pmc.py gpurun_out/sqm2_summary.json gpurun_out/sqm2 > /dev/null
python - <<'PY'
import json
d = json.load(open('gpurun_out/sqm_summary.json')); d2 = json.load(open('gpurun_out/sqm2_summary.json'))
for k, r in d.items():
    if 'move' not in k and 'moments' not in k: continue
    w = r['SQ_WAVES']; r2 = d2.get(k, {})
    print(k.split('(')[0][-20:], 'waves', int(w), 'valu/wave %.0f' % (r['SQ_INSTS_VALU'] / w), 'salu/wave %.0f' % (r['SQ_INSTS_SALU'] / w),
          'smem/wave %.0f' % (r['SQ_INSTS_SMEM'] / w), 'wave_cyc/wave %.0f' % (r['SQ_WAVE_CYCLES'] / w),
          'wait %.2f' % (r['SQ_WAIT_INST_ANY'] / r['SQ_WAVE_CYCLES']), 'valu_active %.2f' % (r['SQ_ACTIVE_INST_VALU'] / r['SQ_WAVE_CYCLES']),
          ' '.join('%s/wave %.0f' % (x.replace('SQ_INSTS_', ''), r2[x] / w) for x in r2 if x.startswith('SQ_INSTS')))
PY
