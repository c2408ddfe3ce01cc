#!/bin/bash
# Move kernels: parity subset + C3/C5 timing per library variant
set -e
mkdir -p gpurun_out
for v in ${VARIANTS:-base inl}; do
  if [ "$v" = base ]; then unset WSMC_LIB; else export WSMC_LIB=$PWD/tools/variants/libwsmc_$v.so; fi
  timeout -k 10 600 python -m pytest tests/test_gpu_parity.py tests/test_gpu_multishard.py tests/test_reference_ports.py -q -m gpu -x -k "move or Move or c3 or c5 or port" > gpurun_out/mvv_$v.log 2>&1 || { tail -20 gpurun_out/mvv_$v.log; exit 1; }
  echo "$v parity: $(tail -1 gpurun_out/mvv_$v.log)"
  timeout -k 10 600 python tools/bench_moves.py > gpurun_out/mvv_$v.json 2>gpurun_out/mvv_$v.err || { tail -5 gpurun_out/mvv_$v.err; exit 1; }
  python -c "
import json
for l in open('gpurun_out/mvv_$v.json'):
    d=json.loads(l); print('$v', d['config'][:3], round(d['seconds_per_run']*1e3,3), 'ms/run', '%.3g' % d['particle_steps_per_s'])"
done
