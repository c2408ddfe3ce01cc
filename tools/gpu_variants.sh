#!/bin/bash
# Block-size variants: parity subset + bench per variant (tools/build_variant.sh builds them).
set -e
mkdir -p gpurun_out
for v in ${VARIANTS:-base s512 u512 both512 s128}; do
  if [ "$v" = base ]; then unset WSMC_LIB; else export WSMC_LIB=$PWD/tools/variants/libwsmc_$v.so; fi
  timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -m gpu -x -k "fused or skewed or statements" > gpurun_out/var_$v.log 2>&1 || { tail -20 gpurun_out/var_$v.log; exit 1; }
  echo "$v parity: $(tail -1 gpurun_out/var_$v.log)"
  for i in 1 2; do
    timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/vb_$v.json 2>/dev/null
    python -c "import json; d=json.load(open('gpurun_out/vb_$v.json')); b=d['breakdown_ms_per_run']; print('$v', round(d['value']/1e10,4), round(b['propagate'],3), round(b['weight_stats'],3), round(b['scan_ancestors'],3))"
  done
done
