#!/bin/bash
# parity, then the 1M bench, then the 8M bench and the 8M resample-kernel ablations
set -o pipefail
bash tools/gpu_quick.sh || exit 1
mkdir -p gpurun_out/b8
timeout -k 10 300 python bench.py --no-cpu-baseline --particles 8000000 --steps 3 --warmup 1 > gpurun_out/b8/bench.json 2> gpurun_out/b8/err || exit 1
python -c "import json;d=json.load(open('gpurun_out/b8/bench.json'));b=d['breakdown_ms_per_run'];print('8M', round(d['value']/1e9,2), 'G/s', round(d['ms_per_step'],3), 'ms/run; prop/stats/fill us', round(b['propagate']*10,2), round(b['weight_stats']*10,2), round(b['scan_ancestors']*10,2), 'traceback ms', round(b['finalize_traceback'],3))"
timeout -k 10 300 python tools/ablate.py 8000000 > gpurun_out/b8/ab.txt 2>&1 || exit 1
grep "kernel 2" gpurun_out/b8/ab.txt
