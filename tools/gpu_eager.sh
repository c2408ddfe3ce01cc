#!/bin/bash
# graph replay vs the same run enqueued eagerly (host submission rate; the multi-GPU path is eager)
set -o pipefail
mkdir -p gpurun_out/eager
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/eager/graph.json 2> gpurun_out/eager/graph.err || exit 1
WSMC_DIAG_NO_GRAPH=1 timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/eager/eager.json 2> gpurun_out/eager/eager.err || exit 1
for f in graph eager; do python -c "import json;d=json.load(open('gpurun_out/eager/$f.json'));print('$f', round(d['value']/1e9,2), 'G/s', round(d['ms_per_step'],3), 'ms/run')"; done
