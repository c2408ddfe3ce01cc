#!/bin/bash
# one-rank RCCL parity (fused island run now graph-captured), then the sharded step timing
set -o pipefail
export TMPDIR=/tmp NCCL_SOCKET_IFNAME=lo
O=gpurun_out/rg
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_multishard.py -x -v -m gpu -k one_rank --timeout 200 --timeout-method thread > $O/rccl1.log 2>&1; rc=$?
tail -4 $O/rccl1.log
[ $rc -eq 0 ] || { grep -B5 -A60 "FAILED\|Error\|NCCL" $O/rccl1.log | head -150; exit $rc; }
timeout -k 10 300 python bench.py --no-cpu-baseline --rccl-one-rank > $O/island.json 2> $O/island.err || { tail -30 $O/island.err; exit 1; }
python -c "import json;d=json.load(open('$O/island.json'));print('island graph', round(d['value']/1e9,2), 'G/s', round(d['ms_per_step'],3), 'ms/run')"
WSMC_DIAG_NO_GRAPH=1 timeout -k 10 300 python bench.py --no-cpu-baseline --rccl-one-rank > $O/island_eager.json 2> $O/island_eager.err || { tail -30 $O/island_eager.err; exit 1; }
python -c "import json;d=json.load(open('$O/island_eager.json'));print('island eager', round(d['value']/1e9,2), 'G/s', round(d['ms_per_step'],3), 'ms/run')"
