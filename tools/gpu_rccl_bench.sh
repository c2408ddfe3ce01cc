#!/bin/bash
# the sharded step path on one GPU: bench.py with a one-rank RCCL communicator (island, exact)
set -o pipefail
export TMPDIR=/tmp NCCL_SOCKET_IFNAME=lo
O=gpurun_out/rb
mkdir -p $O
for m in island exact; do
timeout -k 10 300 python bench.py --no-cpu-baseline --rccl-one-rank --shard-mode $m > $O/$m.json 2> $O/$m.err || { tail -30 $O/$m.err; exit 1; }
python -c "import json;d=json.load(open('$O/$m.json'));b=d['breakdown_ms_per_run'];print('$m', round(d['value']/1e9,2), 'G/s', round(d['ms_per_step'],3), 'ms/run', b and {k: round(v,3) for k,v in b.items() if isinstance(v,float)})"
done
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 > $O/plain.json 2> $O/plain.err || { tail -30 $O/plain.err; exit 1; }
echo "plain stdout lines: $(wc -l < $O/plain.json)"; echo "island stdout lines: $(wc -l < $O/island.json)"
