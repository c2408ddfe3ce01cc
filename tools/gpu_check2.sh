#!/bin/bash
# whole GPU suite, the default bench line, and the one-rank RCCL (sharded path) bench line
set -o pipefail
export TMPDIR=/tmp NCCL_SOCKET_IFNAME=lo
O=gpurun_out/c2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $O/pytest.log | head -100; exit $rc; }
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print('single', round(d['value']/1e9,2), 'G/s', round(d['ms_per_step'],3), 'ms/run')"
timeout -k 10 300 python bench.py --no-cpu-baseline --rccl-one-rank > $O/island.json 2> $O/island.err || { tail -30 $O/island.err; exit 1; }
python -c "import json;d=json.load(open('$O/island.json'));print('one-rank RCCL island', round(d['value']/1e9,2), 'G/s', round(d['ms_per_step'],3), 'ms/run')"
