#!/bin/bash
# Move-kernel variants: parity of every -m gpu test, then C3 / C5 rates with the lean fold
# (default), the lean fold at one particle per thread, and the generic fold.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/lean
rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $O/pytest.log | head -80; exit $rc; }
r() { timeout -k 10 300 env $1 python tools/bench_moves.py $2 > $O/$3.json 2> $O/$3.err || { tail $O/$3.err; exit 1; }
      python -c "import json,sys
for l in open(sys.argv[1]): d=json.loads(l); print(sys.argv[2], d['config'][:60], round(d['seconds_per_run']*1e3,3), 'ms/run')" $O/$3.json $3; }
r X=0 "c3 c3async" c3_lean
r WSMC_DIAG_MOVE_K=1 "c3 c3async" c3_lean_k1
r WSMC_DIAG_MOVE_GENERIC=1 "c3 c3async" c3_generic
r X=0 c5 c5_lean
r WSMC_DIAG_MOVE_GENERIC=1 c5 c5_generic
