#!/bin/bash
# move parity (pytest -m gpu -k move/score/oscillator/linreg) then the C3/C5 move configs
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/mv
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/mv/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/mv/pytest.log
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" gpurun_out/mv/pytest.log | head -100; exit $rc; }
timeout -k 10 600 python tools/bench_moves.py > gpurun_out/mv/moves.json 2> gpurun_out/mv/moves.err || { tail -20 gpurun_out/mv/moves.err; exit 1; }
cat gpurun_out/mv/moves.json
