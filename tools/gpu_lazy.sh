#!/bin/bash
# GPU parity (all -m gpu tests) + the C2 statement-path bench (lazy) beside the fused run
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/lazy
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $O/pytest.log | head -80; exit $rc; }
bash tools/gpu_stmt.sh
