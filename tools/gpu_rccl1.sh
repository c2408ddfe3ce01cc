#!/bin/bash
# the one-rank RCCL tests first (new), then the whole GPU suite
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r1
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_multishard.py -x -v -m gpu -k one_rank --timeout 200 --timeout-method thread > $O/rccl1.log 2>&1; rc=$?
tail -5 $O/rccl1.log
[ $rc -eq 0 ] || { grep -B5 -A60 "FAILED\|Error\|NCCL" $O/rccl1.log | head -150; exit $rc; }
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $O/pytest.log | head -100; exit $rc; }
