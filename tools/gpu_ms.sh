#!/bin/bash
# the multi-shard GPU tests first, then the whole GPU suite
set -o pipefail
export TMPDIR=/tmp NCCL_SOCKET_IFNAME=lo
O=gpurun_out/ms
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_multishard.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/ms.log 2>&1; rc=$?
tail -2 $O/ms.log
[ $rc -eq 0 ] || { grep -B5 -A60 "FAILED\|Error" $O/ms.log | head -150; exit $rc; }
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $O/pytest.log | head -100; exit $rc; }
