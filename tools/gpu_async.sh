#!/bin/bash
# async Resample parity, then the whole GPU suite, then the LGSSM statement timings
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/as
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "async or lgssm" --timeout 200 --timeout-method thread > $O/as.log 2>&1; rc=$?
tail -2 $O/as.log
[ $rc -eq 0 ] || { grep -B5 -A60 "FAILED\|Error" $O/as.log | head -120; exit $rc; }
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $O/pytest.log | head -100; exit $rc; }
timeout -k 10 300 python -u tools/bench_lgssm.py gpu gpu_wait > $O/lg.jsonl 2> $O/lg.err || { tail $O/lg.err; exit 1; }
cat $O/lg.jsonl
