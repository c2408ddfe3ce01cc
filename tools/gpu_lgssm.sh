#!/bin/bash
# parity (pytest -m gpu), the default bench line (with the CPU baseline legs), and the
# reference's own LGSSM benchmark (tools/bench_lgssm.py: GPU statements + CPU fast port)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/lg
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $O/pytest.log | head -100; exit $rc; }
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 400 python -u tools/bench_lgssm.py > $O/lgssm.jsonl 2> $O/lgssm.err || { tail $O/lgssm.err; exit 1; }
cat $O/lgssm.jsonl
