#!/bin/bash
# the sharded run's eager fallback after a failed capture (one-rank RCCL), then the one-rank tests
set -o pipefail
export TMPDIR=/tmp NCCL_SOCKET_IFNAME=lo
O=gpurun_out/fb
mkdir -p $O
WSMC_DIAG_CAPTURE_FAIL=1 timeout -k 10 300 python bench.py --no-cpu-baseline --rccl-one-rank --steps 3 > $O/fb.json 2> $O/fb.err || { tail -30 $O/fb.err; exit 1; }
grep -c "running it eagerly" $O/fb.err
python -c "import json;d=json.load(open('$O/fb.json'));print('fallback', round(d['value']/1e9,2), 'G/s', d['log_evidence_last'])"
timeout -k 10 300 python -u -m pytest tests/test_gpu_multishard.py -x -q -m gpu -k one_rank --timeout 200 --timeout-method thread > $O/r1.log 2>&1; rc=$?
tail -2 $O/r1.log; exit $rc
