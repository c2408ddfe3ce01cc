#!/bin/bash
# statement-path latency: the LGSSM statements with and without spinning host waits
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/sp
mkdir -p $O
WSMC_SYNC_SPIN=0 timeout -k 10 300 python -u tools/bench_lgssm.py gpu > $O/nospin.json 2> $O/nospin.err || { tail $O/nospin.err; exit 1; }
WSMC_SYNC_SPIN=1 timeout -k 10 300 python -u tools/bench_lgssm.py gpu > $O/spin.json 2> $O/spin.err || { tail $O/spin.err; exit 1; }
cat $O/nospin.json $O/spin.json
WSMC_SYNC_SPIN=1 timeout -k 10 300 python -u tools/bench_moves.py c3 > $O/c3.json 2> $O/c3.err || { tail $O/c3.err; exit 1; }
cat $O/c3.json
