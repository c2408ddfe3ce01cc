set -o pipefail
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -q -m gpu -x --timeout 600 --timeout-method thread --durations=5 > $O/pytest_gpu.txt 2>&1 || { tail -40 $O/pytest_gpu.txt; exit 1; }
tail -7 $O/pytest_gpu.txt
timeout -k 10 300 python tools/bench_moves.py c5 c3gated > $O/moves.jsonl 2> $O/moves.err || { tail $O/moves.err; exit 1; }
cut -c1-250 $O/moves.jsonl
WSMC_DIAG_MV_WAVES=4 timeout -k 10 300 python tools/bench_moves.py c5 > $O/moves_w4.jsonl 2> $O/moves_w4.err || { tail $O/moves_w4.err; exit 1; }
cut -c1-250 $O/moves_w4.jsonl
