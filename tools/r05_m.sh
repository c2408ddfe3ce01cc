set -o pipefail
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_expr.py tests/test_gpu_parity.py -q -m gpu -x --timeout 600 --timeout-method thread --durations=8 -k "expr or operator or move_block or oscillator or filter" > $O/pytest_gpu.txt 2>&1 || { tail -40 $O/pytest_gpu.txt; exit 1; }
tail -12 $O/pytest_gpu.txt
timeout -k 10 400 python tools/bench_moves.py c3 c5 > $O/moves.jsonl 2> $O/moves.err || { tail $O/moves.err; exit 1; }
cut -c1-300 $O/moves.jsonl
