set -o pipefail
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_interp.py tests/test_gpu_parity.py tests/test_gpu_multishard.py -q -m gpu -x --timeout 600 --timeout-method thread --durations=5 > $O/pytest_gpu.txt 2>&1 || { tail -40 $O/pytest_gpu.txt; exit 1; }
tail -7 $O/pytest_gpu.txt
timeout -k 10 400 python tools/bench_moves.py c5 c3gated > $O/moves.jsonl 2> $O/moves.err || { tail $O/moves.err; exit 1; }
cut -c1-250 $O/moves.jsonl
