set -o pipefail
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_moves_accept.py -q -m gpu -x --timeout 600 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -40 $O/pytest_gpu.txt; exit 1; }
tail -1 $O/pytest_gpu.txt
timeout -k 10 300 python tools/bench_moves.py c3gated c5 c5async > $O/moves.jsonl 2> $O/moves.err || { tail $O/moves.err; exit 1; }
cut -c1-250 $O/moves.jsonl
bash tools/gpu.sh rccl $1_rccl && bash tools/gpu.sh multirank $1_mr
