set -o pipefail
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_multishard.py -q -m gpu -x --timeout 300 --timeout-method thread -k "lone or symmetric or failure" > $O/p.txt 2>&1 || { tail -30 $O/p.txt; exit 1; }
tail -1 $O/p.txt
timeout -k 10 400 python tools/bench_moves.py c3gated c5 > $O/moves.jsonl 2>$O/moves.err || { tail $O/moves.err; exit 1; }
cut -c1-60,180-270 $O/moves.jsonl
bash tools/gpu.sh c5flops $1f
