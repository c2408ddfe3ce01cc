set -o pipefail
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -q -m gpu -x --timeout 600 --timeout-method thread --durations=5 > $O/pytest_gpu.txt 2>&1 || { tail -40 $O/pytest_gpu.txt; exit 1; }
tail -3 $O/pytest_gpu.txt
timeout -k 10 300 python tools/bench_moves.py c3gated c5 c5async > $O/moves.jsonl 2> $O/moves.err || { tail $O/moves.err; exit 1; }
cut -c1-250 $O/moves.jsonl
timeout -k 10 200 python tools/host_prof.py 4096 > $O/hp.txt 2>&1 || { tail $O/hp.txt; exit 1; }
head -1 $O/hp.txt
