set -o pipefail
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -q -m gpu -x --timeout 600 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -40 $O/pytest_gpu.txt; exit 1; }
tail -1 $O/pytest_gpu.txt
timeout -k 10 400 python tools/bench_moves.py c3gated c5 c5async c3gated c5async > $O/moves.jsonl 2> $O/moves.err || { tail $O/moves.err; exit 1; }
python -c "import json; [print(json.loads(l)['config'][:24], round(json.loads(l)['seconds_per_run']*1e3,4)) for l in open('$O/moves.jsonl')]"
bash tools/gpu.sh sq $1_sq c5 | grep -E "mv_|moments"
