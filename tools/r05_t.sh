set -o pipefail
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 600 --timeout-method thread --durations=15 > $O/pytest_gpu.txt 2>&1 || { tail -40 $O/pytest_gpu.txt; exit 1; }
tail -1 $O/pytest_gpu.txt
bash tools/gpu_quick.sh $1b "" ""
