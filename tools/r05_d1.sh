set -o pipefail
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -q -m gpu -x --timeout 600 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -40 $O/pytest_gpu.txt; exit 1; }
tail -1 $O/pytest_gpu.txt
bash tools/ab.sh $1_ab mom_d1 c5async c3gated_moves
