set -o pipefail
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -q -m gpu -x --timeout 600 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -40 $O/pytest_gpu.txt; exit 1; }
tail -1 $O/pytest_gpu.txt
bash tools/ab_env.sh $1_mv WSMC_DIAG_MV_TABLES_GLOBAL=1 c3gated c5async && bash tools/ab_env_bench.sh $1_st WSMC_DIAG_MV_TABLES_GLOBAL=1 --statements
