set -o pipefail
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -q -m gpu -x --timeout 600 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -40 $O/pytest_gpu.txt; exit 1; }
tail -1 $O/pytest_gpu.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
echo smoke ok
bash tools/ab_env.sh $1_k1 WSMC_DIAG_MV_K1=1 c5async && bash tools/ab_env.sh $1_w4 WSMC_DIAG_MV_WAVES=4 c5async
