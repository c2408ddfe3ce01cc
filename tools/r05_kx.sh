set -o pipefail
O=gpurun_out/$1; mkdir -p $O
bash tools/ab_env.sh $1_k1 WSMC_DIAG_MV_K1=1 c5async && bash tools/ab_env.sh $1_w4 WSMC_DIAG_MV_WAVES=4 c5async
