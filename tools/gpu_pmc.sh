#!/bin/bash
# PMC passes for the fused 2D SSM run (one counter group per rocprofv3 invocation).
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
ARGS="--steps 2 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY --output-format csv -d gpurun_out/pmc/sq -o run -- python bench.py $ARGS > gpurun_out/pmc/sq.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc/fetch -o run -- python bench.py $ARGS > gpurun_out/pmc/fetch.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc/write -o run -- python bench.py $ARGS > gpurun_out/pmc/write.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES TA_BUSY_avr --output-format csv -d gpurun_out/pmc/busy -o run -- python bench.py $ARGS > gpurun_out/pmc/busy.log 2>&1 || true
ls gpurun_out/pmc/*/
