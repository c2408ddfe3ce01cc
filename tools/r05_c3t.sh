set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $O/t -o run -- python tools/bench_moves.py c3gated > $O/t.log 2>&1 || { tail -20 $O/t.log; exit 1; }
python tools/timeline.py $O/t/run_kernel_trace.csv wsmc_ew_p 12
ls $O/t
