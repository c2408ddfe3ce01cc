#!/bin/bash
# Full GPU validation: pytest -m gpu, smoke(), bench (default args), rocprof kernel stats.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo PYTEST=$rc >> gpurun_out/pytest_gpu.log; tail -4 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; echo SMOKE=$?; tail -2 gpurun_out/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err; echo BENCH=$?; cat gpurun_out/bench_default.json
