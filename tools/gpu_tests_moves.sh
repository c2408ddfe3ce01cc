set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pt
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pt/pytest.log 2>&1; rc=$?
tail -2 gpurun_out/pt/pytest.log
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" gpurun_out/pt/pytest.log | head -80; exit $rc; }
bash tools/gpu_moves_round.sh
