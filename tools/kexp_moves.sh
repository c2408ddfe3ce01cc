set -o pipefail
mkdir -p gpurun_out/r04_kx
for k in 1 2 4; do
  WSMC_DIAG_MV_K=$k timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04_kx/k$k -o run -- python tools/bench_moves.py c3gated > gpurun_out/r04_kx/k$k.log 2>&1 || { echo FAIL $k; tail -5 gpurun_out/r04_kx/k$k.log; exit 1; }
  python - gpurun_out/r04_kx/k$k <<'PY'
import csv, json, sys
d = sys.argv[1]
line = [l for l in open(d + '.log') if l.startswith('{')][0]
rows = [r for r in csv.DictReader(open(d + '/run_kernel_stats.csv')) if 'wsmc_mv' in r['Name']]
print(d, 's/run %.5f' % json.loads(line)['seconds_per_run'], ' '.join('%s=%.1fus' % (r['Name'], float(r['AverageNs']) / 1e3) for r in rows))
PY
done
