# ablation timings of the Move kernels (tools/build_variant.sh builds; WSMC_LIB selects):
#   bash tools/abl_moves.sh <tag> <bench_moves config> <variant>...   (variant "base" = the library)
set -o pipefail
export TMPDIR=/tmp
tag=$1; cfg=$2; shift 2
O=gpurun_out/$tag; mkdir -p $O
for v in "$@"; do
  if [ $v = base ]; then L=weightedsampling.jl_amd/wsmc/libwsmc.so; else L=tools/variants/libwsmc_$v.so; fi
  WSMC_LIB=$PWD/$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python tools/bench_moves.py $cfg > $O/$v.log 2>&1 || { echo FAIL $v; tail -20 $O/$v.log; exit 1; }
  python - $O/$v <<'PY'
import csv, json, sys
d = sys.argv[1]
line = [l for l in open(d + '.log') if l.startswith('{')][0]
rows = sorted(csv.DictReader(open(d + '/run_kernel_stats.csv')), key=lambda r: -float(r['TotalDurationNs']))
print(d.split('/')[-1], 's/run %.5f' % json.loads(line)['seconds_per_run'],
      ' '.join('%s=%.1fus' % (r['Name'].split('(')[0].split('::')[-1][:24], float(r['AverageNs']) / 1e3) for r in rows[:5]))
PY
done
