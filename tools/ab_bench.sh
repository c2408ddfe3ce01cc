# A/B of bench.py on one box: tools/ab_bench.sh <tag> <variant> [bench args]: the default library
# and tools/variants/<variant>/libwsmc.so alternated twice, plus a kernel-stats pass of each
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1; V=$2; shift 2; mkdir -p $O
for r in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/a$r.json 2> $O/a$r.err || { tail $O/a$r.err; exit 1; }
  WSMC_LIB=tools/variants/$V/libwsmc.so timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/b$r.json 2> $O/b$r.err || { tail $O/b$r.err; exit 1; }
done
for f in a1 b1 a2 b2; do python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1][-7:], '%.4g' % d['value'], round(d['ms_per_step'],4), 'ms')" $O/$f.json; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/sa -o run -- python bench.py --no-cpu-baseline --steps 20 --warmup 2 "$@" > $O/sa.log 2>&1 || exit 1
WSMC_LIB=tools/variants/$V/libwsmc.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/sb -o run -- python bench.py --no-cpu-baseline --steps 20 --warmup 2 "$@" > $O/sb.log 2>&1 || exit 1
for d in sa sb; do echo $d; head -6 $O/$d/run_kernel_stats.csv | cut -d, -f1-6; done
