# A/B/n of bench.py over library variants on one box, alternated:
#   tools/ab_libs.sh <tag> "<variant> <variant> ..." [bench args]   (variant "default": the product library)
set -o pipefail
O=gpurun_out/$1; V=$2; shift 2; mkdir -p $O
for r in 1 2; do
  for v in $V; do
    lib=tools/variants/$v/libwsmc.so; [ "$v" = default ] && lib=weightedsampling.jl_amd/wsmc/libwsmc.so
    WSMC_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/$v.$r.json 2> $O/$v.$r.err || { tail $O/$v.$r.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); b=d.get('breakdown_ms_per_run',{}); print(sys.argv[1], '%.4g' % d['value'], round(d['ms_per_step'],4), 'ms', {k: round(x,4) for k,x in b.items() if isinstance(x,float)})" $O/$v.$r.json
  done
done
