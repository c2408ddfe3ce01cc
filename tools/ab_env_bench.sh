# A/B of an environment switch on bench.py, one box: tools/ab_env_bench.sh <tag> <VAR=value> [bench args]
set -o pipefail
# the switches are read by the diagnostic build only (python tools/build_variant.py diag -DWSMC_DIAG_BUILD):
# both legs run it, so the A/B isolates the switch
export WSMC_LIB=${WSMC_LIB:-tools/variants/diag/libwsmc.so}
[ -f "$WSMC_LIB" ] || { echo "no diagnostic build at $WSMC_LIB"; exit 2; }
O=gpurun_out/$1; E=$2; shift 2; mkdir -p $O
for r in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/a$r.json 2> $O/a$r.err || { tail $O/a$r.err; exit 1; }
  env $E timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/b$r.json 2> $O/b$r.err || { tail $O/b$r.err; exit 1; }
done
for f in a1 b1 a2 b2; do python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1][-7:], '%.4g' % d['value'], round(d['ms_per_step'],4), 'ms')" $O/$f.json; done
