# A/B of an environment switch on one box: tools/ab_env.sh <tag> <VAR=value> <bench_moves legs...>:
# the legs without and with the setting, alternated twice
set -o pipefail
# the switches are read by the diagnostic build only (python tools/build_variant.py diag -DWSMC_DIAG_BUILD):
# both legs run it, so the A/B isolates the switch
export WSMC_LIB=${WSMC_LIB:-tools/variants/diag/libwsmc.so}
[ -f "$WSMC_LIB" ] || { echo "no diagnostic build at $WSMC_LIB"; exit 2; }
O=gpurun_out/$1; E=$2; shift 2; mkdir -p $O
for r in 1 2; do
  timeout -k 10 300 python tools/bench_moves.py "$@" > $O/a$r.jsonl 2> $O/a$r.err || { tail $O/a$r.err; exit 1; }
  env $E timeout -k 10 300 python tools/bench_moves.py "$@" > $O/b$r.jsonl 2> $O/b$r.err || { tail $O/b$r.err; exit 1; }
done
for f in a1 b1 a2 b2; do python -c "import json,sys; [print(sys.argv[1][-2:], json.loads(l)['config'][:30], round(json.loads(l)['seconds_per_run']*1e3,4), 'ms') for l in open(sys.argv[1]+'.jsonl')]" $O/$f; done
