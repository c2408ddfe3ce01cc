# A/B on one box: tools/ab.sh <tag> <variant> <bench_moves legs...>: the default library and
# tools/variants/<variant>/libwsmc.so, alternated twice
set -o pipefail
O=gpurun_out/$1; V=$2; shift 2; mkdir -p $O
for r in 1 2; do
  timeout -k 10 300 python tools/bench_moves.py "$@" > $O/a$r.jsonl 2> $O/a$r.err || { tail $O/a$r.err; exit 1; }
  WSMC_LIB=tools/variants/$V/libwsmc.so timeout -k 10 300 python tools/bench_moves.py "$@" > $O/b$r.jsonl 2> $O/b$r.err || { tail $O/b$r.err; exit 1; }
done
for f in $O/a1 $O/b1 $O/a2 $O/b2; do python -c "import json,sys; [print(sys.argv[1][-2:], json.loads(l)['config'][:30], round(json.loads(l)['seconds_per_run']*1e3,4), 'ms') for l in open(sys.argv[1]+'.jsonl')]" $f; done
