# A/B of tools/bench_moves.py legs between a library variant and the product library, alternated:
#   tools/ab_moves_libs.sh <tag> <variant> <legs...>
set -o pipefail
O=gpurun_out/$1; V=$2; shift 2; mkdir -p $O
for r in 1 2; do
  WSMC_LIB=tools/variants/$V/libwsmc.so timeout -k 10 300 python tools/bench_moves.py "$@" > $O/a$r.jsonl 2> $O/a$r.err || { tail $O/a$r.err; exit 1; }
  timeout -k 10 300 python tools/bench_moves.py "$@" > $O/b$r.jsonl 2> $O/b$r.err || { tail $O/b$r.err; exit 1; }
done
for f in a1 b1 a2 b2; do python -c "import json,sys; [print(sys.argv[1][-2:], json.loads(l)['config'][:40], round(json.loads(l)['seconds_per_run']*1e3,4), 'ms') for l in open(sys.argv[1]+'.jsonl')]" $O/$f; done
