set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/df; mkdir -p $O
summ() { python -c "import json,sys;d=json.load(open(sys.argv[1]));b=d['breakdown_ms_per_run'];T=d['config']['T'];print(sys.argv[2], round(d['value']/1e9,2), 'G/s', 'prop/stats/fill us', round(b['propagate']*1e3/T,2), round(b['weight_stats']*1e3/T,2), round(b['scan_ancestors']*1e3/T,2))" $1 $2; }
for m in 0 1; do
 WSMC_DIAG_FILL=$m timeout -k 10 300 python bench.py --no-cpu-baseline > $O/b$m.json 2> $O/b$m.err || { tail $O/b$m.err; exit 1; }
 summ $O/b$m.json "1M diag$m"
 WSMC_DIAG_FILL=$m timeout -k 10 300 python bench.py --no-cpu-baseline --particles 8000000 --steps 3 --warmup 1 > $O/c$m.json 2> $O/c$m.err || { tail $O/c$m.err; exit 1; }
 summ $O/c$m.json "8M diag$m"
done
