#!/bin/bash
# quick GPU iteration: a pytest subset, then the bench line with its per-kernel breakdown
#   tools/gpu_quick.sh <tag> "<pytest args>" "<bench args>"
set -o pipefail
tag=$1; O=gpurun_out/$tag; mkdir -p $O
if [ -n "$2" ]; then
  timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread $2 > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
  tail -2 $O/pytest.txt
fi
timeout -k 10 300 python bench.py --no-cpu-baseline $3 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));b=d['breakdown_ms_per_run'] or {};print('%.4g'%d['value'],'%.3f ms/run'%d['ms_per_run'],{k:(round(v*1e3/100,2) if isinstance(v,float) else v) for k,v in b.items()})"
