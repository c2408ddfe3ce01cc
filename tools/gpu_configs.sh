#!/bin/bash
# the non-headline configs of SURVEY.md §8(d): C2 at the example's ess 0.5, C3, C5 (systematic,
# stratified, and the example as written: ess 0.5, 1 sweep, diversity-gated)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/cfg
mkdir -p $O
timeout -k 10 300 python bench.py --ess 0.5 --no-cpu-baseline > $O/c2_ess05.json 2> $O/c2_ess05.err || { tail $O/c2_ess05.err; exit 1; }
python -c "import json;d=json.load(open('$O/c2_ess05.json'));print('c2 ess0.5', round(d['value']/1e9,2), 'G/s resamples', d['breakdown_ms_per_run']['resamples_per_run'])"
timeout -k 10 600 python -u tools/bench_moves.py c3 c5 c5_stratified c5_example > $O/moves.jsonl 2> $O/moves.err || { tail $O/moves.err; exit 1; }
cat $O/moves.jsonl
