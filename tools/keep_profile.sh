#!/bin/bash
# Copy the judged artefacts of one tools/gpu.sh run (gpurun_out/<tag>/) into profiles/ as
# profiles/<tag>_<name>: JSON lines and summaries, kernel statistics, test logs, the MANIFEST.
#   tools/keep_profile.sh <tag>
tag=$1; O=gpurun_out/$tag
[ -d "$O" ] || { echo "no $O"; exit 1; }
cd "$(dirname "$0")/.." || exit 1
for f in MANIFEST bench.json bench_statements.json pmc_summary.json pmc_step_bytes.json moves.jsonl c5_flops.json \
         pytest_gpu.log smoke.log island.json exact.json p.json n1000000.json n8000000.json \
         mr_island.json mr_exact.json mr_strong.json mh_island.json mh_exact.json; do
  [ -f "$O/$f" ] && cp "$O/$f" "profiles/${tag}_${f/pytest_gpu.log/pytest_gpu.txt}"
done
for d in stats gstats st c3 c5; do
  [ -f "$O/$d/run_kernel_stats.csv" ] && cp "$O/$d/run_kernel_stats.csv" "profiles/${tag}_${d}_kernel_stats.csv"
done
for f in "$O"/*.txt; do [ -f "$f" ] && cp "$f" "profiles/${tag}_$(basename "$f")"; done
# a round's profile passes: bench.py's PMC traffic copies (pmc/) follow them
[ -f "profiles/${tag}_pmc_step_bytes.json" ] && python tools/refresh_pmc.py "$tag"
ls profiles | grep "^${tag}_"
