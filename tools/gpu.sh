#!/bin/bash
# One entry point for every GPU-box recipe whose output lands in profiles/ (run through
# gpurun from the repo root, e.g. gpurun --timeout 900 -- 'bash tools/gpu.sh round r03_v1').
# Each recipe writes gpurun_out/<tag>/ plus a MANIFEST (recipe, arguments, HEAD of the tree
# it ran on, UTC time) so every committed profile traces back to one command. Every GPU step
# runs under its own time limit; the first failing step ends the recipe.
#
#   tests <tag> [pytest args]   pytest -m gpu (default: the whole suite)
#   round <tag>                 pytest -m gpu, smoke(), the default bench line, the statement-path
#                               line, rocprofv3 kernel stats of the bench command, FETCH_SIZE /
#                               WRITE_SIZE passes -> pmc_summary.json, pmc_step_bytes.json
#   prof <tag>                  the round's profile passes alone
#   big <tag>                   the 8M line, its kernel stats and PMC step bytes
#   bench <tag> [bench args]    bench.py line + rocprofv3 kernel stats of the same command
#   moves <tag>                 C3 / C5 move-program lines (tools/bench_moves.py) + C3 kernel stats
#   c5flops <tag>               C5 FP64 work (SQ_INSTS_VALU_*_F64) against its kernel durations
#   sq <tag> fused|c3|c5        SQ cycle split and instruction mix per kernel
#   rccl <tag>                  one-rank RCCL bench lines (island, exact)
#   multirank <tag>             bench.py under torch.distributed.run, 2 ranks on one GPU (host exchange)
#   fallback <tag>              the sharded run's eager fallback after a failed graph capture
#   micro <tag> <name>          run tools/micro/<name> (built here from tools/micro/<name>.hip)
set -o pipefail
export TMPDIR=/tmp
recipe=$1; tag=$2
[ -n "$recipe" ] && [ -n "$tag" ] || { echo "usage: tools/gpu.sh <recipe> <tag> [args]"; exit 2; }
shift 2
O=gpurun_out/$tag
mkdir -p $O
{
  echo "recipe: tools/gpu.sh $recipe $tag $*"
  echo "head: $(cat .git_head 2>/dev/null || echo unknown)"
  echo "utc: $(date -u +%Y-%m-%dT%H:%M:%SZ)"
} > $O/MANIFEST

SQ="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES"
step() {   # step <seconds> <log> <cmd...>: one GPU step, its own limit, tail on failure
  local t=$1 lg=$2; shift 2
  timeout -k 10 "$t" "$@" > "$lg" 2>&1 || { echo "FAILED: $*"; tail -30 "$lg"; exit 1; }
}
stats_table() {   # stats_table <kernel_stats.csv> [n]
  python - "$1" "${2:-12}" <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda x: -float(x['TotalDurationNs']))
for x in rows[:int(sys.argv[2])]:
    print(x['Name'][:56], x['Calls'], round(float(x['AverageNs']) / 1e3, 2), 'us avg', round(float(x['TotalDurationNs']) / 1e6, 3), 'ms total')
PY
}
sq_table() {   # sq_table <summary.json> [name filter]
  python - "$1" "${2:-}" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k, r in d.items():
    if sys.argv[2] and not any(f in k for f in sys.argv[2].split(',')): continue
    wc = r.get('SQ_WAVE_CYCLES', 0); w = r.get('SQ_WAVES', 0)
    if not wc or not w: continue
    print(k[:40], 'waves', int(w), 'cyc/wave', int(wc / w),
          'active %.2f parked %.2f stalled %.2f valu-active %.2f' % (r['SQ_ACTIVE_INST_ANY'] / wc, r['SQ_WAIT_ANY'] / wc,
          r['SQ_WAIT_INST_ANY'] / wc, r['SQ_ACTIVE_INST_VALU'] / wc),
          'valu/wave', int(r['SQ_INSTS_VALU'] / w), 'salu/wave', int(r['SQ_INSTS_SALU'] / w))
PY
}
line() { python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], '%.4g' % d['value'], d['unit'], '%.3f ms/run' % d['ms_per_run'], 'frac %.3f' % d['roofline']['frac'])" "$1" "$2"; }

prof_passes() {   # kernel stats of the bench command at its default 300 runs, submitted eagerly
                  # (WSMC_DIAG_NO_GRAPH=1: the same kernels; rocprofv3's kernel trace segfaults on
                  # graph replays past a few thousand dispatches, tools/micro/graph_trace.hip and
                  # DESIGN.md §4), the graph-launched run's stats at 20 runs beside it, then
                  # FETCH_SIZE / WRITE_SIZE in separate passes
  WSMC_DIAG_NO_GRAPH=1 step 600 $O/stats.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python bench.py --no-cpu-baseline --steps 300
  stats_table $O/stats/run_kernel_stats.csv 6
  step 400 $O/gstats.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/gstats -o run -- python bench.py --no-cpu-baseline --steps 20 --warmup 2
  stats_table $O/gstats/run_kernel_stats.csv 6
  A="--steps 2 --warmup 1 --no-cpu-baseline"
  step 300 $O/fetch.log rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python bench.py $A
  step 300 $O/write.log rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python bench.py $A
  python tools/summarize_pmc.py $O/pmc_summary.json $O/fetch $O/write > /dev/null
  python tools/pmc_step_bytes.py $O/pmc_summary.json 1000000 100 $O/pmc_step_bytes.json
}

case $recipe in
tests)   # [pytest args]: files / -k; the whole suite by default
  [ $# -gt 0 ] || set -- tests
  step 1100 $O/pytest_gpu.log python -u -m pytest -q -m gpu -x --timeout 600 --timeout-method thread "$@"
  tail -1 $O/pytest_gpu.log ;;
evidence)   # the round's measurements without the test suite (run `tests` before it)
  timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  line $O/bench.json bench
  timeout -k 10 400 python bench.py --no-cpu-baseline --statements > $O/bench_statements.json 2> $O/bench_statements.err || { tail -20 $O/bench_statements.err; exit 1; }
  line $O/bench_statements.json statements
  step 300 $O/st.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/st -o run -- python bench.py --no-cpu-baseline --statements --steps 20 --warmup 2
  stats_table $O/st/run_kernel_stats.csv 8
  prof_passes ;;
round)
  step 1100 $O/pytest_gpu.log python -u -m pytest tests -q -m gpu -x --timeout 600 --timeout-method thread
  tail -1 $O/pytest_gpu.log
  step 300 $O/smoke.log python -c "import __graft_entry__ as g; g.smoke()"
  echo smoke ok
  timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  line $O/bench.json bench
  timeout -k 10 400 python bench.py --no-cpu-baseline --statements > $O/bench_statements.json 2> $O/bench_statements.err || { tail -20 $O/bench_statements.err; exit 1; }
  line $O/bench_statements.json statements
  prof_passes ;;
big)    # the beyond-MALL line: 8M particles, its kernel stats and PMC step bytes
  timeout -k 10 400 python bench.py --particles 8000000 --steps 40 --warmup 3 > $O/bench8m.json 2> $O/bench8m.err || { tail -20 $O/bench8m.err; exit 1; }
  line $O/bench8m.json bench-8M
  step 400 $O/stats8m.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats8m -o run -- python bench.py --no-cpu-baseline --particles 8000000 --steps 10 --warmup 2
  stats_table $O/stats8m/run_kernel_stats.csv 6
  A="--particles 8000000 --steps 2 --warmup 1 --no-cpu-baseline"
  step 300 $O/fetch.log rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python bench.py $A
  step 300 $O/write.log rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python bench.py $A
  python tools/summarize_pmc.py $O/pmc_summary8m.json $O/fetch $O/write > /dev/null
  python tools/pmc_step_bytes.py $O/pmc_summary8m.json 8000000 100 $O/pmc_step_bytes8m.json
  cat $O/pmc_step_bytes8m.json ;;
prof)   # the round's profile passes alone (kernel stats, FETCH_SIZE / WRITE_SIZE)
  prof_passes ;;
bench)  timeout -k 10 400 python bench.py "$@" > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  line $O/bench.json bench
  step 400 $O/stats.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python bench.py --no-cpu-baseline --steps 20 --warmup 2 "$@"
  stats_table $O/stats/run_kernel_stats.csv 8 ;;
moves)
  timeout -k 10 400 python tools/bench_moves.py c3 c3async c3gated_moves c3gated c5 c5async c5block c5blockasync c3cpu > $O/moves.jsonl 2> $O/moves.err || { tail $O/moves.err; exit 1; }
  cut -c1-330 $O/moves.jsonl
  step 300 $O/c3.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/c3 -o run -- python tools/bench_moves.py c3gated
  stats_table $O/c3/run_kernel_stats.csv 10
  step 300 $O/c5.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5 -o run -- python tools/bench_moves.py c5
  stats_table $O/c5/run_kernel_stats.csv 8 ;;
c5flops)
  step 600 $O/stats.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python tools/bench_moves.py c5
  step 900 $O/pmc.log rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 --output-format csv -d $O/pmc -o run -- python tools/bench_moves.py c5
  python tools/summarize_pmc.py $O/pmc_summary.json $O/pmc > /dev/null
  python tools/c5_flops.py $O ;;
sq)
  case $1 in
    fused) for n in 1000000 8000000; do
             step 120 $O/n$n.log rocprofv3 --kernel-trace --pmc $SQ --output-format csv -d $O/n$n -o run -- python bench.py --particles $n --steps 1 --warmup 1 --no-cpu-baseline
             python tools/summarize_pmc.py $O/n$n.json $O/n$n > /dev/null
             sq_table $O/n$n.json prop,fill,sums,final
           done ;;
    c3|c5) w=$1; [ $w = c3 ] && w=c3gated
           step 300 $O/p.log rocprofv3 --kernel-trace --pmc $SQ --output-format csv -d $O/p -o run -- python tools/bench_moves.py $w
           python tools/summarize_pmc.py $O/p.json $O/p > /dev/null
           sq_table $O/p.json ;;
    *) echo "sq: fused|c3|c5"; exit 2 ;;
  esac ;;
ew)   # the statement path (bench.py --statements): its line, kernel stats, FETCH / WRITE and SQ passes
  timeout -k 10 400 python bench.py --no-cpu-baseline --statements "$@" > $O/bench_statements.json 2> $O/bench_statements.err || { tail -20 $O/bench_statements.err; exit 1; }
  line $O/bench_statements.json statements
  step 400 $O/stats.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python bench.py --no-cpu-baseline --statements --steps 20 --warmup 2 "$@"
  stats_table $O/stats/run_kernel_stats.csv 10
  A="--steps 2 --warmup 1 --no-cpu-baseline --statements"
  step 300 $O/fetch.log rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python bench.py $A "$@"
  step 300 $O/write.log rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python bench.py $A "$@"
  python tools/summarize_pmc.py $O/pmc_summary.json $O/fetch $O/write
  step 300 $O/sq.log rocprofv3 --kernel-trace --pmc $SQ --output-format csv -d $O/sq -o run -- python bench.py $A "$@"
  python tools/summarize_pmc.py $O/sq.json $O/sq > /dev/null
  sq_table $O/sq.json ew_batch,lazy_trace,rs_ ;;
segv)  # the r03 crash under the kernel tracer: the libwsmc-free repro on plain stream
       # launches, the bench's default 300 runs submitted eagerly (WSMC_DIAG_NO_GRAPH=1) under the
       # tracer, then the repro's graph replays at R = $1 (a crash ends the recipe: it runs last)
  step 300 $O/stream_trace.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/st -o run -- tools/micro/graph_trace 100 300 1000000 0 0
  tail -1 $O/stream_trace.log
  WSMC_DIAG_NO_GRAPH=1 step 600 $O/stats.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python bench.py --no-cpu-baseline --steps 300
  stats_table $O/stats/run_kernel_stats.csv 6
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/gt -o run -- tools/micro/graph_trace 100 ${1:-100} > $O/graph_trace.log 2>&1
  rc=$?; echo "graph replays R=${1:-100} under the tracer: exit $rc"; tail -1 $O/graph_trace.log ;;
rccl)
  export NCCL_SOCKET_IFNAME=lo
  for m in island exact; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --rccl-one-rank --shard-mode $m "$@" > $O/$m.json 2> $O/$m.err || { tail -30 $O/$m.err; exit 1; }
    line $O/$m.json rccl-one-rank-$m
  done ;;
multirank)   # bench.py's multi-rank path with 2 ranks on the box's one GPU (host exchange: RCCL
             # refuses two ranks on one device): weak island, weak exact, strong (ragged) island
  MR="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1"
  A="--gpus 2 --steps 3 --warmup 1 --no-cpu-baseline --exchange host --same-device"
  timeout -k 10 400 $MR --master-port 29611 bench.py $A --shard-mode island > $O/mr_island.json 2> $O/mr_island.err || { tail -30 $O/mr_island.err; exit 1; }
  line $O/mr_island.json multirank-island
  timeout -k 10 400 $MR --master-port 29612 bench.py $A --shard-mode exact > $O/mr_exact.json 2> $O/mr_exact.err || { tail -30 $O/mr_exact.err; exit 1; }
  line $O/mr_exact.json multirank-exact
  timeout -k 10 400 $MR --master-port 29613 bench.py $A --global-particles 1000001 > $O/mr_strong.json 2> $O/mr_strong.err || { tail -30 $O/mr_strong.err; exit 1; }
  line $O/mr_strong.json multirank-strong
  # the same two shards in one process (one handle, in-process exchange: the device path of
  # the sharded run with a memcpy for the collective), island and exact
  for m in island exact; do
    timeout -k 10 400 python bench.py --multi-shards 2 --steps 5 --warmup 2 --no-cpu-baseline --shard-mode $m > $O/mh_$m.json 2> $O/mh_$m.err || { tail -30 $O/mh_$m.err; exit 1; }
    line $O/mh_$m.json multihandle-$m
  done ;;
fallback)   # the sharded run's eager fallback after a failed capture (one-rank RCCL)
  export NCCL_SOCKET_IFNAME=lo
  WSMC_DIAG_CAPTURE_FAIL=1 timeout -k 10 300 python bench.py --no-cpu-baseline --rccl-one-rank --steps 3 > $O/fb.json 2> $O/fb.err || { tail -30 $O/fb.err; exit 1; }
  grep -c "running it eagerly" $O/fb.err
  line $O/fb.json capture-fallback ;;
abn)   # A/B/n of environment settings on the diagnostic build (python tools/build_variant.py diag
       # -DWSMC_DIAG_BUILD), alternated twice:  abn <tag> "<bench args>" SPEC...  (SPEC: VAR=v[,VAR=v] or base)
  export WSMC_LIB=${WSMC_LIB:-tools/variants/diag/libwsmc.so}
  [ -f "$WSMC_LIB" ] || { echo "no diagnostic build at $WSMC_LIB"; exit 2; }
  args=$1; shift
  for r in 1 2; do
    for spec in "$@"; do
      f=$O/$(echo "$spec" | tr '=,' '__')_$r
      ev=""; [ "$spec" = base ] || ev=$(echo "$spec" | tr ',' ' ')
      env $ev timeout -k 10 300 python bench.py --no-cpu-baseline $args > $f.json 2> $f.err || { tail -20 $f.err; exit 1; }
      python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], '%.4g' % d['value'], round(d['ms_per_step'], 4), 'ms')" $f.json "$spec"
    done
  done ;;
timeline)   # per-kernel durations and the gaps between them over a few graph-replayed runs:
            # timeline <tag> "<bench args>" [kernel filter]
  step 300 $O/t.log rocprofv3 --kernel-trace --output-format csv -d $O/t -o run -- python bench.py --no-cpu-baseline --steps 3 --warmup 1 $1
  python tools/timeline.py $O/t/run_kernel_trace.csv "${2:-void wsmc::k_ssm2d_prop}" 24 ;;
micro)   # the binary is built here (hipcc ... -o tools/micro/<name> tools/micro/<name>.hip): the
         # micro sources do not travel (.gpurunignore)
  name=$1
  step 300 $O/$name.txt tools/micro/$name
  cat $O/$name.txt ;;
*) echo "unknown recipe $recipe"; exit 2 ;;
esac
