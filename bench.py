#!/usr/bin/env python3
"""North-star benchmark: 2D SSM bootstrap filter (examples/2D_ssm.jl), particle-steps/s.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

One bench "step" = one full run! of the T-step filter over one synthetic observation
sequence (T = 100, the BASELINE.json configs[1] workload), including the final
history trace-back that materialises x_1..x_{T+1} exactly as the reference's store holds
them. N = 1,000,000 particles per GPU (weak scaling: each rank owns a 1M shard;
`--global-particles G` splits one population of G over the ranks instead, for C4's strong
scaling, e.g. G = 8,000,000 on 1/2/4/8 GPUs). Island
resampling by default — ranks exchange one statistics payload per step over RCCL;
`--shard-mode exact` resamples the whole population with the single-GPU bits (particles
move between ranks).

`--gpus N` is what the line measures, or the run refuses (exit 2, the reason on stderr):
  * under a launcher (WORLD_SIZE set) WORLD_SIZE must equal N, and each node must see a HIP
    device per local rank (unless `--same-device`, the one-GPU test mode);
  * without a launcher and N > 1, one process drives N devices through one multi-device
    handle (wsmc_create_multi: ncclCommInitAll over devices 0..N-1, peer access, one host
    thread per shard issuing its own collectives, as a process per GPU would); fewer than N
    visible devices is a refusal, never a one-GPU run.
The line's `ranks` object carries what the communicator itself reports (ncclCommCount), the
devices and the particles per shard.

Rank 0 prints ONE JSON line (metric/value/.../roofline/cpu_baseline). Everything else
goes to stderr.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import pathlib
import sys
import time

REPO = pathlib.Path(__file__).resolve().parent
sys.path.insert(0, str(REPO / "weightedsampling.jl_amd"))

import numpy as np  # noqa: E402

METRIC = json.loads((REPO / "BASELINE.json").read_text())["metric"] if (REPO / "BASELINE.json").exists() else \
    "particle-steps/sec (N_particles × T_steps / wall-s), 2D SSM bootstrap filter"
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
PROP_BYTES_STEADY = 76         # propagate kernel, per particle, 2 <= t < T after a resample: the model's state,
PROP_BYTES_Q = 8               # + q, the Resample statistics taken in the same pass, when the propagate stores it
                               # (statistics mode 1, below 3M particles a GPU)
PROP_BYTES_FIRST = 56          # step 1: x0/v0 are constants (read w, write x, v, w, and w for a replay)
PROP_BYTES_LAST_DV = 16        # dv is stored at the last step only
STEP_BYTES = 104               # whole step algorithmic bytes


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# ---- the multi-GPU line's own parity proof ----------------------------
CHECK_PARTICLES = 65536   # per GPU
CHECK_T = 8


def state_digests(ctx, lo, hi):
    """xxh3-64 of the weights and of every column (name order) over particles [lo, hi) of the
    context's view, plus the log evidence's bits: the fingerprint two runs must share."""
    import xxhash
    h = xxhash.xxh3_64()
    for name in sorted(ctx.col_names()):
        a = ctx.col_download(ctx.col_find(name))
        h.update(name.encode())
        h.update(np.ascontiguousarray(a[..., lo:hi]).tobytes())
    h.update(np.ascontiguousarray(ctx.weights_download()[lo:hi]).tobytes())
    return h.hexdigest()


def check_verdict(ref, got, ev_ref, ev_got):
    """ref / got: per-shard digests of the one-GPU context and of the sharded run; the sharded
    line stands only if every shard and the evidence are bit-identical."""
    bad = [g for g, (a, b) in enumerate(zip(ref, got)) if a != b]
    ok = not bad and len(ref) == len(got) and ev_ref == ev_got
    return {"exact_vs_1gpu": ok, "mismatched_shards": bad, "evidence_equal": ev_ref == ev_got,
            "digests": got}


def refuse_on_mismatch(verdict):
    if not verdict["exact_vs_1gpu"]:
        log(f"bench: the sharded run differs from one GPU (shards {verdict['mismatched_shards']}, "
            f"evidence equal: {verdict['evidence_equal']}): refusing the line")
        sys.exit(2)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 1000 runs of T = 100 steps: about 4 s of timed GPU work at 1M (long enough for a sampler
    # outside the process to see the GPU busy, and a steadier per-run figure), still seconds
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--particles", type=int, default=1_000_000, help="particles per GPU (weak scaling)")
    ap.add_argument("--global-particles", type=int, default=0,
                    help="total particles split over the ranks (strong scaling, C4's 8M on 1/2/4/8 GPUs)")
    ap.add_argument("--T", type=int, default=100)
    ap.add_argument("--ess", type=float, default=1.0)
    ap.add_argument("--scheme", choices=["stratified", "systematic", "multinomial"], default="stratified")
    ap.add_argument("--no-history", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-particles", type=int, default=1_000_000, help="all-cores port sample")
    ap.add_argument("--cpu-T", type=int, default=100)
    ap.add_argument("--cpu-threads", type=int, default=0, help="0: OMP_NUM_THREADS or the affinity mask")
    ap.add_argument("--cpu-1t-particles", type=int, default=500_000, help="single-thread statement-oracle sample")
    ap.add_argument("--seed", type=int, default=42)
    # test hooks for the multi-rank code path on a one-GPU box (RCCL refuses two ranks on
    # one device): exchange shard records through the host rendezvous, all ranks on GPU 0
    ap.add_argument("--exchange", choices=["rccl", "host"], default="rccl")
    ap.add_argument("--same-device", action="store_true")
    # island (default): one record all-gather per step, shard-local resampling;
    # exact: population-wide resampling, the single-GPU bits (particles move between ranks)
    ap.add_argument("--shard-mode", choices=["island", "exact"], default="island")
    # diagnostics: one rank with a one-rank RCCL communicator, so the run takes the sharded
    # (eager, RCCL all-gather per step) path on one GPU — the multi-GPU step cost minus xGMI
    ap.add_argument("--rccl-one-rank", action="store_true")
    # the same workload through the generic statement operators (one C-ABI call per statement,
    # the path a Julia run! on HipColumnStore takes) instead of the fused runner; with
    # --eager-store the store gathers every column at every resample, as the reference's
    # ColumnStore does (src/stores.jl:105-128)
    # diagnostics: one process, one multi-device handle of this many shards on GPU 0 with the
    # in-process exchange (wsmc_create_multi, transport HOST): the sharded run's device path
    # with a memcpy for a collective (the one-GPU stand-in for RCCL between ranks); N per shard
    ap.add_argument("--multi-shards", type=int, default=0)
    # a sharded line first proves itself: an exact-shard run of CHECK_PARTICLES a GPU x CHECK_T
    # steps against one context holding that population (digests of every column and weight)
    ap.add_argument("--no-self-check", action="store_true")
    # every stream wait of a sharded run is bounded (wsmc_comm_set_timeout: the communicator is
    # aborted and the run exits non-zero), and the whole process by the double of it
    ap.add_argument("--watchdog", type=float, default=120.0)
    ap.add_argument("--statements", action="store_true")
    ap.add_argument("--eager-store", action="store_true")
    return ap.parse_args()


class LayoutError(Exception):
    """--gpus N cannot be measured as labelled (bench.py exits 2 with this message)."""


def visible_devices_note(env) -> str:
    vis = [f"{k}={env[k]}" for k in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES")
           if k in env]
    return ", ".join(vis) if vis else "no *_VISIBLE_DEVICES set"


def plan_layout(gpus: int, env, device_count, same_device: bool = False, multi_shards: int = 0) -> dict:
    """How `--gpus N` maps onto processes and devices. `device_count()` is called only when
    the answer depends on it (it initialises HIP). Raises LayoutError rather than measure a
    different number of GPUs than the line would say."""
    if gpus < 1:
        raise LayoutError(f"--gpus must be >= 1 (got {gpus})")
    ws = env.get("WORLD_SIZE")
    if ws is not None:
        world = int(ws)
        if world != gpus:
            raise LayoutError(f"--gpus {gpus} but the launcher started WORLD_SIZE={world} ranks: the line would "
                              f"not measure what it labels; launch --nproc-per-node {gpus} or pass --gpus {world}")
        if multi_shards > 1 and world > 1:
            raise LayoutError("--multi-shards is a one-process diagnostic; do not combine it with a launcher")
        local_world = int(env.get("LOCAL_WORLD_SIZE", world))
        if world > 1 and not same_device:
            n = device_count()
            if n < local_world:
                raise LayoutError(f"{local_world} ranks on this node need {local_world} HIP devices (one per rank); "
                                  f"{n} visible ({visible_devices_note(env)})")
        return {"mode": "launcher" if world > 1 else "single", "world": world}
    if gpus > 1:
        if multi_shards > 1:
            raise LayoutError("--multi-shards (shards on GPU 0, host exchange) measures one GPU: use it with --gpus 1")
        n = device_count()
        if n < gpus:
            raise LayoutError(f"--gpus {gpus} needs {gpus} HIP devices; {n} visible ({visible_devices_note(env)}); "
                              f"refusing to measure fewer GPUs than the line would say")
        return {"mode": "in-process", "world": gpus, "devices": list(range(gpus))}
    return {"mode": "single", "world": 1}


def cpu_threads(requested: int) -> int:
    if requested > 0:
        return requested
    env = os.environ.get("OMP_NUM_THREADS", "")
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    return max(1, min(int(env), aff) if env.isdigit() and int(env) > 0 else aff)


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown CPU"


CPU_REPS = 5   # timed all-cores CPU runs after the warm-up; the median is reported


def pin_openmp() -> dict:
    """Bind the CPU ports' OpenMP threads one per core, spread over the whole affinity mask
    (OMP_PLACES=cores, OMP_PROC_BIND=spread): both sockets / NUMA nodes take threads, and the
    threads do not pile onto the first cores of the mask, where other jobs on a shared host
    pack theirs (round 3 bound them `close` and measured 4x apart from box to box). The ports
    first-touch their buffers in the same parallel loops that use them, so every node holds
    the pages its threads work on. Must run before the oracle library (and its OpenMP runtime)
    loads."""
    os.environ.setdefault("OMP_PLACES", "cores")
    os.environ.setdefault("OMP_PROC_BIND", "spread")
    return {"OMP_PLACES": os.environ["OMP_PLACES"], "OMP_PROC_BIND": os.environ["OMP_PROC_BIND"]}


def cpu_topology() -> dict:
    """Physical cores (distinct (package, core) pairs) and NUMA nodes of this process's
    affinity mask, the host's node count and its load average when the ports ran."""
    cpus = sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else []
    cores, nodes = set(), set()
    for c in cpus:
        base = f"/sys/devices/system/cpu/cpu{c}"
        try:
            pkg = open(f"{base}/topology/physical_package_id").read().strip()
            core = open(f"{base}/topology/core_id").read().strip()
            cores.add((pkg, core))
            for e in os.listdir(base):
                if e.startswith("node") and e[4:].isdigit():
                    nodes.add(int(e[4:]))
        except OSError:
            pass
    try:
        total = len([e for e in os.listdir("/sys/devices/system/node") if e.startswith("node") and e[4:].isdigit()])
    except OSError:
        total = None
    try:
        load = [round(x, 2) for x in os.getloadavg()]
    except OSError:
        load = None
    return {"affinity_cpus": len(cpus), "physical_cores": len(cores) or None, "nodes_used": sorted(nodes),
            "host_nodes": total, "loadavg_1_5_15": load}


def rep_stats(ts) -> dict:
    t = sorted(ts)
    return {"min_s": t[0], "median_s": t[len(t) // 2], "max_s": t[-1], "reps": len(t)}


def _oracle():
    sys.path.insert(0, str(REPO / "oracle"))
    import oracle  # test infrastructure: only the cpu_baseline leg loads it
    return oracle


def cpu_baseline_mt(obs, n, T, ess, scheme, threads, seed):
    """The bit-exact all-cores port of the same fused run (oracle/wsmc_port_mt.c, OpenMP over
    particles, gather-on-read + one trace-back), which the tests hold bit-identical to the
    statement oracle and so to the device. Returns (particle-steps/s, seconds)."""
    oracle = _oracle()
    oracle.keep_heap()
    oracle.ssm2d_run_mt(n, obs[:T], seed=seed, ess_perc_min=ess, scheme=scheme, threads=threads,
                        outputs=False)   # warm-up: thread pool, first touch of the run's buffers
    ts = []
    for _ in range(CPU_REPS):
        t0 = time.perf_counter()
        oracle.ssm2d_run_mt(n, obs[:T], seed=seed, ess_perc_min=ess, scheme=scheme, threads=threads,
                            outputs=False)
        ts.append(time.perf_counter() - t0)
    dt = sorted(ts)[len(ts) // 2]   # median
    return n * T / dt, dt, rep_stats(ts)


def cpu_baseline_fast(obs, n, T, ess, threads, seed):
    """The reference's algorithm at the reference's speed (oracle/wsmc_port_fast.c:
    xoshiro256++ + ziggurat normals, libm, the f64 icdf merge; statistically, not bitwise,
    equal — tests/test_port_fast.py), the same fused organisation (gather-on-read, one
    trace-back). The fastest CPU implementation here, hence the baseline `value` (SURVEY.md
    §8(d) ii with threads = all host cores, i with threads = 1)."""
    oracle = _oracle()
    oracle.keep_heap()
    oracle.fast_ssm2d_run(n, obs[:T], ess_perc_min=ess, seed=seed, threads=threads)   # warm-up (first touch)
    ts = []
    for _ in range(CPU_REPS if threads > 1 else 1):
        t0 = time.perf_counter()
        oracle.fast_ssm2d_run(n, obs[:T], ess_perc_min=ess, seed=seed, threads=threads)
        ts.append(time.perf_counter() - t0)
    dt = sorted(ts)[len(ts) // 2]   # median
    return n * T / dt, dt, rep_stats(ts)


def cpu_fairness_lgssm(n=100_000, T=200, seed=42):
    """SURVEY.md §8(d) CPU-baseline sanity check: the same fast port on the reference's own
    benchmark model (benchmarks/ssm/WeightedSampling/lgssm1d.jl, forced resampling), 1
    thread, N = 1e5, against the reference's published 5.30e7 particle-steps/s
    (benchmarks/ssm/results/grid_results.csv:46)."""
    oracle = _oracle()
    import wsmc
    data = wsmc.models.lgssm1d_data(T, seed=seed)
    oracle.keep_heap()
    oracle.fast_lgssm1d_run(n, data[:10], ess_perc_min=1.0, seed=seed, threads=1)   # warm-up (first touch)
    t0 = time.perf_counter()
    oracle.fast_lgssm1d_run(n, data, ess_perc_min=1.0, seed=seed, threads=1)
    dt = time.perf_counter() - t0
    return n * T / dt, dt


def cpu_baseline_1t(obs, n, T, ess, scheme, seed):
    """One thread, bit-exact: the statement oracle, i.e. the reference's algorithm with its
    eager ColumnStore gathers of every column at each resample (src/stores.jl:105-128)."""
    from oracle import Oracle  # noqa: F401  (path set by _oracle)
    _oracle()
    import wsmc
    o = Oracle(n, seed=seed)
    t0 = time.perf_counter()
    wsmc.models.ssm2d_statements(o, obs[:T], ess_perc_min=ess, scheme=scheme)
    dt = time.perf_counter() - t0
    o.close()
    return n * T / dt, dt


def sharded_self_check(args, wsmc, abi, comm, rank, world, local, lay, G, obs, scheme):
    """Before a sharded line is timed: the same population of CHECK_PARTICLES a GPU, CHECK_T steps,
    once on exact shards over the line's own layout and transport, once on one context; the
    shards' digests (state_digests) and the evidence must be bit-identical."""
    n = CHECK_PARTICLES
    gn = n * G
    kw = dict(ess_perc_min=args.ess, scheme=scheme if scheme != abi.RESAMPLE_MULTINOMIAL else abi.RESAMPLE_STRATIFIED,
              keep_history=True)
    o = obs[:CHECK_T]
    info = {"particles": gn, "T": CHECK_T, "shard_mode": "exact"}
    if comm is None:   # one process: a multi-device handle, or shards on GPU 0 (host transport)
        devs = lay["devices"] if lay["mode"] == "in-process" else [0] * G
        tr = abi.TRANSPORT_RCCL if lay["mode"] == "in-process" else abi.TRANSPORT_HOST
        ref = wsmc.Context(gn, seed=args.seed, device=devs[0])
        ev_ref = ref.ssm2d_run(o, **kw)
        dref = [state_digests(ref, g * n, (g + 1) * n) for g in range(G)]
        ref.close()
        m = wsmc.Context.multi(gn, G, seed=args.seed, devices=devs, transport=tr)
        m.comm_set_shard_mode(abi.SHARD_EXACT)
        if tr == abi.TRANSPORT_RCCL and args.watchdog > 0:
            m.comm_set_timeout(args.watchdog)
        ev = m.ssm2d_run(o, **kw)
        dgot = [state_digests(m, g * n, (g + 1) * n) for g in range(G)]
        m.close()
        info.update(check_verdict(dref, dgot, ev_ref, ev))
        info["transport"] = "rccl" if tr == abi.TRANSPORT_RCCL else "host"
        return info
    # a launcher's ranks: each runs its shard; rank 0 also the one-GPU population
    c = wsmc.Context(n, seed=args.seed, device=0 if args.same_device else local)
    if args.exchange == "host":
        c.comm_init_host(comm.allgather, world, rank, rank * n, gn)
    else:
        uid = comm.broadcast(wsmc.Context.comm_unique_id() if rank == 0 else None)
        c.comm_init(uid, world, rank, rank * n, gn)
        if args.watchdog > 0:
            c.comm_set_timeout(args.watchdog)
    c.comm_set_shard_mode(abi.SHARD_EXACT)
    ev = c.ssm2d_run(o, **kw)
    mine = state_digests(c, 0, n)
    c.close()
    got = comm.allgather([mine, ev])
    verdict = None
    if rank == 0:
        ref = wsmc.Context(gn, seed=args.seed, device=0 if args.same_device else local)
        ev_ref = ref.ssm2d_run(o, **kw)
        dref = [state_digests(ref, g * n, (g + 1) * n) for g in range(world)]
        ref.close()
        verdict = check_verdict(dref, [g[0] for g in got], ev_ref, got[0][1])
        if any(g[1] != got[0][1] for g in got):
            verdict["exact_vs_1gpu"] = False
    verdict = json.loads(comm.broadcast(json.dumps(verdict) if rank == 0 else None))   # (hostcomm sends no dicts)
    info.update(verdict)
    info["transport"] = args.exchange
    return info


def main():
    args = parse()
    # stdout carries the one JSON line only: native libraries write to fd 1 too (RCCL prints
    # its version banner at communicator creation), so fd 1 points at stderr for the run and
    # the JSON line goes to a private duplicate of the original stdout
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import wsmc
    from wsmc import abi
    from wsmc.hostcomm import from_env

    def ndev():
        try:
            return wsmc.Context.device_count()
        except Exception as e:   # no HIP runtime / no device: zero devices, said so
            log(f"bench: device count failed: {e}")
            return 0
    try:
        lay = plan_layout(args.gpus, os.environ, ndev, same_device=args.same_device,
                          multi_shards=args.multi_shards)
    except LayoutError as e:
        log(f"bench: refusing --gpus {args.gpus}: {e}")
        sys.exit(2)
    inproc = lay["mode"] == "in-process"
    world = 1 if inproc else lay["world"]   # processes
    G = lay["world"]                         # GPUs the line measures
    # host rendezvous / barriers / max-over-ranks over TCP; the rank process never imports
    # torch (its bundled HIP runtime would clash with libwsmc's ROCm one). The data path
    # between ranks is RCCL inside libwsmc.
    comm = from_env() if world > 1 else None

    scheme = {"stratified": abi.RESAMPLE_STRATIFIED, "systematic": abi.RESAMPLE_SYSTEMATIC,
              "multinomial": abi.RESAMPLE_MULTINOMIAL}[args.scheme]
    if args.global_particles > 0:   # strong scaling: ragged contiguous shards of one population
        P = args.global_particles
        N = P // world + (1 if rank < P % world else 0)
        goff = rank * (P // world) + min(rank, P % world)
        gN = P
    else:                           # weak scaling: N per GPU
        N = args.particles
        goff, gN = rank * N, world * N
    if inproc:   # one process, G devices: the handle splits gN into G contiguous shards
        gN = args.global_particles if args.global_particles > 0 else G * args.particles
        N, goff = gN // G, 0
    T = args.T
    obs = wsmc.models.ssm2d_data(max(T, args.cpu_T), seed=args.seed)
    # one seed for every rank: the Philox streams are keyed by the global particle index
    if inproc:
        log(f"bench: one process over {G} devices {lay['devices']} (wsmc_create_multi, RCCL), {gN} particles")
        ctx = wsmc.Context.multi(gN, G, seed=args.seed, devices=lay["devices"], transport=abi.TRANSPORT_RCCL)
        if args.shard_mode == "exact":
            ctx.comm_set_shard_mode(abi.SHARD_EXACT)
    elif args.multi_shards > 1 and comm is None:
        MS = args.multi_shards
        gN = MS * N
        ctx = wsmc.Context.multi(gN, MS, seed=args.seed, devices=[0] * MS, transport=abi.TRANSPORT_HOST)
        if args.shard_mode == "exact":
            ctx.comm_set_shard_mode(abi.SHARD_EXACT)
    else:
        ctx = wsmc.Context(N, seed=args.seed, device=0 if args.same_device else local)
    if comm is not None:
        if args.exchange == "host":
            ctx.comm_init_host(comm.allgather, world, rank, goff, gN)
        else:
            uid = comm.broadcast(wsmc.Context.comm_unique_id() if rank == 0 else None)
            ctx.comm_init(uid, world, rank, goff, gN)
        if args.shard_mode == "exact":
            ctx.comm_set_shard_mode(abi.SHARD_EXACT)
    if comm is None and args.rccl_one_rank:
        ctx.comm_init(wsmc.Context.comm_unique_id(), 1, 0, 0, N)
        if args.shard_mode == "exact":
            ctx.comm_set_shard_mode(abi.SHARD_EXACT)
    exact = (comm is not None or args.rccl_one_rank or args.multi_shards > 1 or inproc) and args.shard_mode == "exact"
    # what the communicator reports: every rank's view in rank order (a launcher's ranks
    # gather theirs over the host rendezvous)
    info = ctx.comm_info()
    if comm is not None:
        got = comm.allgather([info["rank"], info["rccl_ranks"], info["devices"][0], info["shard_n"][0]])
        ranks = {"launcher": "torch.distributed.run", "processes": world, "rccl_ranks": info["rccl_ranks"],
                 "transport": info["transport"], "devices": [g[2] for g in got], "shard_n": [g[3] for g in got]}
    else:
        ranks = {"launcher": None, "processes": 1, "rccl_ranks": info["rccl_ranks"], "transport": info["transport"],
                 "devices": info["devices"], "shard_n": info["shard_n"]}
    if (inproc or comm is not None) and args.exchange == "rccl" and ranks["rccl_ranks"] != G:
        log(f"bench: the RCCL communicator reports {ranks['rccl_ranks']} ranks, --gpus {G}: refusing the line")
        sys.exit(2)
    sharded = inproc or comm is not None or args.multi_shards > 1
    if sharded and args.watchdog > 0:
        import faulthandler
        # the process as a whole: a hang anywhere (a host exchange included) ends it with the
        # Python stacks on stderr; a collective's own wait is bounded below it
        faulthandler.dump_traceback_later(2 * args.watchdog + 60 * (args.steps + args.warmup) * T / 100, exit=True)
        if args.exchange == "rccl" or inproc:
            ctx.comm_set_timeout(args.watchdog)

    self_check = None
    if sharded and not args.no_self_check:
        S = G if inproc else args.multi_shards if args.multi_shards > 1 else world   # shards
        self_check = sharded_self_check(args, wsmc, abi, comm, rank, world, local, lay, S, obs, scheme)
        refuse_on_mismatch(self_check)
        log(f"bench: self-check passed (exact shards x{S} == one GPU, {self_check['particles']} particles, "
            f"T={CHECK_T})")
    if os.environ.get("WSMC_DUMP_MAPS"):   # diagnostics: the load map, to symbolise a crash's raw frames
        with open(os.environ["WSMC_DUMP_MAPS"], "w") as f:
            f.write(open("/proc/self/maps").read())

    def barrier():
        ctx.sync()
        if comm is not None:
            comm.barrier()

    if args.statements:
        if args.eager_store:
            ctx.store_set_lazy(False)

        def one_run():
            # run!(ssm(obs), state) statement by statement; no `if resampled` in the model, so
            # no Resample returns its flag to the host. The history x_1..x_{T+1} is brought up
            # to date at the end (one trace over the Resample log), as the fused run traces back.
            wsmc.models.ssm2d_statements(ctx, obs[:T], ess_perc_min=args.ess, scheme=scheme, wait=False)
            ctx.store_materialize()
    else:
        def one_run():
            return ctx.ssm2d_run(obs[:T], ess_perc_min=args.ess, scheme=scheme,
                                 keep_history=not args.no_history, want_evidence=False)

    for _ in range(args.warmup):
        one_run()
    # timed region: K full filter runs, no instrumentation
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        one_run()
    barrier()
    elapsed = time.perf_counter() - t0
    if comm is not None:
        elapsed = comm.max(elapsed)
    st = ctx.get_state()
    ev = ctx.log_evidence()
    xst = ctx.debug_exact() if exact else None   # exact shards: block / window needs, re-runs, history traces

    # per-kernel durations: HIP events recorded on the context stream around every launch of
    # the same graph (a separate instrumented pass of `steps` runs); not available on exact
    # shards (their eager, host-driven run is not instrumented)
    prop_ms = red_ms = rs_ms = fin_ms = tot_ms = 0.0
    nres = 0
    if not exact and not args.statements and args.multi_shards <= 1 and not inproc:
        ctx.set_timing(True)
        inst_runs = max(1, min(args.steps, 5))
        one_run()  # capture the instrumented graph
        for _ in range(inst_runs):
            one_run()
            tm = ctx.timing()
            prop_ms += tm["propagate_ms"]; red_ms += tm["reduce_ms"]; rs_ms += tm["resample_ms"]
            fin_ms += tm["finalize_ms"]; tot_ms += tm["total_ms"]; nres += tm["n_resamples"]
        ctx.set_timing(False)
        prop_ms /= inst_runs; red_ms /= inst_runs; rs_ms /= inst_runs; fin_ms /= inst_runs; tot_ms /= inst_runs
        nres //= inst_runs

    units = gN * T * args.steps
    value = units / elapsed
    ms_per_step = elapsed / args.steps * 1e3
    # propagate-kernel algorithmic bytes per run (forced resampling: every step after t=1 reads
    # through ancestors; t = 1 starts from the constant x0/v0)
    # every step resampled (step 1 of a fresh single-GPU state has equal weights, ESS = 1)
    forced = nres >= T - 1
    qmode = ctx.run_stats()["qstat_mode"] if hasattr(ctx, "run_stats") else 1
    steady = PROP_BYTES_STEADY + (PROP_BYTES_Q if qmode == 1 else 0)
    prop_bytes = N * (PROP_BYTES_FIRST + (T - 1) * steady + PROP_BYTES_LAST_DV)
    prop_gbs = prop_bytes / (prop_ms * 1e-3) / 1e9 if prop_ms > 0 else None
    def pmc(name):   # PMC-measured bytes (profiles/), reported only for the N they were measured at
        f = REPO / "pmc" / name   # copies of the latest profiles/ summaries (profiles/ does not travel)
        try:
            j = json.loads(f.read_text())
            return j if j.get("n_particles", N) == N and j.get("T", T) == T else None
        except Exception:
            return None
    tj = pmc("pmc_propagate_bytes.json")
    traffic = tj.get("bytes_per_launch") if tj else None
    sj = pmc("pmc_step_bytes.json")
    step_traffic = sj.get("bytes_per_particle_step") if sj and not args.statements else None

    cpu = None
    if rank == 0 and G == 1 and not args.no_cpu_baseline:   # the baseline is an N=1 figure
        if scheme == abi.RESAMPLE_MULTINOMIAL:   # the MT port covers the strata (the reference's scheme)
            cpu = None
        else:
            nth = cpu_threads(args.cpu_threads)
            omp = pin_openmp()
            topo = cpu_topology()   # before the ports run: OpenMP then binds this thread to one core
            n, T = args.cpu_particles, args.cpu_T
            fps, fdt, fst = cpu_baseline_fast(obs, n, T, args.ess, nth, args.seed)
            f1, f1dt, _ = cpu_baseline_fast(obs, args.cpu_1t_particles, T, args.ess, 1, args.seed)
            cps, cdt, cst = cpu_baseline_mt(obs, n, T, args.ess, scheme, nth, args.seed)
            c1, c1dt = cpu_baseline_1t(obs, args.cpu_1t_particles, T, args.ess, scheme, args.seed)
            lg, lgdt = cpu_fairness_lgssm()
            fast_leg = {"value": fps, "unit": "particle-steps/s", "cores": nth, "kind": "port",
                    "sample": f"oracle/wsmc_port_fast.c (the reference's algorithm with xoshiro256++/ziggurat/"
                              f"libm, OpenMP over particles, {nth} threads on {cpu_model()}): the full 2D SSM "
                              f"run, N={n} T={T} ess_perc_min={args.ess}, history traced back: {fdt:.2f} s (median of {CPU_REPS})",
                    "reps": fst}
            exact_leg = {"value": cps, "unit": "particle-steps/s", "cores": nth, "kind": "port",
                     "sample": f"oracle/wsmc_port_mt.c (bit-identical to the device; OpenMP over particles, "
                               f"{nth} threads on {cpu_model()}): the full 2D SSM run, N={n} T={T} "
                               f"ess_perc_min={args.ess}, history traced back: {cdt:.2f} s (median of {CPU_REPS})",
                     "reps": cst}
            # the baseline is the faster of the two all-cores ports; the other is reported beside it
            best, other, other_key = ((fast_leg, exact_leg, "exact_port") if fps >= cps
                                      else (exact_leg, fast_leg, "fast_port"))
            cpu = dict(best)
            pc = topo["physical_cores"] or nth
            cpu.update({
                "threads": nth, "binding": omp, "numa": topo, "cpu_model": cpu_model(),
                # the GPU pool sets OMP_NUM_THREADS to the job's CPU share of the shared host (16
                # for one GPU) and asks jobs to leave it: `threads` honours it. For scale, the
                # same rate per thread times every physical core of the mask — a linear upper
                # bound on the whole host (memory bandwidth would cap it first), labelled so
                "threads_policy": ("OMP_NUM_THREADS (the GPU pool's CPU share of the host, left as set)"
                                   if os.environ.get("OMP_NUM_THREADS", "").isdigit() else "affinity mask"),
                "all_physical_cores_linear_bound": {
                    "value": best["value"] / nth * pc, "cores": pc, "kind": "extrapolation",
                    "gpu_over_it": value / (best["value"] / nth * pc)},
                other_key: other,
                "single_thread": {"value": f1, "unit": "particle-steps/s", "cores": 1, "kind": "port",
                                  "sample": f"oracle/wsmc_port_fast.c, 1 thread, N={args.cpu_1t_particles} "
                                            f"T={T}: {f1dt:.2f} s"},
                "exact_single_thread": {"value": c1, "unit": "particle-steps/s", "cores": 1, "kind": "port",
                                        "sample": f"oracle/wsmc_oracle.c statements (the reference's eager "
                                                  f"ColumnStore gathers), N={args.cpu_1t_particles} T={T}: "
                                                  f"{c1dt:.2f} s"},
                "fairness_lgssm1d_1t": {"value": lg, "unit": "particle-steps/s", "cores": 1,
                                        "reference_published": 5.30e7, "ratio": lg / 5.30e7,
                                        "sample": "oracle/wsmc_port_fast.c on benchmarks/ssm/WeightedSampling/"
                                                  f"lgssm1d.jl, N=100000 T=200 forced, 1 thread: {lgdt:.2f} s"},
                "gpu_over_cpu": value / best["value"],
                "gpu_over_single_thread": value / f1})
    if rank == 0:
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "particle-steps/s",
            "n_gpus": G,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,          # one bench step = one full T-step run
            "ms_per_run": ms_per_step,
            "us_per_filter_step": ms_per_step * 1e3 / T,
            "higher_is_better": True,
            "scaling": "strong" if args.global_particles > 0 else "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic: examples/2D_ssm.jl observation recurrence (numpy Philox seed 42)",
            "config": {"workload": "2D SSM bootstrap filter (examples/2D_ssm.jl), BASELINE configs[1]"
                                   + (" through the generic statement operators (one C-ABI call per statement, "
                                      + ("eager store: every column gathered at every resample)" if args.eager_store
                                         else "lazy genealogy)") if args.statements else ""),
                       "n_particles_per_gpu": N, "global_particles": gN, "T": T,
                       "ess_perc_min": args.ess, "scheme": args.scheme, "keep_history": not args.no_history,
                       # island shards resample within themselves after the global decision: a
                       # different (unbiased) estimator than the reference's single-population
                       # Resample, which exact shards reproduce bit for bit
                       "estimator": ("reference (single population)" if (G == 1 and not args.rccl_one_rank
                                                                         and args.multi_shards <= 1)
                                     or args.shard_mode == "exact"
                                     else "island resampling (per-shard strata, global decision)"),
                       "parallelism": (f"{args.shard_mode}-shard x{G}, one process over {G} GPUs "
                                       "(wsmc_create_multi: ncclCommInitAll, one host thread per shard)") if inproc else
                                      (f"{args.shard_mode}-shard x{args.multi_shards} in one handle on one GPU "
                                       "(in-process exchange, diagnostic)") if args.multi_shards > 1 else
                                      (f"{args.shard_mode}-shard x{world}"
                                       + (" (host exchange, test mode)" if args.exchange == "host" else ""))
                           if world > 1 else ("single GPU, one-rank RCCL communicator (diagnostic)"
                                              if args.rccl_one_rank else "single GPU")},
            # the whole step against HBM — achieved = particle-steps/s per GPU x
            # 104 algorithmic B (CDF materialisation and trace-back count as overhead); traffic =
            # the PMC-measured HBM bytes per particle-step of every kernel of the run (trace-back
            # included). The dominant kernel's own figure (HIP events on its dispatches) beside it.
            "roofline": {"bound": "hbm", "achieved": value / G * STEP_BYTES / 1e9, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": value / G * STEP_BYTES / 1e9 / HBM_PEAK_GBS,
                         "traffic": step_traffic, "algorithmic_bytes_per_particle_step": STEP_BYTES,
                         "definition": "whole step: particle-steps/s per GPU x 104 B / 8 TB/s (SURVEY.md 8d)",
                         "dominant_kernel": None if args.statements else {
                             "kernel": "k_ssm2d_prop (propagate+observe+max)", "achieved": prop_gbs,
                             "peak": HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": (prop_gbs / HBM_PEAK_GBS) if prop_gbs else None, "traffic": traffic,
                             "algorithmic_bytes_per_run": prop_bytes,
                             "avg_launch_us": prop_ms * 1e3 / T if prop_ms > 0 else None}},
            "cpu_baseline": cpu,
            "breakdown_ms_per_run": None if exact or args.statements else {
                "propagate": prop_ms, "weight_stats": red_ms, "scan_ancestors": rs_ms,
                "finalize_traceback": fin_ms, "instrumented_total": tot_ms,
                "resamples_per_run": nres, "forced_every_step": forced},
            "log_evidence_last": ev,
            "ranks": ranks,
        }
        if xst is not None:
            line["exact_stats"] = xst
        if self_check is not None:
            line["self_check"] = self_check
        os.write(json_fd, (json.dumps(line) + "\n").encode())
    ctx.close()
    if comm is not None:
        comm.barrier()
        comm.close()


if __name__ == "__main__":
    main()
