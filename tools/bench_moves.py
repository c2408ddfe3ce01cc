"""Throughput of the MH-move configs through the generic operator path (one GPU):
  C3  linear regression + autoRW moves after each resample (examples/linear_regression.jl),
      N = 1M, ess_perc_min = 1.0 (a move pair every step), T = 10
  C5  damped oscillator, systematic resampling, 5 ungated sweeps of the bounded 4-D and 1-D
      autoRW moves per step (examples/damped_oscillator.jl), N = 4M (the config's 4 GPUs
      worth on one), T = 60
Prints one JSON line per config: particle-steps/s and, for C5, the score-fold work
(terms evaluated) as a rate. Diagnostics for DESIGN.md; bench.py stays the headline."""
import json
import math
import sys
import time
import pathlib

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1] / "weightedsampling.jl_amd"))
import wsmc
from wsmc import models


def _ctx(N, one_rank):
    ctx = wsmc.Context(N, seed=42)
    if one_rank:   # the sharded code path (record / moment exchanges) through a one-rank communicator
        ctx.comm_init(wsmc.Context.comm_unique_id(), 1, 0, 0, N)
    return ctx


def c3(N=1_000_000, reps=3, wait_moves=True, one_rank=False, gated=False, block=True):
    xs, ys = models.linreg_data()
    best = math.inf
    for _ in range(reps + 1):
        ctx = _ctx(N, one_rank)
        ctx.sync()
        t0 = time.perf_counter()
        acc = models.linreg_statements(ctx, xs, ys, ess_perc_min=1.0, wait_moves=wait_moves, gated=gated,
                                       block=block)
        ctx.sync()
        dt = time.perf_counter() - t0
        ev = ctx.log_evidence()
        ctx.close()
        best = min(best, dt)
    T = len(xs)
    return {"config": "C3 linear regression + autoRW (N=1M, T=10, ess 1.0)"
                      + ("" if wait_moves or gated else ", asynchronous moves (no accepted counts)")
                      + (", `if resampled` lowered to device-gated moves (no host read in the loop)" if gated else "")
                      + (", the two Moves as one statement block (wsmc_move_block)" if gated and block else "")
                      + (", sharded path (one-rank RCCL communicator)" if one_rank else ""), "N": N, "T": T,
            "seconds_per_run": best, "particle_steps_per_s": N * T / best, "moves": 2 * T if gated else 2 * len(acc),
            "log_evidence": ev}


def c5(N=4_000_000, T=60, sweeps=5, reps=1, scheme="systematic", ess=1.0, diversity=None, one_rank=False,
       wait_moves=True, block=False):
    t_obs, y_obs = models.oscillator_data(n=T)
    sch = {"systematic": wsmc.RESAMPLE_SYSTEMATIC, "stratified": wsmc.RESAMPLE_STRATIFIED}[scheme]
    best, moved = math.inf, 0
    for _ in range(reps + 1):
        ctx = _ctx(N, one_rank)
        ctx.sync()
        t0 = time.perf_counter()
        acc = models.oscillator_statements(ctx, t_obs, y_obs, ess_perc_min=ess, scheme=sch, sweeps=sweeps,
                                           diversity=diversity, wait_moves=wait_moves, block=block)
        ctx.sync()
        dt = time.perf_counter() - t0
        ctx.close()
        best = min(best, dt)
        moved = sum(x for a in acc for x in a) if wait_moves else None   # accepted proposals
    gate = "ungated" if diversity is None else f"diversity={diversity}"
    out = {"config": f"C5 damped oscillator, {scheme}, {sweeps} {gate} sweep(s) (N={N}, T={T}, ess {ess})"
                     + ("" if wait_moves else ", asynchronous moves (no accepted counts)")
                     + (", each sweep one Move block (wsmc_move_block)" if block else "")
                     + (", sharded path (one-rank RCCL communicator)" if one_rank else ""),
           "N": N, "T": T, "seconds_per_run": best, "particle_steps_per_s": N * T / best,
           "accepted": moved, "moves_offered": 2 * sweeps * T}
    if diversity is None and ess >= 1.0:
        # score terms evaluated per particle: every move folds s_new over the 5 priors + t
        # observations; s_old is the carried score, continued over the one new observation by
        # the step's first move (0 terms afterwards)
        terms = sum(2 * sweeps * (5 + t) + 1 for t in range(1, T + 1))
        out.update({"score_terms_per_particle": terms, "score_terms_per_s": N * terms / best})
    return out


def _oracle():
    """the CPU port (test infrastructure: a baseline leg only), OpenMP threads bound one per
    core before its library loads"""
    import os
    os.environ.setdefault("OMP_PLACES", "cores")
    os.environ.setdefault("OMP_PROC_BIND", "close")
    sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1] / "oracle"))
    from oracle import Oracle
    return Oracle, int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))


def c3cpu(N=100_000, reps=2):
    """C3 on the CPU port (the oracle: OpenMP over particles in the Move, serial elsewhere) at a
    bounded N: the baseline beside the device's C3 lines"""
    Oracle, threads = _oracle()
    xs, ys = models.linreg_data()
    best = math.inf
    for _ in range(reps):
        o = Oracle(N, seed=42)
        t0 = time.perf_counter()
        models.linreg_statements(o, xs, ys, ess_perc_min=1.0, gated=True, block=False)
        best = min(best, time.perf_counter() - t0)
        o.close() if hasattr(o, "close") else None
    T = len(xs)
    return {"config": f"C3 on the CPU port (oracle, {threads} OpenMP threads bound to cores), N={N}, T={T}, ess 1.0",
            "N": N, "T": T, "seconds_per_run": best, "particle_steps_per_s": N * T / best, "threads": threads}


LEGS = {
    "c3cpu": c3cpu,
    "c3": c3,
    "c5": c5,                                                             # canonical (systematic)
    "c5_stratified": lambda: c5(scheme="stratified"),                     # the reference's scheme
    "c5_example": lambda: c5(sweeps=1, scheme="stratified", ess=0.5, diversity=0.9),   # as written
    "c3async": lambda: c3(wait_moves=False),
    "c3gated": lambda: c3(gated=True),
    "c3gated_moves": lambda: c3(gated=True, block=False),                 # two wsmc_move_gated
    "c5async": lambda: c5(wait_moves=False),
    "c5block": lambda: c5(block=True),
    "c5blockasync": lambda: c5(block=True, wait_moves=False),
    "c3_rccl1": lambda: c3(one_rank=True),
    "c3async_rccl1": lambda: c3(wait_moves=False, one_rank=True),
    "c5_rccl1": lambda: c5(one_rank=True),
}


if __name__ == "__main__":
    for w in sys.argv[1:] or ["c3", "c5"]:
        print(json.dumps(LEGS[w]()), flush=True)
