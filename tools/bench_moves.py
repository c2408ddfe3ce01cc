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


def c3(N=1_000_000, reps=3):
    xs, ys = models.linreg_data()
    best = math.inf
    for _ in range(reps + 1):
        ctx = wsmc.Context(N, seed=42)
        ctx.sync()
        t0 = time.perf_counter()
        acc = models.linreg_statements(ctx, xs, ys, ess_perc_min=1.0)
        ctx.sync()
        dt = time.perf_counter() - t0
        ev = ctx.log_evidence()
        ctx.close()
        best = min(best, dt)
    T = len(xs)
    return {"config": "C3 linear regression + autoRW (N=1M, T=10, ess 1.0)", "N": N, "T": T,
            "seconds_per_run": best, "particle_steps_per_s": N * T / best, "moves": 2 * len(acc),
            "log_evidence": ev}


def c5(N=4_000_000, T=60, sweeps=5, reps=1):
    t_obs, y_obs = models.oscillator_data(n=T)
    best = math.inf
    for _ in range(reps + 1):
        ctx = wsmc.Context(N, seed=42)
        ctx.sync()
        t0 = time.perf_counter()
        acc = models.oscillator_statements(ctx, t_obs, y_obs, ess_perc_min=1.0, scheme=wsmc.RESAMPLE_SYSTEMATIC,
                                           sweeps=sweeps, diversity=None)
        ctx.sync()
        dt = time.perf_counter() - t0
        ctx.close()
        best = min(best, dt)
    # score terms per particle: every move folds twice over the 5 priors + t observations
    terms = sum(2 * 2 * sweeps * (5 + t) for t in range(1, T + 1))
    return {"config": f"C5 damped oscillator, systematic, {sweeps} ungated sweeps (N={N}, T={T}, ess 1.0)",
            "N": N, "T": T, "seconds_per_run": best, "particle_steps_per_s": N * T / best,
            "score_terms_per_particle": terms, "score_terms_per_s": N * terms / best}


if __name__ == "__main__":
    which = sys.argv[1:] or ["c3", "c5"]
    for w in which:
        print(json.dumps(c3() if w == "c3" else c5()), flush=True)
