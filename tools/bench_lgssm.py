"""The reference's own published CPU benchmark, run here (SURVEY.md §8(d) "CPU baseline sanity
check"): the 1D linear-Gaussian SSM of benchmarks/ssm/WeightedSampling/lgssm1d.jl
(x ~ Normal(0.9x, 1), y => Normal(x, 0.5), forced resampling), T = 1000.

  gpu        the statement operators through the C ABI (Sample, Resample, Observe, Resample per
             step: the generic drop-in path a `@model` lowers to), N = 1e6, against the
             reference's published run! wall at the same N and T (22.170888 s,
             benchmarks/ssm/results/grid_results.csv:14, one Julia thread, hardware unstated)
  cpu_1t     oracle/wsmc_port_fast.c (the reference's algorithm at the reference's speed:
             xoshiro256++, ziggurat, libm, f64 icdf) on 1 thread, N = 1e5 — the fairness check
             against the published 5.30e7 (single update, N = 1e5, grid_results.csv:46) and
             4.51e7 (run!, N = 1e6, :14) particle-steps/s
  cpu_all    the same port on all host threads, N = 1e6

One JSON line per leg. Diagnostics for DESIGN.md; bench.py stays the headline."""
import json
import os
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "weightedsampling.jl_amd"), str(ROOT / "oracle"), str(ROOT)]
import wsmc  # noqa: E402
from wsmc import models  # noqa: E402

PUBLISHED_RUN_S = 22.170888          # grid_results.csv:14 (N = 1e6, T = 1000)
PUBLISHED_1T_RATE = 5.30e7           # grid_results.csv:46 (single update, N = 1e5)


def threads() -> int:
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit():
        return int(env)
    return len(os.sched_getaffinity(0))


def gpu(N=1_000_000, T=1000, reps=2, wait=False):
    data = models.lgssm1d_data(T)
    best, ev = float("inf"), None
    for _ in range(reps + 1):           # the first run is the warm-up
        ctx = wsmc.Context(N, seed=42)
        ctx.sync()
        t0 = time.perf_counter()
        models.lgssm1d_statements(ctx, data, ess_perc_min=1.0, wait=wait)   # no `if resampled`: no flags needed
        ctx.sync()
        dt = time.perf_counter() - t0
        ev = ctx.log_evidence()
        nres = ctx.get_state()["n_resamples"]
        ctx.close()
        best = min(best, dt)
    return {"leg": "gpu statements" + (", flags to the host" if wait else ", decisions on the device"),
            "N": N, "T": T, "seconds_per_run": best, "particle_steps_per_s": N * T / best, "resamples": nres, "log_evidence": ev, "reference_published_s": PUBLISHED_RUN_S,
            "speedup_vs_published": PUBLISHED_RUN_S / best}


def cpu(N, T, nth, reps=1):
    import oracle  # test infrastructure: a CPU baseline leg
    data = models.lgssm1d_data(T)
    best, out = float("inf"), None
    for _ in range(reps + 1):
        t0 = time.perf_counter()
        out = oracle.fast_lgssm1d_run(N, data, ess_perc_min=1.0, threads=nth)
        best = min(best, time.perf_counter() - t0)
    rate = N * T / best
    return {"leg": f"cpu fast port, {nth} thread(s)", "N": N, "T": T, "seconds_per_run": best,
            "particle_steps_per_s": rate, "log_evidence": out[0], "resamples": out[2],
            "vs_published_1t_rate": rate / PUBLISHED_1T_RATE}


if __name__ == "__main__":
    which = sys.argv[1:] or ["gpu", "gpu_wait", "cpu_1t", "cpu_all"]
    for w in which:
        if w == "gpu":
            r = gpu()
        elif w == "gpu_wait":
            r = gpu(wait=True)
        elif w == "cpu_1t":
            r = cpu(100_000, 1000, 1)
        else:
            r = cpu(1_000_000, 1000, threads())
        print(json.dumps(r), flush=True)
