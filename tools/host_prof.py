"""Host-side cost of the statement path at a population small enough that the device work is a
few microseconds a kernel, so the run's wall time is the host's enqueue cost; then cProfile's
top functions over the same runs. python tools/host_prof.py [N] [c3|c2]: C3 (gated, one Move
block a step) or C2 (the 2D SSM statements, no flag read, history brought up to date)."""
import cProfile
import pathlib
import pstats
import sys
import time

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1] / "weightedsampling.jl_amd"))
import wsmc
from wsmc import models

N = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
MODEL = sys.argv[2] if len(sys.argv) > 2 else "c3"
xs, ys = models.linreg_data()
obs = models.ssm2d_data(100)


def run():
    ctx = wsmc.Context(N, seed=42)
    ctx.sync()
    t0 = time.perf_counter()
    if MODEL == "c2":
        models.ssm2d_statements(ctx, obs, ess_perc_min=1.0, wait=False)
        ctx.store_materialize()
    else:
        models.linreg_statements(ctx, xs, ys, ess_perc_min=1.0, gated=True, block=True)
    t1 = time.perf_counter()
    ctx.sync()
    t2 = time.perf_counter()
    ctx.close()
    return t1 - t0, t2 - t0


for _ in range(3):
    run()
best = min(run() for _ in range(10))
T = len(obs) if MODEL == "c2" else len(xs)
print(f"N={N}: enqueue {best[0] * 1e6 / T:.1f} us a step, with the sync {best[1] * 1e6 / T:.1f} us a step")
pr = cProfile.Profile()
pr.enable()
for _ in range(20):
    run()
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
