"""Host-side cost of one fused 2D-SSM run (wsmc_ssm2d_run): wall time a run at a population small
enough that the device work is microseconds (so the wall time is the host's: Python, the C entry,
the graph launch, the end-of-run read-back), and cProfile's top entries over the same runs.
    python tools/host_run_prof.py [N] [T]"""
import cProfile
import pathlib
import pstats
import sys
import time

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1] / "weightedsampling.jl_amd"))
import wsmc
from wsmc import models

N = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
T = int(sys.argv[2]) if len(sys.argv) > 2 else 100
obs = models.ssm2d_data(T)
ctx = wsmc.Context(N, seed=42)
for _ in range(5):
    ctx.ssm2d_run(obs, ess_perc_min=1.0, want_evidence=False)
ctx.sync()
R = 200
t0 = time.perf_counter()
for _ in range(R):
    ctx.ssm2d_run(obs, ess_perc_min=1.0, want_evidence=False)
ctx.sync()
dt = (time.perf_counter() - t0) / R
print(f"N={N} T={T}: {dt * 1e6:.1f} us a run (wall)")
pr = cProfile.Profile()
pr.enable()
for _ in range(50):
    ctx.ssm2d_run(obs, ess_perc_min=1.0, want_evidence=False)
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(8)
