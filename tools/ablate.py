"""Resample-kernel ablations on MI355X (diagnostics). Two weight states:
  spread — a fused 2D SSM run (resampled every step) followed by one Weight by a
           Normal on v[0]: one step's worth of likelihood spread (the bench case)
  skewed — a run that never resamples: 20 steps of accumulated skew"""
import sys, pathlib
sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1] / "weightedsampling.jl_amd"))
import wsmc
from wsmc import abi
from wsmc.dsl import Normal
N = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
c = wsmc.Context(N, seed=1)
obs = wsmc.models.ssm2d_data(20)
for name, ess in (("spread", 1.0), ("skewed", 0.0)):
    c.ssm2d_run(obs, ess_perc_min=ess, keep_history=False)
    if name == "spread":
        c.weight(Normal(0.0, 0.3).dist(c.col_find), [abi.Operand.column(c.col_find("v"), 0)])
    for k, modes in ((0, (0, 1, 4)), (1, range(4)), (2, range(4)), (3, (0, 1))):
        for m in modes:
            c.debug_kernel_bench(k, m, 5)
            print(f"{name} kernel {k} mode {m}: {c.debug_kernel_bench(k, m, 100):.2f} us", flush=True)
