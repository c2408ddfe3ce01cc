"""Resample-kernel ablations on MI355X (diagnostics). Runs a fused 2D SSM first so the
weights have a realistic spread: ess 1.0 (resampled every step: one step of likelihood
spread, the bench case) and ess 0.0 (never resampled: 20 steps of accumulated skew)."""
import sys, pathlib
sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1] / "weightedsampling.jl_amd"))
import wsmc
N = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
c = wsmc.Context(N, seed=1)
obs = wsmc.models.ssm2d_data(20)
for ess in (1.0, 0.0):
    c.ssm2d_run(obs, ess_perc_min=ess, keep_history=False)
    for k, modes in ((0, (0, 1, 4)), (1, [0]), (2, range(4))):
        for m in modes:
            c.debug_kernel_bench(k, m, 5)
            print(f"ess {ess} kernel {k} mode {m}: {c.debug_kernel_bench(k, m, 100):.2f} us", flush=True)
