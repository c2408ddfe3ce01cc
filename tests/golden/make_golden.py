#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ from the CPU oracle.

The reference (Julia) cannot run here and ships no golden vectors, so
these fixtures freeze the oracle restatement's outputs on the configs' small cases
(SURVEY.md §8c items 2-3): C1 (1D SSM, N=1000, T=50, seed 7) and C2 (2D SSM, N=1024, T=8,
seed 42) at ess_perc_min 0.5 and 1.0, plus edge cases. tests/test_golden.py checks the
oracle and (under -m gpu) the HIP path against them bit for bit.

    python tests/golden/make_golden.py
"""
import pathlib
import sys

import numpy as np

HERE = pathlib.Path(__file__).resolve().parent
REPO = HERE.parents[1]
sys.path[:0] = [str(REPO / "weightedsampling.jl_amd"), str(REPO / "oracle")]

import wsmc  # noqa: E402
from oracle import Oracle  # noqa: E402


def dump(ctx, path, flags, **extra):
    cols = {f"col__{n}": ctx.col_download(ctx.col_find(n)) for n in ctx.col_names()}
    st = ctx.get_state()
    np.savez_compressed(path, weights=ctx.weights_download(), ancestors=ctx.last_ancestors(),
                        resampled=np.array(flags, dtype=np.int8), log_evidence=np.array([ctx.log_evidence()]),
                        state=np.array([st["depth"], st["n_terms"], st["op_counter"], st["n_resamples"]]),
                        colnames=np.array(ctx.col_names()), **cols, **extra)


def main():
    for ess in (0.5, 1.0):
        tag = f"{int(ess * 10):02d}"
        obs = wsmc.models.ssm1d_data(50)
        o = Oracle(1000, seed=7)
        f = wsmc.models.ssm1d_statements(o, obs, ess_perc_min=ess)
        dump(o, HERE / f"c1_ssm1d_ess{tag}.npz", f, obs=obs)
        obs = wsmc.models.ssm2d_data(8)
        o = Oracle(1024, seed=42)
        f = wsmc.models.ssm2d_statements(o, obs, ess_perc_min=ess)
        dump(o, HERE / f"c2_ssm2d_ess{tag}.npz", f, obs=obs)
    xs, ys = wsmc.models.linreg_data()
    o = Oracle(2048, seed=42)
    acc = wsmc.models.linreg_statements(o, xs, ys, ess_perc_min=1.0)
    dump(o, HERE / "c3_linreg_ess10.npz", [], accepted=np.array(acc), xs=xs, ys=ys)
    t, y = wsmc.models.oscillator_data(n=8)
    o = Oracle(2048, seed=42)
    acc = wsmc.models.oscillator_statements(o, t, y, ess_perc_min=1.0, scheme=wsmc.RESAMPLE_SYSTEMATIC,
                                            sweeps=2, diversity=None)
    dump(o, HERE / "c5_oscillator_ess10.npz", [], accepted=np.array(acc), t=t, y=y)
    for p in sorted(HERE.glob("*.npz")):
        print(p.name, p.stat().st_size)


if __name__ == "__main__":
    main()
