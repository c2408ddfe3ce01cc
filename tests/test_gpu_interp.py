"""The Move interpreter kernels stay covered.

Move blocks and single autoRW Moves run on kernels compiled for their shape
(csrc/wsmc_mv_body.h). The interpreter kernels they replace (k_move_blk, k_move_c /
k_move_ci) remain the fallback when a shape does not compile, and `WSMC_DIAG_NO_JIT=1` /
`WSMC_DIAG_NO_BLOCK1=1` select them. The switches are read once per process, so each
combination runs C3 (examples/linear_regression.jl, its `if resampled` Moves as a gated
block) and a short C5 (examples/damped_oscillator.jl, bounded 4-D and 1-D Moves) in a child
process against the oracle, bit for bit.
"""
import os
import pathlib
import subprocess
import sys

import pytest

REPO = pathlib.Path(__file__).resolve().parents[1]

CHILD = r"""
import sys
sys.path[:0] = [{pkg!r}, {orc!r}, {tests!r}]
import wsmc
from wsmc import abi, models
from oracle import Oracle
from test_gpu_parity import assert_same_state

xs, ys = models.linreg_data()
g, o = wsmc.Context(3001, seed=5), Oracle(3001, seed=5)
models.linreg_statements(g, xs, ys, ess_perc_min=0.7, gated=True, block=True)
models.linreg_statements(o, xs, ys, ess_perc_min=0.7, gated=True, block=True)
assert_same_state(g, o)
assert g.log_evidence() == o.log_evidence()
t, y = models.oscillator_data(n=8)
g, o = wsmc.Context(2001, seed=6), Oracle(2001, seed=6)
ag = models.oscillator_statements(g, t, y, ess_perc_min=1.0, scheme=wsmc.RESAMPLE_SYSTEMATIC, sweeps=2,
                                  diversity=None)
ao = models.oscillator_statements(o, t, y, ess_perc_min=1.0, scheme=wsmc.RESAMPLE_SYSTEMATIC, sweeps=2,
                                  diversity=None)
assert ag == ao
assert_same_state(g, o)
st = abi.mv_jit_stats()
print("MVJIT", st["launched"], st["interpreted"])
"""


@pytest.mark.gpu
@pytest.mark.parametrize("env", [{"WSMC_DIAG_NO_JIT": "1"}, {"WSMC_DIAG_NO_JIT": "1", "WSMC_DIAG_NO_BLOCK1": "1"}])
def test_move_interpreter_kernels_match_oracle(gpu_available, env):
    code = CHILD.format(pkg=str(REPO / "weightedsampling.jl_amd"), orc=str(REPO / "oracle"),
                        tests=str(REPO / "tests"))
    r = subprocess.run([sys.executable, "-c", code], env={**os.environ, **env}, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("MVJIT")][0]
    launched, interpreted = map(int, line.split()[1:])
    assert launched == 0 and interpreted > 0, line
