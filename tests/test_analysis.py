"""Analysis reductions (src/utils.jl): expectation / @E, describe's weighted mean and std
(corrected=false), min/max, ESS. The oracle is checked against numpy here (CPU); the HIP
path against the oracle bit for bit (-m gpu)."""
import math

import numpy as np
import pytest

import wsmc
from wsmc import abi, models
from oracle import Oracle


def _setup(c):
    rng = np.random.default_rng(0)
    n = c.n
    c.col_create("a")
    c.col_create("x2", 2)
    c.col_upload(c.col_find("a"), rng.standard_normal(n))
    c.col_upload(c.col_find("x2"), rng.standard_normal((2, n)) * [[1.0], [3.0]] + [[0.5], [-2.0]])
    c.weights_upload(-0.5 * rng.standard_normal(n) ** 2)
    return c


def test_oracle_moments_match_numpy():
    o = _setup(Oracle(5000, seed=1))
    a = o.col_download(o.col_find("a"))
    x2 = o.col_download(o.col_find("x2"))
    w = np.exp(o.weights_download() - o.weights_download().max())
    w /= w.sum()
    ex = [abi.Operand.column(o.col_find("a")), abi.Operand.column(o.col_find("x2"), 1),
          abi.Operand.column(o.col_find("x2"), 0, coef=2.0, c0=1.0)]
    mean, cov = o.weighted_moments(ex)
    vals = np.stack([a, x2[1], 1.0 + 2.0 * x2[0]])
    m_ref = vals @ w
    c_ref = ((vals - m_ref[:, None]) * w) @ (vals - m_ref[:, None]).T
    np.testing.assert_allclose(mean, m_ref, rtol=1e-12)
    np.testing.assert_allclose(cov, c_ref, rtol=1e-10)
    mn, mx = o.col_minmax(o.col_find("x2"), 1)
    assert (mn, mx) == (x2[1].min(), x2[1].max())
    ess = 1.0 / (len(w) * np.sum(w ** 2))
    assert abs(o.ess() - ess) < 1e-6 * ess


def test_oracle_minmax_nan_propagates():
    o = Oracle(10, seed=1)
    c = o.col_create("v")
    v = np.arange(10.0)
    v[3] = np.nan
    o.col_upload(c, v)
    mn, mx = o.col_minmax(c)
    assert math.isnan(mn) and math.isnan(mx)


@pytest.mark.gpu
@pytest.mark.parametrize("N", [1, 999, 300001])
def test_analysis_hip_matches_oracle(gpu_available, N):
    g, o = _setup(wsmc.Context(N, seed=1)), _setup(Oracle(N, seed=1))
    for ctx in (g, o):
        assert ctx.col_names() == ["a", "x2"]
    ex = [abi.Operand.column(1, 0), abi.Operand.column(1, 1), abi.Operand.column(0),
          abi.Operand.column(0, coef=-1.5, c0=0.25)]
    mg, cg = g.weighted_moments(ex)
    mo, co = o.weighted_moments(ex)
    np.testing.assert_array_equal(mg, mo)
    np.testing.assert_array_equal(cg, co)
    for col, comp in ((0, 0), (1, 0), (1, 1)):
        assert g.col_minmax(col, comp) == o.col_minmax(col, comp)
    assert g.ess() == o.ess()
    # no state change
    sg, so = g.get_state(), o.get_state()
    for k in sg:
        assert sg[k] == so[k] or (isinstance(sg[k], float) and math.isnan(sg[k]) and math.isnan(so[k])), k


@pytest.mark.gpu
def test_describe_and_expectation_mirror(gpu_available):
    st = wsmc.SMCState(20000, seed=3)
    _setup(st.ctx)
    rows = wsmc.describe(st)
    w = np.exp(st.weights - st.weights.max())
    w /= w.sum()
    a = st["a"]
    assert rows[0]["variable"] == "a"
    assert abs(rows[0]["mean"] - a @ w) < 1e-12
    assert abs(rows[0]["std"] - math.sqrt(((a - a @ w) ** 2) @ w)) < 1e-12
    assert rows[1]["min"] == list(st["x2"].min(axis=1))
    assert abs(wsmc.expectation(st, wsmc.Col("a") * 2.0 + 1.0) - (2.0 * a + 1.0) @ w) < 1e-12
