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


# ---- describe's weighted median and sparkline (src/utils.jl:120-141, :233-240) -----------
def _statsbase_median(v, w):
    """StatsBase.quantile(v, Weights(w), 0.5) (StatsBase 0.34, non-frequency weights),
    restated in Python floats: zero weights dropped, (value, weight) sorted, walk to h."""
    vw = sorted((float(a), float(b)) for a, b in zip(v, w) if b != 0)
    W, w1 = sum(b for _, b in vw), vw[0][1]
    h = 0.5 * (W - w1) + w1
    Sk = Skold = vk = vkold = 0.0
    k = 0
    while Sk <= h:
        k += 1
        if k > len(vw):
            return vw[-1][0]
        Skold, vkold = Sk, vk
        vk, wk = vw[k - 1]
        Sk += wk
    return vkold + (h - Skold) / (Sk - Skold) * (vk - vkold)


def _julia_hist_levels(v, w, nbins=8):
    """_histogram(values, weights) (src/utils.jl:134-141): edges = range(lo, hi, length=9)
    (correctly rounded here), searchsortedlast bins, ceil(counts / max * 8) levels."""
    import bisect
    from fractions import Fraction
    lo, hi = float(np.min(v)), float(np.max(v))
    if lo == hi:
        return [8] * nbins
    edges = [float(Fraction(lo) + (Fraction(hi) - Fraction(lo)) * k / nbins) for k in range(nbins + 1)]
    counts = np.zeros(nbins)
    for a, b in zip(v, w):
        counts[min(max(bisect.bisect_right(edges, a), 1), nbins) - 1] += b
    mx = counts.max()
    return [int(min(max(math.ceil(c / mx * 8), 1), 8)) for c in counts]


def _weights(o):
    lw = o.weights_download()
    w = np.exp(lw - lw.max())
    return w / w.sum()


@pytest.mark.parametrize("kind", ["normal", "ties", "zeros"])
def test_oracle_median_and_hist_match_restatements(kind):
    rng = np.random.default_rng(5)
    n = 3001
    o = Oracle(n, seed=2)
    c = o.col_create("a")
    a = rng.standard_normal(n) * 2.0
    lw = -0.5 * rng.standard_normal(n) ** 2
    if kind == "ties":
        a = np.round(a * 2) / 2                     # many equal values
    if kind == "zeros":
        lw[::3] = -np.inf                           # zero weights are dropped
    o.col_upload(c, a)
    o.weights_upload(lw)
    w = _weights(o)
    med = o.weighted_median(c)
    assert abs(med - _statsbase_median(a, w)) <= 1e-9 * max(1.0, abs(med))
    assert list(o.histogram(c)) == _julia_hist_levels(a, w)


def test_oracle_median_hist_edge_cases():
    o = Oracle(8, seed=1)
    c = o.col_create("a")
    o.col_upload(c, np.full(8, 2.5))
    assert o.weighted_median(c) == 2.5 and list(o.histogram(c)) == [8] * 8   # lo == hi
    v = np.arange(8.0)
    v[4] = np.nan
    o.col_upload(c, v)
    assert math.isnan(o.weighted_median(c))
    o1 = Oracle(1, seed=1)
    c1 = o1.col_create("a")
    o1.col_upload(c1, np.array([-3.0]))
    assert o1.weighted_median(c1) == -3.0


@pytest.mark.gpu
@pytest.mark.parametrize("N", [1, 999, 300001])
@pytest.mark.parametrize("kind", ["normal", "ties", "zeros"])
def test_median_hist_hip_matches_oracle(gpu_available, N, kind):
    rng = np.random.default_rng(N)
    g, o = wsmc.Context(N, seed=1), Oracle(N, seed=1)
    a = rng.standard_normal((2, N)) * [[1.0], [4.0]]
    lw = -0.5 * rng.standard_normal(N) ** 2
    if kind == "ties":
        a = np.round(a)
    if kind == "zeros" and N > 1:
        lw[::2] = -np.inf
    for ctx in (g, o):
        ctx.col_create("x2", 2)
        ctx.col_upload(0, a)
        ctx.weights_upload(lw)
    for comp in (0, 1):
        assert g.weighted_median(0, comp) == o.weighted_median(0, comp)
        np.testing.assert_array_equal(g.histogram(0, comp), o.histogram(0, comp))


@pytest.mark.gpu
def test_describe_median_hist_mirror(gpu_available):
    st = wsmc.SMCState(5000, seed=3)
    _setup(st.ctx)
    o = _setup(Oracle(5000, seed=3))
    rows = wsmc.describe(st)
    assert rows[0]["median"] == o.weighted_median(0)
    assert rows[0]["hist"] == "".join(wsmc.transformers.SPARK_CHARS[v - 1] for v in o.histogram(0))
    assert rows[1]["median"] == [o.weighted_median(1, 0), o.weighted_median(1, 1)] and rows[1]["hist"] == ""
