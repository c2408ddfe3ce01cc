"""sample(state, n; replace) and DataFrame(state) (src/utils.jl:69-118): the oracle's draws
against an independent Python restatement, their distribution, and the reference's
ArgumentErrors; the device path against the oracle (-m gpu)."""
import bisect
import math

import numpy as np
import pytest

import oracle as O
from oracle import Oracle
import wsmc
from wsmc import abi, models

L = O.lib()
MASK = (1 << 64) - 1


def _word(seed, op, n):
    z = seed ^ ((op * 0x9E3779B97F4A7C15) & MASK) ^ ((n * 0xD1B54A32D192ED03) & MASK) ^ 0x2545F4914F6CDD1D
    z ^= z >> 33
    z = (z * 0xFF51AFD7ED558CCD) & MASK
    z ^= z >> 33
    z = (z * 0xC4CEB9FE1A85EC53) & MASK
    z ^= z >> 33
    return z


def _state(lw, seed=3):
    o = Oracle(len(lw), seed=seed)
    c = o.col_create("x", 1)
    o.col_upload(c, np.arange(len(lw), dtype=float))
    v = o.col_create("v", 2)
    o.col_upload(v, np.stack([np.arange(len(lw), dtype=float), -np.arange(len(lw), dtype=float)]))
    o.weights_upload(lw)
    return o


def _q(o):
    w = o.weights_download()
    N = len(w)
    K, M = L.or_qbits(N), L.or_qref(float(np.max(w)))   # q against the reference point ceil(max)
    return [L.or_qweight(float(x), M, K) for x in w]


@pytest.mark.parametrize("N,n", [(1, 3), (10, 25), (1000, 777)])
def test_sample_with_replacement_restated(N, n):
    lw = np.random.default_rng(N).standard_normal(N) * 2
    lw[1::4] = -np.inf
    if N == 1:
        lw[0] = 0.0
    o = _state(lw, seed=5)
    op = o.get_state()["op_counter"]
    idx = o.sample_particles(n, replace=True)
    C, acc = [], 0
    for q in _q(o):
        acc += q
        C.append(acc)
    want = [bisect.bisect_right(C, (_word(5, op, j) * C[-1]) >> 64) for j in range(n)]
    np.testing.assert_array_equal(idx, want)
    assert o.get_state()["op_counter"] == op + 1          # one op, like the reference's RNG draw


@pytest.mark.parametrize("N,n", [(1, 1), (10, 10), (1000, 300)])
def test_sample_without_replacement_restated(N, n):
    lw = np.random.default_rng(N + 1).standard_normal(N)
    lw[2::5] = -np.inf
    if N == 1:
        lw[0] = 0.0
    o = _state(lw, seed=6)
    op = o.get_state()["op_counter"]
    idx = o.sample_particles(n, replace=False)
    keys = [L.or_es_key(6, op, i, q) for i, q in enumerate(_q(o))]
    order = sorted(range(N), key=lambda i: (-keys[i], i))
    np.testing.assert_array_equal(idx, order[:n])
    assert len(set(idx.tolist())) == n


def test_sample_frequencies():
    """With replacement the draws are Multinomial(n, w); without, heavier particles are
    included more often (inclusion probability increases with the weight)."""
    N, n = 50, 40000
    lw = np.log(np.arange(1, N + 1, dtype=float))
    o = _state(lw, seed=9)
    cnt = np.bincount(o.sample_particles(n, replace=True), minlength=N)
    w = np.arange(1, N + 1) / np.sum(np.arange(1, N + 1))
    chi2 = float(np.sum((cnt - n * w) ** 2 / (n * w)))
    assert abs(chi2 - (N - 1)) < 6 * math.sqrt(2 * N)
    inc = np.zeros(N)
    for r in range(400):
        inc[o.sample_particles(10, replace=False)] += 1
    assert inc[-10:].sum() > inc[:10].sum() * 5


def test_sample_argument_errors():
    o = _state(np.zeros(5))
    with pytest.raises(ValueError):
        o.sample_particles(0)
    with pytest.raises(ValueError):
        o.sample_particles(6, replace=False)
    o2 = _state(np.full(4, -np.inf))
    with pytest.raises(RuntimeError):
        o2.sample_particles(2)


# ---- device ----------------------------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("N", [1, 1000, 70001])
@pytest.mark.parametrize("replace", [True, False])
def test_sample_device_matches_oracle(gpu_available, N, replace):
    g, o = wsmc.Context(N, seed=12), Oracle(N, seed=12)
    obs = models.ssm1d_data(4)
    models.ssm1d_statements(g, obs, ess_perc_min=0.3)
    models.ssm1d_statements(o, obs, ess_perc_min=0.3)
    for n in sorted({1, max(1, N // 3), N}):
        a, b = g.sample_particles(n, replace), o.sample_particles(n, replace)
        np.testing.assert_array_equal(a, b)
        for name in o.col_names():
            np.testing.assert_array_equal(g.col_gather_rows(g.col_find(name), a),
                                          o.col_gather_rows(o.col_find(name), b), err_msg=name)
    assert g.get_state()["op_counter"] == o.get_state()["op_counter"]


@pytest.mark.gpu
def test_sample_device_skewed_and_errors(gpu_available):
    N = 3_000_001
    lw = np.full(N, -np.inf)
    lw[[5, 1_000_000, 2_999_999]] = [0.0, -1.0, -0.5]
    g, o = wsmc.Context(N, seed=2), Oracle(N, seed=2)
    for c in (g, o):
        c.weights_upload(lw)
    for replace in (True, False):
        np.testing.assert_array_equal(g.sample_particles(100, replace), o.sample_particles(100, replace))
    with pytest.raises(wsmc.WSMCError):
        g.sample_particles(0)
    with pytest.raises(wsmc.WSMCError):
        g.sample_particles(N + 1, replace=False)


@pytest.mark.gpu
def test_sample_and_dataframe_mirrors(gpu_available):
    st = wsmc.SMCState(2000, seed=4, ess_perc_min=0.5)
    models.ssm2d_statements(st.ctx, models.ssm2d_data(3))
    s = wsmc.sample(st, 50)
    assert set(s) == set(st.store.colnames()) and s["x_4"].shape == (50, 2)
    df = wsmc.dataframe(st)
    assert df["log_weight"].shape == (2000,) and df["v"].shape == (2000, 2)
