"""MvNormal(μ, Σ) with a full constant covariance (src/default_kernels.jl:93; Distributions'
MvNormal factors Σ once through PDMats): the WSMC_FAM_MVNORMAL family, dim ≤ 3.

Independent pins (nothing imported from the shared headers): draws against μ + chol(Σ)·z with
numpy's own Cholesky and the numpy Philox/Box–Muller restatement of the stream, log-weights
against refmath.mvnormal_logpdf (-(d log 2π + log det Σ + rᵀ Σ⁻¹ r)/2 through numpy's solve),
both within 1e-12 relative; the oracle and the HIP path against them, and the HIP path bit for
bit against the oracle, including a Move whose score fold carries a full-covariance term and a
statement batch (consecutive Sample / Observe / Weight join one kernel on the device).
"""
import math

import numpy as np
import pytest

import refmath as R
import wsmc
from backends import BACKENDS, make_ctx
from oracle import Oracle
from wsmc import abi
from wsmc.dsl import Col, MvNormal, Normal
from wsmc.models import resolver

SEED = 977
RTOL = 1e-12
COVS = {
    2: np.array([[1.0, 0.6], [0.6, 2.0]]),
    3: np.array([[2.0, 0.3, -0.5], [0.3, 1.0, 0.2], [-0.5, 0.2, 1.5]]),
}


def _const(vals):
    return [abi.Operand.const(float(v)) for v in vals]


def _close(a, b, what):
    ok = R.close(a, b, RTOL)
    assert np.all(ok), f"{what}: {np.count_nonzero(~ok)} values beyond {RTOL}"


def _program(ctx, d, checked):
    """m ~ Normal(0, 1); x ~ MvNormal([m, 0.5, ...], Σ); o => MvNormal(x + m, Σ); returns
    nothing, checks every step against numpy when `checked`."""
    Rz = resolver(ctx)
    S = COVS[d]
    cm = ctx.col_create("m")
    ctx.sample(cm, Normal(0.0, 1.0).dist(Rz))
    cx = ctx.col_create("x", d)
    mean = [Col("m")] + [0.5] * (d - 1)
    op = ctx.get_state()["op_counter"]
    ctx.sample(cx, MvNormal(mean, S).dist(Rz))
    obs = [0.3, -0.4, 1.1][:d]
    ctx.observe(MvNormal([Col("x", k) + Col("m") for k in range(d)], S).dist(Rz), _const(obs))
    ctx.weight(MvNormal([0.1] * d, S).dist(Rz), [abi.Operand.column(cx, k) for k in range(d)])
    if not checked:
        return
    m = ctx.col_download(cm)
    x = ctx.col_download(cx).reshape(d, -1)
    n = m.shape[0]
    idx = np.arange(n, dtype=np.uint64)
    z = np.array([R.normal_k(SEED, op, idx, k) for k in range(d)])
    L = np.linalg.cholesky(S)
    mu = np.array([m] + [np.full(n, 0.5)] * (d - 1))
    _close(x, mu + L @ z, f"draws d={d}")
    want = R.mvnormal_logpdf(np.asarray(obs)[:, None], x + m, S)
    want = want + R.mvnormal_logpdf(x, np.full((d, 1), 0.1), S)
    _close(ctx.weights_download(), want, f"log-weights d={d}")


@pytest.mark.parametrize("backend", BACKENDS)
@pytest.mark.parametrize("d", [2, 3])
def test_full_covariance_matches_numpy(backend, d, request):
    if backend == "hip":
        request.getfixturevalue("gpu_available")
    n = 2000 if backend == "oracle" else 100_003
    ctx = make_ctx(backend, n, seed=SEED)
    _program(ctx, d, checked=True)
    ctx.close()


@pytest.mark.gpu
@pytest.mark.parametrize("d", [2, 3])
def test_full_covariance_device_bit_exact(gpu_available, d):
    """The HIP path against the oracle, bit for bit: the statements, a Resample, then Moves
    whose fold scores the full-covariance terms."""
    from test_gpu_parity import assert_same_state
    g, o = wsmc.Context(4099, seed=SEED), Oracle(4099, seed=SEED)
    accs = []
    for c in (g, o):
        _program(c, d, checked=False)
        c.resample(1.0)
        cm = c.col_find("m")
        acc = [c.move(abi.PROPOSAL_RW, [cm], 0.4), c.move(abi.PROPOSAL_AUTORW, [cm], 1e-3)]
        accs.append(acc)
    assert accs[0] == accs[1]
    assert_same_state(g, o)
    g.close()
    o.close()


def test_full_covariance_arguments():
    """Σ must be exactly symmetric (LinearAlgebra.cholesky's ishermitian check) and positive
    definite (PosDefException); dim ≤ 3 for a full Σ; Σ = v·I keeps the isotropic family."""
    Rz = lambda name: 0
    with pytest.raises(wsmc.WSMCError) as e:
        MvNormal([0.0, 0.0], np.array([[1.0, 0.5], [0.4, 1.0]])).dist(Rz)
    assert e.value.code == abi.WSMC_EARG
    with pytest.raises(wsmc.WSMCError) as e:
        MvNormal([0.0, 0.0], np.array([[1.0, 2.0], [2.0, 1.0]])).dist(Rz)
    assert e.value.code == abi.WSMC_ENOTPD
    with pytest.raises(ValueError):
        MvNormal([0.0] * 4, np.diag([1.0, 2.0, 3.0, 4.0]))
    assert MvNormal([0.0, 0.0], 0.5 * np.eye(2)).family == abi.FAM_MVNORMAL_ISO
    k = MvNormal([0.0, 0.0, 0.0], COVS[3])
    d = k.dist(Rz)
    assert d.family == abi.FAM_MVNORMAL
    # every operand stays a constant: the packed factor never reads as a column
    for o in list(d.mu) + [d.scale]:
        assert o.col[0] == -1 and o.col[1] == -1
    assert k.columns() == []


def test_full_covariance_packing_is_the_cholesky_factor():
    """The packed numbers (wsmc_terms.h layout) are numpy's Cholesky factor and log det Σ."""
    for d, S in COVS.items():
        dist = MvNormal([0.0] * d, S).dist(lambda name: 0)
        fields = []
        for k in range(d, 4):
            o = dist.mu[k]
            fields += [o.c0, o.coef[0], o.coef[1]]
        fields += [dist.scale.c0, dist.scale.coef[0], dist.scale.coef[1], dist.param[0], dist.param[1]]
        L = np.linalg.cholesky(S)
        want = [L[i, j] for i in range(d) for j in range(i + 1)] + [2.0 * np.sum(np.log(np.diag(L)))]
        _close(np.array(fields[:len(want)]), np.array(want), f"packed factor d={d}")
        assert math.isfinite(fields[len(want) - 1])


def test_full_covariance_c_abi_rejections():
    """wsmc_dist_mvnormal_cov through the C ABI (host only): dim outside 1..3, an oscillator
    mean and null pointers are argument errors; the dist is untouched by a rejection."""
    import ctypes as C
    lib = abi.load_library()
    S = (C.c_double * 16)(*np.eye(4).ravel())
    d = abi.Dist()
    d.dim = 4
    assert lib.wsmc_dist_mvnormal_cov(C.byref(d), S) == abi.WSMC_EARG
    assert d.family == 0
    d.dim, d.mean_fn = 2, abi.MEAN_OSCILLATOR
    assert lib.wsmc_dist_mvnormal_cov(C.byref(d), S) == abi.WSMC_EARG
    assert lib.wsmc_dist_mvnormal_cov(None, S) == abi.WSMC_EARG
    d.mean_fn = abi.MEAN_AFFINE
    S2 = (C.c_double * 4)(4.0, 2.0, 2.0, 5.0)
    assert lib.wsmc_dist_mvnormal_cov(C.byref(d), S2) == abi.WSMC_OK
    assert d.family == abi.FAM_MVNORMAL
    # L = [[2, 0], [1, 2]]: packed into mu[2].c0, mu[2].coef[0], mu[2].coef[1], then mu[3].c0
    assert (d.mu[2].c0, d.mu[2].coef[0], d.mu[2].coef[1]) == (2.0, 1.0, 2.0)
    assert d.mu[3].c0 == 2.0 * (math.log(2.0) + math.log(2.0))
