"""The per-particle math of every config against independent numpy f64 restatements.

The bit-exact parity tests compare the HIP library with the oracle, and both compile the same
include/wsmc_math.h / include/wsmc_terms.h. A bug shared by those headers would be invisible
to them. This file closes that gap: it re-derives each step of the configs' models from the
reference's own definitions with numpy/libm f64 (tests/refmath.py; nothing from the headers),
fed the build's random stream (Philox4x32-10 + Box–Muller, restated from its definition), and
checks the oracle (CPU) and, under -m gpu, the HIP library through the C ABI:

  (a) one 2D-SSM step (examples/2D_ssm.jl:7-17): x{t+1} = x{t} + v exactly, dv ~ MvNormal(0,
      0.1 I) with 0.1 I a COVARIANCE (sd √0.1), v += dv, and o_t => MvNormal(x{t+1}, 0.5 I)
      through the general Cholesky logpdf (src/default_kernels.jl:12-23), then the Resample
      (src/transformers.jl:474-498, restated in tests/test_resample_reference.py) and the
      gather of every column through its ancestors (src/stores.jl:105-128);
  (b) C3's Normal prior draws and Observe terms (examples/linear_regression.jl:17-27), and the
      score fold with its depth cutoff (src/types.jl:198-206) at every depth;
  (c) autoRW (src/move_kernels.jl:144-151): the uncorrected weighted covariance, the min_step
      fill, λ = 2.38/√d, the Cholesky draw, the MH acceptance of src/transformers.jl:604-621
      with s_old and s_new refolded from scratch (the build carries s_old), and RW's std step;
  (d) the bounded transforms and log|J| (src/move_kernels.jl:37-85) through C5's (0, ∞) 4-D and
      (−π, π) 1-D moves;
  (e) C5's priors (HalfNormal = Truncated(Normal(0, σ), 0, Inf), Uniform(−π, π)) and its
      oscillator Observe term A·exp(−γt)·cos(ωt + ϕ) (examples/damped_oscillator.jl:11, 24-43),
      evaluated directly (the build rolls a phasor).

Tolerances (written here, the north star's bar is 1e-6 relative on log-weights):
  * draws, columns, log-weights, scores: |a − b| ≤ 1e-12 · max(1, |b|)   (libm vs restated ulps)
  * resample decisions identical; ancestors identical except CDF-resolution ties (counted,
    tests/test_resample_reference.py)
  * accept decisions identical except where |log u − (log_pratio + s_new − s_old)| ≤ 1e-9 ·
    max(1, |s_old|) (counted; none expected)
"""
from __future__ import annotations

import math

import numpy as np
import pytest

import refmath as R
import wsmc
from backends import BACKENDS, make_ctx
from test_resample_reference import RefResample, check_against_reference
from wsmc.dsl import Col, HalfNormal, MvNormal, Normal, Oscillator, Uniform, value_operands
from wsmc.models import linreg_data, oscillator_data, resolver, ssm2d_data

RTOL = 1e-12
SEED = 20260101


def _const(vals):
    return [wsmc.abi.Operand.const(float(v)) for v in vals]


def _assert_close(a, b, what, rtol=RTOL):
    ok = R.close(a, b, rtol)
    if not np.all(ok):
        i = int(np.argmin(ok.ravel()))
        raise AssertionError(f"{what}: {np.count_nonzero(~ok)} values differ beyond {rtol}; "
                             f"first {np.ravel(a)[i]!r} vs {np.ravel(b)[i]!r}")


def _cols(ctx, names):
    return {n: ctx.col_download(ctx.col_find(n)) for n in names}


# ---------------------------------------------------------------------------------------
# the random stream restatement itself
# ---------------------------------------------------------------------------------------
def test_numpy_philox_random123_kat():
    """Random123 kat_vectors for philox4x32_10 (the same vectors the oracle is held to)."""
    kat = [([0, 0, 0, 0], [0, 0], [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]),
           ([0xffffffff] * 4, [0xffffffff] * 2, [0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd]),
           ([0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344], [0xa4093822, 0x299f31d0],
            [0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1])]
    for ctr, key, want in kat:
        got = R.philox4x32_10(*[np.array([c], dtype=np.uint32) for c in ctr], *key)
        assert [int(g[0]) for g in got] == want


def test_numpy_draws_match_oracle_stream():
    """The numpy stream (libm log/sqrt/cos/sin) equals the build's restated one to 1e-12."""
    from oracle import lib
    L = lib()
    idx = np.arange(0, 20000, 7, dtype=np.uint64)
    for seed, op in [(42, 0), (SEED, 12345), (2 ** 63 + 11, 2 ** 33 + 5)]:
        for k in range(4):
            want = np.array([L.or_normal_k(seed, op, int(i), k) for i in idx])
            _assert_close(R.normal_k(seed, op, idx, k), want, f"normal k={k}")
            wu = np.array([L.or_uniform_k(seed, op, int(i), k) for i in idx])
            np.testing.assert_array_equal(R.uniform_k(seed, op, idx, k), wu)   # integer words: exact


# ---------------------------------------------------------------------------------------
# shared checks
# ---------------------------------------------------------------------------------------
def checked_resample(ctx, ess_min, scheme, n):
    """Resample.apply! against the numpy restatement of src/transformers.jl:474-498; every
    column is checked to be gathered through the ancestors. Returns the resampled flag."""
    st = ctx.get_state()
    names = ctx.col_names()
    before = _cols(ctx, names)
    lw = ctx.weights_download()
    op = st["op_counter"]
    ev = ctx.log_evidence()
    rs, ess = ctx.resample(ess_min, scheme)
    if not st["weights_changed"]:
        # the gate (src/transformers.jl:475-477): nothing moves, `resampled` keeps its value
        assert rs == bool(st["resampled"])
        np.testing.assert_array_equal(ctx.weights_download(), lw)
        for nm in names:
            np.testing.assert_array_equal(ctx.col_download(ctx.col_find(nm)), before[nm])
        return False
    ref = RefResample(lw, ess_min, SEED, op, scheme)
    anc = ctx.last_ancestors() if rs else None
    out = dict(ess=ess, rs=rs, ev=ev, w=ctx.weights_download(),
               id=anc.astype(np.float64) if rs else None, anc=anc)
    # all-equal weights decide on the exact ESS of 1 (a chosen semantics): the
    # reference's f64 ESS of such a vector is 1 only up to rounding (1 - 7e-16 at N = 100,003)
    check_against_reference("all_equal" if np.all(lw == lw[0]) else "model", lw, out, ref, ess_min)
    after = _cols(ctx, names)
    for nm in names:
        want = before[nm][..., anc] if rs else before[nm]
        np.testing.assert_array_equal(after[nm], want, err_msg=f"column {nm} after Resample")
    return rs


def checked_move(ctx, targets, fold, n, min_step=1e-3, lo=None, hi=None, proposal=None, step=None):
    """One autoRW (or RW) Move against the numpy restatement: the covariance and factor, the
    proposal, the Jacobian, both score folds refolded from scratch and the MH decision.
    `fold(values)` is the model's score over a dict of column values. Returns the number of
    accept-decision ties (|log u - (lpr + s_new - s_old)| within 1e-9)."""
    proposal = wsmc.PROPOSAL_AUTORW if proposal is None else proposal
    st = ctx.get_state()
    op_prop, op_acc = st["op_counter"], st["op_counter"] + 1
    names = ctx.col_names()
    cur = _cols(ctx, names)
    lw = ctx.weights_download()
    d = len(targets)
    lo_ = [-math.inf] * d if lo is None else lo
    hi_ = [math.inf] * d if hi is None else hi
    bounded = lo is not None or hi is not None
    X = np.array([cur[t] for t in targets])
    Z = np.array([R.to_unconstrained(X[k], lo_[k], hi_[k]) for k in range(d)]) if bounded else X
    if proposal == wsmc.PROPOSAL_AUTORW:
        _, Lf = R.autorw_factor(Z, lw, min_step)
    else:
        Lf = step * np.eye(d)                    # RW: std `step` (src/move_kernels.jl:189-212)
    idx = np.arange(n, dtype=np.uint64)
    xi = np.array([R.normal_k(SEED, op_prop, idx, k) for k in range(d)])
    Zn = Z + Lf @ xi
    Xn = np.array([R.from_unconstrained(Zn[k], lo_[k], hi_[k]) for k in range(d)]) if bounded else Zn
    lpr = np.zeros(n)
    if bounded:
        for k in range(d):
            lpr = lpr + (R.log_abs_jacobian(Zn[k], lo_[k], hi_[k]) - R.log_abs_jacobian(Z[k], lo_[k], hi_[k]))
    prop = dict(cur)
    for k, t in enumerate(targets):
        prop[t] = Xn[k]
    s_old, s_new = fold(cur), fold(prop)
    log_u = np.log(R.uniform_k(SEED, op_acc, idx, 0))
    acc_ref = R.mh_accept(log_u, lpr, s_new, s_old)

    cids = [ctx.col_find(t) for t in targets]
    kw = dict(lo=lo, hi=hi)
    n_acc = ctx.move(proposal, cids, min_step if proposal == wsmc.PROPOSAL_AUTORW else step, **kw)
    Xa = np.array([ctx.col_download(c) for c in cids])
    acc_dev = np.any(Xa != X, axis=0)
    assert n_acc == int(np.count_nonzero(acc_dev)), "accepted count vs changed particles"
    with np.errstate(invalid="ignore"):
        margin = np.abs(log_u - ((lpr + s_new) - s_old))
    mism = acc_dev != acc_ref
    tol = 1e-9 * np.maximum(1.0, np.abs(s_old))
    bad = mism & ~(margin <= tol)
    assert not np.any(bad), (f"{int(bad.sum())} accept decisions differ away from a tie; first particle "
                             f"{int(np.argmax(bad))}: margin {margin[np.argmax(bad)]}")
    both = acc_dev & acc_ref
    _assert_close(Xa[:, both], Xn[:, both], f"accepted proposals of {targets}")
    rej = ~acc_dev
    np.testing.assert_array_equal(Xa[:, rej], X[:, rej])
    np.testing.assert_array_equal(ctx.weights_download(), lw)          # a Move never reweights
    return int(np.count_nonzero(mism))


# ---------------------------------------------------------------------------------------
# (a) the 2D SSM step
# ---------------------------------------------------------------------------------------
def run_ssm2d_checked(backend, n, T, ess_min, scheme=wsmc.RESAMPLE_STRATIFIED):
    ctx = make_ctx(backend, n, seed=SEED)
    Rz = resolver(ctx)
    obs = ssm2d_data(T)
    q_var, r_var = 0.1, 0.5
    I2 = np.eye(2)
    idx = np.arange(n, dtype=np.uint64)
    cx1 = ctx.col_create("x_1", 2)
    ctx.assign(cx1, _const((0.0, 0.0)))
    cv = ctx.col_create("v", 2)
    ctx.assign(cv, _const((1.0, 0.0)))
    dv_dist = MvNormal([0.0, 0.0], q_var * I2).dist(Rz)
    cdv, n_rs = -1, 0
    for t, o in enumerate(obs, start=1):
        xt, xn = f"x_{t}", f"x_{t + 1}"
        X = ctx.col_download(ctx.col_find(xt))
        V = ctx.col_download(cv)
        W = ctx.weights_download()
        cxn = ctx.col_create(xn, 2)
        if t == 1:
            cdv = ctx.col_create("dv", 2)
        ctx.assign(cxn, value_operands(Col(xt) + Col("v"), 2, Rz))         # x{t+1} .= x{t} + v
        Xn = ctx.col_download(cxn)
        np.testing.assert_array_equal(Xn, X + V)
        op = ctx.get_state()["op_counter"]
        ctx.sample(cdv, dv_dist)                                            # dv ~ MvNormal(0, 0.1 I)
        z0, z1 = R.normal_pair(SEED, op, idx, 0)
        sd = math.sqrt(q_var)                                               # 0.1 I is a covariance
        dv = ctx.col_download(cdv)
        _assert_close(dv, np.array([sd * z0, sd * z1]), f"dv at t={t}")
        checked_resample(ctx, ess_min, scheme, n)                           # auto-inserted no-op
        ctx.assign(cv, value_operands(Col("v") + Col("dv"), 2, Rz))         # v .= v + dv
        np.testing.assert_array_equal(ctx.col_download(cv), V + dv)
        ctx.observe(MvNormal(Col(xn), r_var * I2).dist(Rz), _const(o))      # o => MvNormal(x{t+1}, 0.5 I)
        want = W + R.mvnormal_logpdf(np.asarray(o)[:, None], Xn, r_var * I2)
        _assert_close(ctx.weights_download(), want, f"log-weights at t={t}")
        n_rs += checked_resample(ctx, ess_min, scheme, n)
    ctx.close()
    return n_rs


@pytest.mark.parametrize("backend", BACKENDS)
@pytest.mark.parametrize("ess_min", [0.5, 1.0])
def test_ssm2d_steps_match_reference_math(backend, ess_min, request):
    if backend == "hip":
        request.getfixturevalue("gpu_available")
    n = 4096 if backend == "oracle" else 100_003
    n_rs = run_ssm2d_checked(backend, n, 8, ess_min)
    # step 1 observes x_2 = x_1 + v, equal for every particle: ESS is exactly 1, no resample
    assert n_rs >= (7 if ess_min == 1.0 else 1)


@pytest.mark.gpu
def test_ssm2d_systematic_steps_match_reference_math(gpu_available):
    assert run_ssm2d_checked("hip", 65_537, 6, 0.7, wsmc.RESAMPLE_SYSTEMATIC) >= 1


# ---------------------------------------------------------------------------------------
# (b) + (c) linear regression: Normal terms, score fold with depth, autoRW and RW
# ---------------------------------------------------------------------------------------
def linreg_fold(xs_seen, ys_seen, prior_sd=10.0, obs_sd=1.0):
    """score_logpdf over α, β priors and the observations so far (src/types.jl:198-206: 0.0,
    then += each term in program order)."""
    def fold(cols, depth=None):
        a, b = cols["α"], cols["β"]
        terms = [lambda: R.normal_logpdf(a, 0.0, prior_sd), lambda: R.normal_logpdf(b, 0.0, prior_sd)]
        terms += [(lambda x=x, y=y: R.normal_logpdf(y, a + b * x, obs_sd)) for x, y in zip(xs_seen, ys_seen)]
        s = np.zeros(len(a))
        for j, term in enumerate(terms):
            if depth is not None and j >= depth:
                break
            s = s + term()
        return s
    return fold


@pytest.mark.parametrize("backend", BACKENDS)
@pytest.mark.parametrize("ess_min", [1.0, 0.5])
def test_linreg_terms_fold_and_moves_match_reference_math(backend, ess_min, request):
    if backend == "hip":
        request.getfixturevalue("gpu_available")
    n = 4096 if backend == "oracle" else 200_000
    ctx = make_ctx(backend, n, seed=SEED)
    Rz = resolver(ctx)
    idx = np.arange(n, dtype=np.uint64)
    xs, ys = linreg_data()
    for name in ("α", "β"):
        c = ctx.col_create(name, 1)
        op = ctx.get_state()["op_counter"]
        ctx.sample(c, Normal(0.0, 10.0).dist(Rz))
        _assert_close(ctx.col_download(c), 10.0 * R.normal_k(SEED, op, idx, 0), f"prior draw {name}")
        checked_resample(ctx, ess_min, wsmc.RESAMPLE_STRATIFIED, n)
    ties = moves = 0
    for k, (x, y) in enumerate(zip(xs, ys)):
        W = ctx.weights_download()
        cur = _cols(ctx, ["α", "β"])
        ctx.observe(Normal(Col("α") + Col("β") * float(x), 1.0).dist(Rz), _const([y]))
        _assert_close(ctx.weights_download(), W + R.normal_logpdf(y, cur["α"] + cur["β"] * x, 1.0),
                      f"Observe at x={x}")
        fold = linreg_fold(xs[:k + 1], ys[:k + 1])
        depth = ctx.get_state()["depth"]
        for dd in range(depth + 1):                   # the depth cutoff (test/score_test.jl:20-54)
            _assert_close(ctx.score(dd), fold(cur, dd), f"score at depth {dd}")
        if checked_resample(ctx, ess_min, wsmc.RESAMPLE_STRATIFIED, n):
            ties += checked_move(ctx, ["α"], fold, n)
            ties += checked_move(ctx, ["β"], fold, n)
            moves += 2
    # RW with a std step, unbounded (x + step randn) and bounded (walk in log space)
    ties += checked_move(ctx, ["α"], fold, n, proposal=wsmc.PROPOSAL_RW, step=0.3)
    ties += checked_move(ctx, ["α", "β"], fold, n, proposal=wsmc.PROPOSAL_AUTORW, min_step=1e-3)
    assert moves >= 2
    assert ties <= 2, ties
    ctx.close()


# ---------------------------------------------------------------------------------------
# (d) + (e) damped oscillator: priors, oscillator Observe, bounded autoRW
# ---------------------------------------------------------------------------------------
PRIORS = [("A", "half", 5.0), ("ω", "half", 5.0), ("γ", "half", 1.0), ("ϕ", "unif", math.pi), ("σ", "half", 1.0)]


def oscillator_fold(ts, ys):
    def fold(cols):
        s = np.zeros(len(cols["A"]))
        for name, kind, p in PRIORS:
            s = s + (R.halfnormal_logpdf(cols[name], p) if kind == "half" else R.uniform_logpdf(cols[name], -p, p))
        for t, y in zip(ts, ys):
            mu = R.oscillator(t, cols["A"], cols["ω"], cols["γ"], cols["ϕ"])
            s = s + R.normal_logpdf(y, mu, cols["σ"])
        return s
    return fold


def run_oscillator_checked(backend, n, T, sweeps, scheme, ess_min=1.0, obs_rtol=1e-12):
    ctx = make_ctx(backend, n, seed=SEED)
    Rz = resolver(ctx)
    idx = np.arange(n, dtype=np.uint64)
    kern = {"half": HalfNormal, "unif": lambda p: Uniform(-p, p)}
    for name, kind, p in PRIORS:
        c = ctx.col_create(name, 1)
        op = ctx.get_state()["op_counter"]
        ctx.sample(c, kern[kind](p).dist(Rz))
        if kind == "half":   # rand(Truncated(Normal(0, σ), 0, Inf)) = σ |z|
            want = p * np.abs(R.normal_k(SEED, op, idx, 0))
        else:
            want = -p + (p - -p) * R.uniform_k(SEED, op, idx, 0)
        _assert_close(ctx.col_download(c), want, f"prior draw {name}")
        checked_resample(ctx, ess_min, scheme, n)
    ts, ys = oscillator_data()
    ts, ys = ts[:T], ys[:T]
    joint = ["A", "ω", "γ", "σ"]
    ties = 0
    for k, (t, y) in enumerate(zip(ts, ys)):
        W = ctx.weights_download()
        cur = _cols(ctx, [p[0] for p in PRIORS])
        mean = Oscillator(float(t), Col("A"), Col("ω"), Col("γ"), Col("ϕ"))
        ctx.observe(Normal(mean, Col("σ")).dist(Rz), _const([y]))
        inc = R.normal_logpdf(y, R.oscillator(t, cur["A"], cur["ω"], cur["γ"], cur["ϕ"]), cur["σ"])
        _assert_close(ctx.weights_download(), W + inc, f"oscillator Observe at t={t:.4f}", obs_rtol)
        fold = oscillator_fold(ts[:k + 1], ys[:k + 1])
        # the absolute score (priors' normalising constants included; the MH ratio cancels them)
        _assert_close(ctx.score(ctx.get_state()["depth"]), fold(cur), f"score after t={t:.4f}", obs_rtol)
        checked_resample(ctx, ess_min, scheme, n)
        for _ in range(sweeps):
            ties += checked_move(ctx, joint, fold, n, lo=[0.0] * 4, hi=[math.inf] * 4)
            ties += checked_move(ctx, ["ϕ"], fold, n, lo=[-math.pi], hi=[math.pi])
    ctx.close()
    return ties


@pytest.mark.parametrize("scheme", [wsmc.RESAMPLE_STRATIFIED, wsmc.RESAMPLE_SYSTEMATIC])
def test_oscillator_matches_reference_math_oracle(scheme):
    assert run_oscillator_checked("oracle", 2048, 6, 2, scheme) <= 2


@pytest.mark.gpu
@pytest.mark.parametrize("scheme", [wsmc.RESAMPLE_SYSTEMATIC, wsmc.RESAMPLE_STRATIFIED])
def test_oscillator_full_horizon_matches_reference_math_hip(scheme, gpu_available):
    """C5's 60 observations (the rotation blocks included), one sweep per step."""
    assert run_oscillator_checked("hip", 16_384, 60, 1, scheme) <= 4


# ---------------------------------------------------------------------------------------
# the one-pass autoRW covariance with an outlying pivot
# ---------------------------------------------------------------------------------------
@pytest.mark.parametrize("D", [0.0, 1e2, 1e4])
def test_autorw_pivot_outlier_error_bound(D):
    """wsmc_autorw_factor takes the population's particle 0 as the pivot of its one-pass
    moments (S = T2/T0 - m m^T relative to it). With particle 0 D standard deviations from the
    weighted mean and a weight of e^-600, the cancellation costs about eps (D/sd)^2 relative:
    measured here against the numpy two-pass covariance (tests/refmath.py) — 1e-12 at D = 0,
    within 64 eps D^2 beyond. The configs' pivots sit inside the weighted mass (D of a few)."""
    from oracle import Oracle
    n = 4096
    rng = np.random.default_rng(7)
    Z = rng.normal(0.0, 1.0, size=(2, n))
    Z[1] = 0.5 * Z[0] + Z[1]
    Z[:, 0] = (D, -D)
    lw = rng.normal(0.0, 0.3, size=n)
    lw[0] = -600.0
    o = Oracle(n, seed=SEED)
    ca, cb = o.col_create("a"), o.col_create("b")
    o.col_upload(ca, Z[0])
    o.col_upload(cb, Z[1])
    o.weights_upload(lw)
    ok, cov, _ = o.autorw_cov([ca, cb], 1e-3)
    assert ok
    want, _ = R.autorw_factor(Z, lw, 1e-3)
    rel = np.max(np.abs(cov - want)) / np.max(np.abs(want))
    bound = max(1e-12, 64 * np.finfo(float).eps * D * D)
    assert rel <= bound, (D, rel, bound)
    o.close()
