"""The Resample numerics against an independent f64 restatement of the reference.

`RefResample` below restates src/resampling.jl:13-77 and the decision of
src/transformers.jl:474-498 in numpy f64, exactly as the reference computes them (exp_norm,
ess_perc = 1/(N sum w^2), logsumexp, the stratified uniforms us[n] = (n-1)/N + rand()/N and
the sequential icdf merge). It uses nothing from include/wsmc_math.h: the build's integer
CDF, fixed-point sums and rank arithmetic are never consulted. The only shared input is the
uniform each slot draws (`rand()` of src/resampling.jl:40 is the build's 32-bit stratum word,
restated below from its definition, a keyed lowbias32 hash of the slot), so
the two sides resample the same weights with the same uniforms.

Checked on benign, heavy-tailed, dominant, near-threshold (ESS = 0.5 +- 1e-6), -Inf,
all-equal and very wide weight vectors, on the oracle (CPU) and, under -m gpu, on the HIP
library through the C ABI:
  * ESS%         relative difference <= 1e-12 (exact 85-bit sums)
  * log-mean     (logsumexp - log N, the value weights are reset to) within 1e-12
  * decision     identical (strict <, src/transformers.jl:484)
  * ancestors    identical, except slots whose uniform lies within the integer CDF's
                 resolution of a CDF boundary: every q_i = floor(e_i 2^K) drops < 1 unit,
                 so the integer CDF sits within (m+1) units of the exact one at particle m
                 and a disagreement needs |C_m - u_n| <= 2(N+1)/Q. Those ties are counted
                 and reported (identical weights make the truncation systematic, so the
                 dominant-particle cases show the most: ~0.07 % of slots at N = 300001).
The all-equal-weights case is the documented semantic choice: the build's
ESS is exactly 1, the reference's f64 value is 1 up to rounding.
"""
import math

import numpy as np
import pytest

import wsmc
from backends import make_ctx
from wsmc.dsl import Uniform
from wsmc.models import resolver

M32 = (1 << 32) - 1
M64 = (1 << 64) - 1


# ---------------------------------------------------------------------------------------
# the reference, restated in numpy f64 (src/resampling.jl, src/transformers.jl:474-498)
# ---------------------------------------------------------------------------------------
def ref_exp_norm(lw):
    """exp_norm (src/resampling.jl:72-77)."""
    m = np.max(lw)
    w = np.exp(lw - m)
    return w / np.sum(w)


def ref_ess_perc(w):
    """ess_perc (src/resampling.jl:51-54)."""
    return 1.0 / (len(w) * np.sum(w * w))


def ref_logsumexp(lw):
    """logsumexp (src/resampling.jl:61-64)."""
    m = np.max(lw)
    return m + math.log(np.sum(np.exp(lw - m)))


def ref_stratified_us(n, rand):
    """us[n] = (n-1)*inv_N + rand()*inv_N, n = 1..N (src/resampling.jl:38-41), 0-based here."""
    inv_n = 1.0 / n
    return np.arange(n, dtype=np.float64) * inv_n + rand * inv_n


def ref_icdf(w, us):
    """icdf (src/resampling.jl:13-26): s = w[1]; while s < us[n]: m += 1; s += w[m].
    The running s is a sequential f64 sum (np.cumsum adds left to right), and the merge's
    answer for slot n is the smallest m with s_m >= us[n] (searchsorted 'left'). Slots past
    the last running sum would be the reference's BoundsError; they are returned as N."""
    c = np.cumsum(w)
    return np.searchsorted(c, us, side="left"), c


def strat_key(seed, op):
    """The per-Resample key: murmur3's fmix64 over (seed, op)."""
    z = (seed ^ ((op * 0x9E3779B97F4A7C15) & M64) ^ 0x5851F42D4C957F2D) & M64
    z ^= z >> 33
    z = (z * 0xFF51AFD7ED558CCD) & M64
    z ^= z >> 33
    z = (z * 0xC4CEB9FE1A85EC53) & M64
    z ^= z >> 33
    return z


def strat_word(seed, op, n):
    """The 32-bit uniform word of resampling slot n (the build's stream for rand() of
    src/resampling.jl:40): the keyed lowbias32 hash of the slot."""
    k = strat_key(seed, op)
    x = (n ^ k) & M32
    x ^= (((n >> 32) * 0x85EBCA6B) & M32) ^ (k >> 32)
    x ^= x >> 16
    x = (x * 0x7FEB352D) & M32
    x ^= x >> 15
    x = (x * 0x846CA68B) & M32
    x ^= x >> 16
    return x


def strat_words(seed, op, n, start=0):
    k = strat_key(seed, op)
    idx = np.arange(start, start + n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        x = ((idx ^ np.uint64(k)) & np.uint64(M32)).astype(np.uint32)
        x ^= ((idx >> np.uint64(32)).astype(np.uint32) * np.uint32(0x85EBCA6B)) ^ np.uint32(k >> 32)
        x ^= x >> np.uint32(16)
        x *= np.uint32(0x7FEB352D)
        x ^= x >> np.uint32(15)
        x *= np.uint32(0x846CA68B)
        x ^= x >> np.uint32(16)
    return x.astype(np.float64)


class RefResample:
    """Resample.apply! of src/transformers.jl:474-498 on a weight vector."""

    def __init__(self, lw, ess_min, seed, op, scheme=wsmc.RESAMPLE_STRATIFIED):
        lw = np.asarray(lw, dtype=np.float64)
        n = len(lw)
        self.w = ref_exp_norm(lw)
        self.ess = ref_ess_perc(self.w)
        self.resampled = self.ess < ess_min
        self.mean = ref_logsumexp(lw) - math.log(n)
        r = strat_words(seed, op, n) / 4294967296.0
        if scheme == wsmc.RESAMPLE_SYSTEMATIC:
            r = np.full(n, r[0])
        self.us = ref_stratified_us(n, r)
        self.anc, self.cdf = ref_icdf(self.w, self.us)


# ---------------------------------------------------------------------------------------
# weight vectors
# ---------------------------------------------------------------------------------------
def near_threshold(n, target, rng):
    """Two-level weights (a fraction p at log a, the rest at 0) with ESS% = target."""
    k = n // 4
    p = k / n
    # ESS = (p a + 1 - p)^2 / (p a^2 + 1 - p) = target, solved for a > 1
    A = p * p - target * p
    B = 2 * p * (1 - p)
    Cc = (1 - p) ** 2 - target * (1 - p)
    a = (-B - math.sqrt(B * B - 4 * A * Cc)) / (2 * A)
    lw = np.zeros(n)
    lw[rng.permutation(n)[:k]] = math.log(a)
    return lw


def weight_cases(n, rng):
    z = rng.standard_normal(n)
    yield "benign", -0.5 * z * z
    yield "heavy_tailed", 3.0 * np.log(rng.pareto(0.7, n) + 1.0)      # exp-weights with infinite variance
    yield "cauchy_loglik", -np.log1p(rng.standard_cauchy(n) ** 2) * 40.0
    dom = np.full(n, -15.0)
    dom[rng.integers(n)] = 0.0
    yield "dominant_m15", dom                                          # ESS 41 % low before
    dom40 = np.full(n, -40.0)
    dom40[rng.integers(n)] = 0.0
    dom40[rng.integers(n)] = -1.0
    yield "dominant_m40", dom40                                        # the rest below 2^-K: q = 0
    neg = -0.5 * z * z
    neg[rng.permutation(n)[: n // 7]] = -np.inf
    yield "neg_inf", neg
    yield "wide", rng.uniform(-700.0, 0.0, n) + 3.0
    yield "all_equal", np.full(n, -3.25)
    yield "near_threshold_lo", near_threshold(n, 0.5 - 1e-6, rng)
    yield "near_threshold_hi", near_threshold(n, 0.5 + 1e-6, rng)


def _mark_changed(ctx):
    """A zero log-density Weight (Uniform(0,1) at 0.5: log 1 = 0) — sets weights_changed the
    way a model would, leaving every weight bit unchanged."""
    ctx.weight(Uniform(0.0, 1.0).dist(resolver(ctx)), [wsmc.abi.Operand.const(0.5)] * 4)


def run_case(backend, lw, ess_min, scheme, seed=20240607):
    n = len(lw)
    ctx = make_ctx(backend, n, seed=seed)
    cid = ctx.col_create("id", 1)
    ctx.col_upload(cid, np.arange(n, dtype=np.float64))
    ctx.weights_upload(lw)
    _mark_changed(ctx)
    assert np.array_equal(ctx.weights_download(), lw)
    op = ctx.get_state()["op_counter"]
    ev = ctx.log_evidence()
    rs, ess = ctx.resample(ess_min, scheme)
    ref = RefResample(lw, ess_min, seed, op, scheme)
    out = dict(ess=ess, rs=rs, ev=ev, w=ctx.weights_download(), id=ctx.col_download(cid),
               anc=ctx.last_ancestors() if rs else None)
    ctx.close()
    return out, ref


def check_against_reference(name, lw, out, ref, ess_min):
    n = len(lw)
    # ESS% to 1e-12 relative
    assert abs(out["ess"] - ref.ess) <= 1e-12 * ref.ess, (name, out["ess"], ref.ess)
    # log-mean / evidence (logsumexp(w) - log N) to 1e-12
    assert abs(out["ev"] - ref.mean) <= 1e-12 * max(1.0, abs(ref.mean)), (name, out["ev"], ref.mean)
    if name == "all_equal":
        # exact sums give ESS% = 1 and `1 < ess_min` decides; the reference's
        # f64 value is 1 within rounding (numpy: 1 - O(1e-16))
        assert out["ess"] == 1.0
        assert abs(ref.ess - 1.0) < 1e-14
        assert out["rs"] == (1.0 < ess_min)
        return 0
    assert out["rs"] == ref.resampled, (name, out["ess"], ref.ess)
    if not out["rs"]:
        np.testing.assert_array_equal(out["w"], lw)
        return 0
    # weights reset to the log-mean
    assert np.all(np.abs(out["w"] - ref.mean) <= 1e-12 * max(1.0, abs(ref.mean)))
    anc = out["anc"].astype(np.int64)
    np.testing.assert_array_equal(out["id"], anc.astype(np.float64))     # the store gathered through them
    assert np.all(np.diff(anc) >= 0)                                     # monotone, as icdf's merge
    ra = np.minimum(ref.anc, n - 1)                                      # clamp the BoundsError overrun
    bad = np.nonzero(anc != ra)[0]
    # every disagreement is a tie: the slot's uniform within the integer CDF's resolution of
    # the CDF boundary between the two answers
    qtot = ref.w.sum() * 2.0 ** wsmc_qbits(n)
    tol = 2.0 * (n + 1) / qtot + 64 * n * np.finfo(float).eps
    for s in bad:
        lo = min(anc[s], ra[s])
        gap = abs(ref.cdf[lo] - ref.us[s])
        assert gap <= tol, (name, int(s), int(anc[s]), int(ra[s]), gap, tol)
    assert len(bad) <= max(2, n // 100), (name, len(bad))
    return len(bad)


def wsmc_qbits(n):
    return min(43, 63 if n <= 1 else 63 - (n - 1).bit_length())


def test_strat_word_restatement_matches_oracle():
    from oracle import lib
    L = lib()
    for seed, op, n in [(0, 0, 0), (42, 7, 12345), (2 ** 63 + 5, 2 ** 40 + 3, 999999), (1, 1, 2 ** 31 - 1)]:
        assert strat_word(seed, op, n) == L.or_strat_word(seed, op, n)
        assert strat_words(seed, op, 2, start=n)[0] == float(strat_word(seed, op, n))


def test_ref_icdf_is_the_sequential_merge():
    rng = np.random.default_rng(3)
    for n in (1, 2, 17, 1000):
        w = ref_exp_norm(rng.standard_normal(n) * 3)
        us = ref_stratified_us(n, rng.random(n))
        anc, _ = ref_icdf(w, us)
        # literal loop of src/resampling.jl:13-26 (0-based)
        s, m, lit = w[0], 0, []
        for u in us:
            while s < u and m + 1 < n:
                m += 1
                s += w[m]
            lit.append(m)
        np.testing.assert_array_equal(np.minimum(anc, n - 1), lit)


CASE_SIZES = [(1000, 11), (65536 + 17, 5), (300001, 9)]


@pytest.mark.parametrize("scheme", [wsmc.RESAMPLE_STRATIFIED, wsmc.RESAMPLE_SYSTEMATIC])
@pytest.mark.parametrize("n,rseed", CASE_SIZES)
def test_oracle_resample_matches_reference_f64(n, rseed, scheme):
    ties = {}
    rng = np.random.default_rng(rseed)
    for name, lw in weight_cases(n, rng):
        for ess_min in ((0.5,) if name.startswith("near") else (0.5, 1.0, 2.0)):
            out, ref = run_case("oracle", lw, ess_min, scheme)
            ties[(name, ess_min)] = check_against_reference(name, lw, out, ref, ess_min)
    print(f"N={n} scheme={scheme}: CDF-boundary ties {sum(ties.values())} "
          f"over {sum(1 for _ in ties)} resamples: {ties}")


@pytest.mark.gpu
@pytest.mark.parametrize("scheme", [wsmc.RESAMPLE_STRATIFIED, wsmc.RESAMPLE_SYSTEMATIC])
@pytest.mark.parametrize("n,rseed", CASE_SIZES + [(1_000_000, 13)])
def test_hip_resample_matches_reference_f64(n, rseed, scheme, gpu_available):
    rng = np.random.default_rng(rseed)
    for name, lw in weight_cases(n, rng):
        for ess_min in ((0.5,) if name.startswith("near") else (0.5, 1.0, 2.0)):
            out, ref = run_case("hip", lw, ess_min, scheme)
            check_against_reference(name, lw, out, ref, ess_min)
            if n <= 300001:
                o, _ = run_case("oracle", lw, ess_min, scheme)
                assert o["ess"] == out["ess"] and o["rs"] == out["rs"] and o["ev"] == out["ev"]
                if o["rs"]:
                    np.testing.assert_array_equal(o["anc"], out["anc"])


@pytest.mark.gpu
def test_hip_ess_matches_reference_f64(gpu_available):
    """wsmc_ess (describe's ESS field) on the same vectors, no state change."""
    rng = np.random.default_rng(21)
    for name, lw in weight_cases(200_003, rng):
        c = wsmc.Context(len(lw), seed=1)
        c.weights_upload(lw)
        e = c.ess()
        ref = ref_ess_perc(ref_exp_norm(lw))
        if name == "all_equal":
            assert e == 1.0
        else:
            assert abs(e - ref) <= 1e-12 * ref, (name, e, ref)
        c.close()
