"""Independent numpy f64 restatements of the reference's per-particle math.

TEST INFRASTRUCTURE. Nothing here reads include/wsmc_math.h or include/wsmc_terms.h, calls
the oracle, or reuses the build's restated exp/log/sin/cos: every density, transform and
covariance is numpy/libm f64 written from the reference's own definitions (each function
cites the reference file:line it follows). The only thing shared with the build is the
definition of its random stream (the build cannot reproduce Julia's Xoshiro/ziggurat, see
DESIGN.md §2): Philox4x32-10 keyed by (seed, op counter, particle index, block) and
Box–Muller, restated here from that definition (Salmon et al. 2011 rounds and constants,
checked against the Random123 known-answer vectors) so that both sides draw the same
normals and uniforms. numpy's libm differs from the build's restated functions by a few
ulps, so comparisons carry a written tolerance (1e-12 relative unless stated).
"""
from __future__ import annotations

import math

import numpy as np

M32 = 0xFFFFFFFF

# ---------------------------------------------------------------------------------------
# the build's random stream, restated (DESIGN.md §2 "RNG")
# ---------------------------------------------------------------------------------------
_PH_M0 = np.uint64(0xD2511F53)
_PH_M1 = np.uint64(0xCD9E8D57)


def philox4x32_10(c0, c1, c2, c3, k0: int, k1: int):
    """Philox4x32-10 (Salmon, Moraes, Dror, Shaw, SC'11) on uint32 arrays; scalar key."""
    c0, c1, c2, c3 = (np.asarray(c, dtype=np.uint32).copy() for c in (c0, c1, c2, c3))
    k0 &= M32
    k1 &= M32
    for _ in range(10):
        p0 = c0.astype(np.uint64) * _PH_M0
        p1 = c2.astype(np.uint64) * _PH_M1
        hi0 = (p0 >> np.uint64(32)).astype(np.uint32)
        lo0 = (p0 & np.uint64(M32)).astype(np.uint32)
        hi1 = (p1 >> np.uint64(32)).astype(np.uint32)
        lo1 = (p1 & np.uint64(M32)).astype(np.uint32)
        c0, c1, c2, c3 = hi1 ^ c1 ^ np.uint32(k0), lo1, hi0 ^ c3 ^ np.uint32(k1), lo0
        k0 = (k0 + 0x9E3779B9) & M32
        k1 = (k1 + 0xBB67AE85) & M32
    return c0, c1, c2, c3


def rng_block(seed: int, op: int, idx, block: int):
    """Counter {idx lo32, idx hi32 ^ (block << 16), op lo32, op hi32}, key = seed."""
    idx = np.asarray(idx, dtype=np.uint64)
    c0 = (idx & np.uint64(M32)).astype(np.uint32)
    c1 = ((idx >> np.uint64(32)) ^ np.uint64((block << 16) & M32)).astype(np.uint32)
    n = idx.shape
    c2 = np.full(n, op & M32, dtype=np.uint32)
    c3 = np.full(n, (op >> 32) & M32, dtype=np.uint32)
    return philox4x32_10(c0, c1, c2, c3, seed & M32, (seed >> 32) & M32)


def _u53(hi, lo):
    return ((hi.astype(np.uint64) << np.uint64(32)) | lo.astype(np.uint64)) >> np.uint64(11)


def u01(hi, lo):
    """53-bit uniform in [0, 1)."""
    return _u53(hi, lo).astype(np.float64) * 2.0 ** -53


def u01_open0(hi, lo):
    """53-bit uniform in (0, 1]."""
    return (_u53(hi, lo) + np.uint64(1)).astype(np.float64) * 2.0 ** -53


def normal_pair(seed, op, idx, block):
    """Box–Muller on one Philox block: r cos(2 pi u2), r sin(2 pi u2), r = sqrt(-2 log u1)."""
    w0, w1, w2, w3 = rng_block(seed, op, idx, block)
    u1 = u01_open0(w0, w1)
    u2 = u01(w2, w3)
    r = np.sqrt(-2.0 * np.log(u1))
    return r * np.cos(2.0 * np.pi * u2), r * np.sin(2.0 * np.pi * u2)


def normal_k(seed, op, idx, k):
    """The k-th standard normal of (op, particle)."""
    z0, z1 = normal_pair(seed, op, idx, k >> 1)
    return z1 if k & 1 else z0


def uniform_k(seed, op, idx, k):
    """The k-th uniform in [0, 1) of (op, particle)."""
    w0, w1, w2, w3 = rng_block(seed, op, idx, (k >> 1) | 0x80)
    return u01(w2, w3) if k & 1 else u01(w0, w1)


# ---------------------------------------------------------------------------------------
# densities (Distributions.jl semantics, src/default_kernels.jl:12-23)
# ---------------------------------------------------------------------------------------
LOG2PI = math.log(2.0 * math.pi)


def normal_logpdf(x, mu, sigma):
    """logpdf(Normal(mu, sigma), x): sigma is a standard deviation (StatsFuns.normlogpdf)."""
    z = (np.asarray(x, float) - mu) / sigma
    return -0.5 * z * z - np.log(sigma) - 0.5 * LOG2PI


def halfnormal_logpdf(x, sigma):
    """Truncated(Normal(0, sigma), 0, Inf) (examples/damped_oscillator.jl:24-28): the Normal
    density renormalised by 1/2 on the support, -Inf outside it."""
    x = np.asarray(x, float)
    v = normal_logpdf(x, 0.0, sigma) + math.log(2.0)
    return np.where(x >= 0.0, v, -np.inf)


def uniform_logpdf(x, a, b):
    x = np.asarray(x, float)
    return np.where((x >= a) & (x <= b), -math.log(b - a), -np.inf)


def mvnormal_logpdf(x, mu, cov):
    """logpdf(MvNormal(mu, Σ), x) with Σ a COVARIANCE matrix (src/default_kernels.jl:12-23 with
    PDMats): -(d log 2π + log det Σ + (x-μ)ᵀ Σ⁻¹ (x-μ)) / 2, through a Cholesky factor — the
    general formula, not the isotropic shortcut the build evaluates. x, mu: [d][N]."""
    cov = np.asarray(cov, float)
    d = cov.shape[0]
    L = np.linalg.cholesky(cov)
    r = np.asarray(x, float) - np.asarray(mu, float)
    y = np.linalg.solve(L, r)
    return -0.5 * (d * LOG2PI + 2.0 * np.sum(np.log(np.diag(L))) + np.sum(y * y, axis=0))


def oscillator(t, A, om, ga, ph):
    """examples/damped_oscillator.jl:11: A exp(-γ t) cos(ω t + ϕ)."""
    return A * np.exp(-ga * t) * np.cos(om * t + ph)


# ---------------------------------------------------------------------------------------
# bound transforms (src/move_kernels.jl:37-85)
# ---------------------------------------------------------------------------------------
def to_unconstrained(x, lo, hi):
    if math.isfinite(lo) and math.isfinite(hi):
        return np.log(x - lo) - np.log(hi - x)
    if math.isfinite(lo):
        return np.log(x - lo)
    if math.isfinite(hi):
        return np.log(hi - x)
    return np.asarray(x, float)


def from_unconstrained(z, lo, hi):
    if math.isfinite(lo) and math.isfinite(hi):
        return lo + (hi - lo) / (1.0 + np.exp(-z))
    if math.isfinite(lo):
        return lo + np.exp(z)
    if math.isfinite(hi):
        return hi - np.exp(z)
    return np.asarray(z, float)


def log1pexp(z):
    """_log1pexp (src/move_kernels.jl:66)."""
    z = np.asarray(z, float)
    return np.where(z > 0, z + np.log1p(np.exp(-np.abs(z))), np.log1p(np.exp(np.minimum(z, 0.0))))


def log_abs_jacobian(z, lo, hi):
    if math.isfinite(lo) and math.isfinite(hi):
        return math.log(hi - lo) - log1pexp(z) - log1pexp(-z)
    if math.isfinite(lo) or math.isfinite(hi):
        return np.asarray(z, float)
    return np.zeros_like(np.asarray(z, float))


# ---------------------------------------------------------------------------------------
# exp_norm and autoRW's covariance (src/resampling.jl:72-77, src/move_kernels.jl:144-151)
# ---------------------------------------------------------------------------------------
def exp_norm(lw):
    lw = np.asarray(lw, float)
    w = np.exp(lw - np.max(lw))
    return w / np.sum(w)


def weighted_cov_uncorrected(Z, w):
    """StatsBase cov(Z, ProbabilityWeights(w)) with corrected=false: Σ w (z - z̄)(z - z̄)ᵀ / Σ w.
    Z: [d][N]."""
    Z = np.asarray(Z, float)
    sw = np.sum(w)
    mean = (Z @ w) / sw
    C = Z - mean[:, None]
    return (C * w) @ C.T / sw


def autorw_factor(Z, lw, min_step):
    """_adaptive_changes (src/move_kernels.jl:144-151): Σ = cov(Z, pw(exp_norm(w))),
    Σ[Σ .== 0] .= min_step, λ = 2.38 d^(-1/2), rand(MvNormal(λΣ)) = chol(λΣ).L · ξ.
    Returns (the covariance λΣ, its lower Cholesky factor)."""
    d = Z.shape[0]
    S = weighted_cov_uncorrected(Z, exp_norm(lw))
    S = np.where(S == 0.0, min_step, S)
    S = (2.38 * d ** -0.5) * S
    return S, np.linalg.cholesky(S)


def mh_accept(log_u, log_pratio, s_new, s_old):
    """src/transformers.jl:615: accept iff log(rand()) < log_pratio + s_new - s_old."""
    return log_u < (log_pratio + s_new) - s_old


def close(a, b, rtol=1e-12, floor=1.0):
    """|a - b| <= rtol · max(floor, |b|) elementwise (inf == inf, nan == nan)."""
    a = np.asarray(a, float)
    b = np.asarray(b, float)
    same = (a == b) | (np.isnan(a) & np.isnan(b))
    with np.errstate(invalid="ignore"):
        ok = np.abs(a - b) <= rtol * np.maximum(floor, np.abs(b))
    return same | ok
