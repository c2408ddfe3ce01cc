"""The scalar families beyond the configs' (WSMC_FAM_BERNOULLI .. WSMC_FAM_GEOMETRIC; the
reference's default_kernels, src/default_kernels.jl:83-102) on the CPU oracle: logpdf against
scipy.stats at every support edge, and the draws' distribution against the CDF (a
Kolmogorov–Smirnov bound for the continuous families, frequencies for the discrete ones). The
HIP kernels are compared with the oracle bit for bit in tests/test_gpu_families.py.
Parity with Julia's draws is not claimed: the streams are Philox (include/wsmc_math.h)."""
import numpy as np
import pytest
from scipy import stats

import wsmc
from oracle import Oracle
from wsmc import abi, models
from wsmc.dsl import Col

# (kernel, scipy frozen distribution, test points)
CASES = {
    "bernoulli": (lambda: wsmc.Bernoulli(0.3), stats.bernoulli(0.3), [0.0, 1.0, 0.5, -1.0, 2.0]),
    "bernoulli_logit": (lambda: wsmc.BernoulliLogit(-0.7), stats.bernoulli(1 / (1 + np.exp(0.7))), [0.0, 1.0, 0.3]),
    "exponential": (lambda: wsmc.Exponential(2.5), stats.expon(scale=2.5), [0.0, 0.1, 3.0, 40.0, -1.0]),
    "lognormal": (lambda: wsmc.LogNormal(0.3, 0.8), stats.lognorm(s=0.8, scale=np.exp(0.3)), [1e-3, 0.5, 1.0, 7.0, 0.0, -2.0]),
    "laplace": (lambda: wsmc.Laplace(1.0, 0.5), stats.laplace(1.0, 0.5), [-3.0, 1.0, 1.2, 9.0]),
    "cauchy": (lambda: wsmc.Cauchy(-1.0, 2.0), stats.cauchy(-1.0, 2.0), [-1.0, 0.0, 30.0, -1e6]),
    "logistic": (lambda: wsmc.Logistic(0.5, 1.5), stats.logistic(0.5, 1.5), [-40.0, 0.5, 2.0, 100.0]),
    "gumbel": (lambda: wsmc.Gumbel(0.5, 2.0), stats.gumbel_r(0.5, 2.0), [-3.0, 0.5, 4.0, 30.0]),
    "rayleigh": (lambda: wsmc.Rayleigh(1.7), stats.rayleigh(scale=1.7), [0.0, 0.3, 1.7, 9.0, -1.0]),
    "geometric": (lambda: wsmc.Geometric(0.25), stats.geom(0.25, loc=-1), [0.0, 1.0, 7.0, 2.5, -1.0]),
}
DISCRETE = ("bernoulli", "bernoulli_logit", "geometric")


def observe_at(kernel, xs):
    o = Oracle(len(xs), seed=1)
    cx = o.col_create("x")
    o.col_upload(cx, np.asarray(xs, float))
    o.observe(kernel.dist(models.resolver(o)), Col("x").operand(models.resolver(o)))
    return o.weights_download()


@pytest.mark.parametrize("name", sorted(CASES))
def test_logpdf_matches_scipy(name):
    kern, ref, xs = CASES[name]
    got = observe_at(kern(), xs)
    want = ref.logpmf(xs) if name in DISCRETE else ref.logpdf(xs)
    finite = np.isfinite(want)
    assert np.array_equal(np.isfinite(got), finite), (got, want)
    assert np.all(got[~finite] == -np.inf)
    np.testing.assert_allclose(got[finite], want[finite], rtol=5e-14, atol=1e-15)


@pytest.mark.parametrize("name", sorted(CASES))
def test_draws_follow_the_distribution(name):
    kern, ref, _ = CASES[name]
    N = 40_000
    o = Oracle(N, seed=7)
    cx = o.col_create("x")
    o.sample(cx, kern().dist(models.resolver(o)))
    x = o.col_download(cx)
    assert np.all(np.isfinite(x))
    if name in DISCRETE:
        ks = np.arange(0, 12)
        freq = np.array([(x == k).mean() for k in ks])
        np.testing.assert_allclose(freq, ref.pmf(ks), atol=4.5 * np.sqrt(0.25 / N))
        assert np.all(x == np.floor(x)) and np.all(x >= 0)
    else:
        d, p = stats.kstest(x, ref.cdf)
        assert p > 1e-4, (d, p)


def test_columns_as_parameters_and_unknown_families_are_refused_on_host():
    """p from a column (examples/fire_alarm.jl: Bernoulli(fire ? 0.9 : 0.01)); a family
    number beyond the table is refused (checked by the C ABI on the device path)"""
    N = 20_000
    o = Oracle(N, seed=3)
    R = models.resolver(o)
    cf = o.col_create("fire")
    o.sample(cf, wsmc.Bernoulli(0.5).dist(R))
    cp = o.col_create("p")
    prog, lens = wsmc.dsl.xprogram([wsmc.dsl.ifelse(Col("fire"), 0.9, 0.01)], R)
    o.assign_expr(cp, prog, lens)
    cs = o.col_create("smoke")
    o.sample(cs, wsmc.Bernoulli(Col("p")).dist(R))
    f, s = o.col_download(cf), o.col_download(cs)
    assert abs(s[f == 1].mean() - 0.9) < 0.02 and abs(s[f == 0].mean() - 0.01) < 0.01
    assert abi.FAM_GEOMETRIC == 14


def _dec_logpdf_normal(mu, sigma, x):
    """-(z^2 + log 2pi)/2 - log sigma in 60-digit decimal (the textbook formula the reference's
    normlogpdf evaluates)"""
    from decimal import Decimal, getcontext
    getcontext().prec = 60
    pi = Decimal("3.14159265358979323846264338327950288419716939937510582097494459")
    z = (Decimal(x) - Decimal(mu)) / Decimal(sigma)
    return -(z * z + (2 * pi).ln()) / 2 - Decimal(sigma).ln()


@pytest.mark.parametrize("family", ["normal", "halfnormal", "lognormal"])
def test_normal_family_logpdf_against_decimal(family):
    """the Normal log-density is evaluated as fma(-h, h, c) (include/wsmc_math.h
    wsmc_normal_lh) and the goldens were regenerated from the oracle, so nothing pinned it to
    the textbook -(z^2 + log 2pi)/2 - log sigma. Here: Normal, HalfNormal (+ log 2) and LogNormal
    (log-space Normal - log x) against that formula in 60-digit decimal over z in [0, 40] and
    sigma over 1e-3 .. 1e3, including the cancellation z^2/2 ~ -log(sigma sqrt(2 pi)) where the
    density is near 1. The bound is 8 ulp of the terms' magnitudes (log 2pi / 2 + |log sigma| +
    z^2 / 2 + |log x|): the result's absolute error cannot be smaller than their rounding, and
    rh = (1/sigma)/sqrt(2) carries two roundings into h^2 (about 3 ulp of z^2 / 2 measured)."""
    from decimal import Decimal
    rng = np.random.default_rng(11)
    mus, sigmas, xs = [], [], []
    for s in np.exp(rng.uniform(np.log(1e-3), np.log(1e3), 60)):
        c = -0.5 * np.log(2 * np.pi) - np.log(s)
        zs = list(rng.uniform(0, 40, 6)) + ([np.sqrt(2 * c)] if c > 0 else [])   # the density near 1
        for z in zs:
            mus.append(0.0 if family == "halfnormal" else 0.7)
            sigmas.append(float(s))
            xs.append(float((0.0 if family == "halfnormal" else 0.7) + z * s))
    for mu, s, x in zip(mus, sigmas, xs):
        if family == "normal":
            kern, xv = wsmc.Normal(mu, s), x
            want = _dec_logpdf_normal(mu, s, x)
        elif family == "halfnormal":
            kern, xv = wsmc.HalfNormal(s), x
            want = _dec_logpdf_normal(0.0, s, x) + Decimal(2).ln()
        else:
            xv = float(np.exp(x))
            if not (0.0 < xv < np.inf):
                continue
            kern = wsmc.LogNormal(mu, s)
            want = _dec_logpdf_normal(mu, s, Decimal(xv).ln()) - Decimal(xv).ln()
        got = observe_at(kern, [xv])[0]
        z = (x - mu) / s
        # the intermediates' magnitudes (log 2pi / 2, log sigma, z^2 / 2, log x): any f64
        # evaluation of the formula rounds at their scale
        scale = 0.5 * np.log(2 * np.pi) + abs(np.log(s)) + 0.5 * z * z + (abs(np.log(xv)) if family == "lognormal" else 0)
        tol = 8 * np.spacing(max(scale, 1e-300))
        if family == "lognormal":   # log x itself is good to an ulp; (log x - mu)/sigma amplifies that
            tol += 2 * abs(z) * np.spacing(abs(np.log(xv))) / s
        assert abs(Decimal(got) - want) <= Decimal(tol), (family, mu, s, x, got, want)
