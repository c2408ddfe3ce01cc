"""The scalar families beyond the configs' on the GPU against the oracle, bit for bit: draws
and log-densities through single statements and compiled statement batches, parameters read
from columns (examples/fire_alarm.jl run whole, with its `cond ? a : b` arguments as Assign
expressions), and a Move whose score fold holds the new families' terms (a robust regression:
Laplace prior, Cauchy observations, autoRW)."""
import numpy as np
import pytest

import wsmc
from oracle import Oracle
from wsmc import abi, dsl, models
from wsmc.dsl import Col, ifelse, or_

pytestmark = pytest.mark.gpu

KERNELS = {
    "bernoulli": lambda: wsmc.Bernoulli(0.3),
    "bernoulli_logit": lambda: wsmc.BernoulliLogit(-0.7),
    "exponential": lambda: wsmc.Exponential(2.5),
    "lognormal": lambda: wsmc.LogNormal(0.3, 0.8),
    "laplace": lambda: wsmc.Laplace(1.0, 0.5),
    "cauchy": lambda: wsmc.Cauchy(-1.0, 2.0),
    "logistic": lambda: wsmc.Logistic(0.5, 1.5),
    "gumbel": lambda: wsmc.Gumbel(0.5, 2.0),
    "rayleigh": lambda: wsmc.Rayleigh(1.7),
    "geometric": lambda: wsmc.Geometric(0.25),
}


def same(g, o, names):
    for n in names:
        a = g.col_download(g.col_find(n))
        b = o.col_download(o.col_find(n))
        np.testing.assert_array_equal(a.view(np.uint64), b.view(np.uint64), err_msg=n)
    np.testing.assert_array_equal(g.weights_download(), o.weights_download())


def draw_and_score(ctx, kern):
    """x ~ D; y ~ D (one batch: Sample, Sample, Observe, Observe); the weights are
    logpdf(D, x) + logpdf(D, y + 0.25)"""
    R = models.resolver(ctx)
    d = kern.dist(R)
    cx, cy = ctx.col_create("x"), ctx.col_create("y")
    ctx.sample(cx, d)
    ctx.sample(cy, d)
    ctx.observe(d, Col("x").operand(R))
    ctx.observe(d, (Col("y") + 0.25).operand(R))


@pytest.mark.parametrize("name", sorted(KERNELS))
@pytest.mark.parametrize("N", [4096, 1001])
def test_family_draws_and_logpdf_match_the_oracle(gpu_available, name, N):
    g, o = wsmc.Context(N, seed=31), Oracle(N, seed=31)
    for ctx in (g, o):
        draw_and_score(ctx, KERNELS[name]())
    same(g, o, ["x", "y"])


def fire_alarm(ctx, observe_alarm):
    """examples/fire_alarm.jl:9-14 (and :27-32 with `true => Bernoulli(...)`)"""
    R = models.resolver(ctx)

    def expr(out, e):
        c = ctx.col_find(out)
        c = c if c >= 0 else ctx.col_create(out)
        prog, lens = dsl.xprogram([e], R)
        ctx.assign_expr(c, prog, lens)

    for n in ("fire", "smoke", "lever"):
        ctx.col_create(n)
    ctx.sample(ctx.col_find("fire"), wsmc.Bernoulli(0.01).dist(R))
    expr("p_smoke", ifelse(Col("fire"), 0.9, 0.01))
    ctx.sample(ctx.col_find("smoke"), wsmc.Bernoulli(Col("p_smoke")).dist(R))
    expr("p_lever", ifelse(Col("fire"), 0.7, 0.01))
    ctx.sample(ctx.col_find("lever"), wsmc.Bernoulli(Col("p_lever")).dist(R))
    expr("p_alarm", ifelse(or_(Col("smoke"), Col("lever")), 0.98, 0.01))
    if observe_alarm:
        ctx.observe(wsmc.Bernoulli(Col("p_alarm")).dist(R), models._const([1.0]))
    else:
        ctx.col_create("alarm")
        ctx.sample(ctx.col_find("alarm"), wsmc.Bernoulli(Col("p_alarm")).dist(R))
    ctx.resample(0.5)


@pytest.mark.parametrize("observe_alarm", [False, True])
def test_fire_alarm_matches_the_oracle(gpu_available, observe_alarm):
    N = 100_000
    g, o = wsmc.Context(N, seed=42), Oracle(N, seed=42)
    fire_alarm(g, observe_alarm)
    fire_alarm(o, observe_alarm)
    g.store_materialize()
    names = ["fire", "smoke", "lever", "p_smoke", "p_lever", "p_alarm"] + ([] if observe_alarm else ["alarm"])
    same(g, o, names)
    if observe_alarm:   # P(fire | alarm) is about 0.3 for this network
        f = g.col_download(g.col_find("fire"))
        assert 0.2 < f.mean() < 0.45


def robust_regression(ctx, xs, ys):
    """θ ~ Laplace(0, 1); β ~ Normal(0, 3); y_k => Cauchy(θ + β x_k, 0.5); Resample;
    θ << autoRW(); β << autoRW() — the Moves fold the Laplace / Cauchy terms (generic fold)"""
    R = models.resolver(ctx)
    ct, cb = ctx.col_create("θ"), ctx.col_create("β")
    ctx.sample(ct, wsmc.Laplace(0.0, 1.0).dist(R))
    ctx.sample(cb, wsmc.Normal(0.0, 3.0).dist(R))
    acc = []
    for x, y in zip(xs, ys):
        ctx.observe(wsmc.Cauchy(Col("θ") + Col("β") * float(x), 0.5).dist(R), models._const([y]))
        rs, _ = ctx.resample(1.0)
        if rs:
            acc.append((ctx.move(abi.PROPOSAL_AUTORW, [ct], 1e-3), ctx.move(abi.PROPOSAL_AUTORW, [cb], 1e-3)))
    return acc


def test_moves_over_the_new_families_match_the_oracle(gpu_available):
    N = 8192
    rng = np.random.default_rng(4)
    xs = rng.uniform(-2, 2, 6)
    ys = 0.7 + 1.3 * xs + rng.standard_cauchy(6) * 0.3
    g, o = wsmc.Context(N, seed=9), Oracle(N, seed=9)
    assert robust_regression(g, xs, ys) == robust_regression(o, xs, ys)
    g.store_materialize()
    same(g, o, ["θ", "β"])


def test_family_argument_checks(gpu_available):
    g = wsmc.Context(64, seed=1)
    c = g.col_create("x")
    d = wsmc.Exponential(1.0).dist(models.resolver(g))
    d.family = 15
    with pytest.raises(wsmc.WSMCError):
        g.sample(c, d)
    d = wsmc.Exponential(1.0).dist(models.resolver(g))
    d.dim = 2
    with pytest.raises(wsmc.WSMCError):
        g.sample(c, d)
