"""General Assign expressions on the GPU (wsmc_assign_expr, k_assign_expr) against the oracle's
program machine, bit for bit: every operator, vector outputs reading their own components,
columns read one lazy Resample behind (gather-on-read, the output rewritten through a fresh
buffer when it is one of them), a nonlinear state-space filter driven through the statements,
the multi-device handle, and the host-side refusals through the C ABI."""
import numpy as np
import pytest

import wsmc
from oracle import Oracle
from wsmc import abi, dsl, models
from wsmc.dsl import (Col, Normal, and_, cos, eq, exp, ifelse, log, log1p, max_, min_, not_, or_, sin, sqrt)

pytestmark = pytest.mark.gpu

EXPRS = {
    "exp": lambda: exp(Col("a")),
    "log": lambda: log(Col("b")),
    "log1p": lambda: log1p(Col("b")),
    "sqrt": lambda: sqrt(Col("b")) + sqrt(Col("a")),
    "sincos": lambda: sin(Col("d")) * cos(Col("d") * 3.0 + Col("a")),
    "product": lambda: Col("a") * Col("b") / Col("d") - Col("a"),
    "powi": lambda: Col("a") ** 2 + Col("b") ** -2 + Col("a") ** 3 + Col("b") ** 7 - Col("b") ** -5,
    "pow": lambda: Col("b") ** (Col("a") * 0.5) + Col("a") ** Col("c"),
    "minmax": lambda: min_(Col("a"), Col("d")) + max_(Col("a"), -0.0),
    "compare": lambda: (Col("a") < Col("d")) + 2.0 * (Col("a") >= 0.5) + 4.0 * eq(Col("c"), 1.0),
    "logic": lambda: ifelse(or_(Col("c"), Col("a") > 1.0), 0.98, 0.01) + and_(Col("c"), not_(Col("a") < 0.0)),
    "oscillator": lambda: Col("b") * exp(-0.1 * Col("b") * 3.0) * cos(Col("a") * 3.0 + Col("d")),
    "abs_neg": lambda: abs(Col("a")) - (-Col("d")),
    # |e| from 1e5 to 1e300: the Payne-Hanek reduction past 2^19 pi/2 (include/wsmc_math.h)
    "sincos_large": lambda: sin(Col("e")) - 2.0 * cos(Col("e")),
}


def fill(ctx, N, seed=3):
    rng = np.random.default_rng(seed)
    vals = {"a": rng.normal(0.0, 2.0, N), "b": rng.uniform(0.1, 3.0, N), "c": rng.integers(0, 2, N).astype(float),
            "d": rng.normal(0.0, 30.0, N),
            "e": np.exp(rng.uniform(np.log(1e5), np.log(1e300), N)) * rng.choice([-1.0, 1.0], N)}
    vals["a"][:4] = [-0.0, 0.0, np.nan, np.inf]
    for name, v in vals.items():
        ctx.col_upload(ctx.col_create(name), v)
    ctx.col_upload(ctx.col_create("v", 2), np.stack([rng.normal(size=N), rng.normal(size=N)]))


def assign(ctx, out, exprs):
    exprs = exprs if isinstance(exprs, list) else [exprs]
    c = ctx.col_find(out)
    if c < 0:
        c = ctx.col_create(out, len(exprs))
    prog, lens = dsl.xprogram(exprs, models.resolver(ctx))
    ctx.assign_expr(c, prog, lens)


def same_bits(g, o, name):
    """bit for bit; a NaN matches any NaN (an invalid operation's default NaN is negative on
    x86 and positive on the GPU)"""
    a = g.col_download(g.col_find(name))
    b = o.col_download(o.col_find(name))
    ok = (a.view(np.uint64) == b.view(np.uint64)) | (np.isnan(a) & np.isnan(b))
    assert ok.all(), (name, np.flatnonzero(~ok.ravel())[:8], a.ravel()[~ok.ravel()][:4], b.ravel()[~ok.ravel()][:4])


@pytest.mark.parametrize("N", [4096, 1001])
def test_every_operator_matches_the_oracle(gpu_available, N):
    g, o = wsmc.Context(N, seed=5), Oracle(N, seed=5)
    for ctx in (g, o):
        fill(ctx, N)
        for name, e in EXPRS.items():
            assign(ctx, "out_" + name, e())
        assign(ctx, "v", [Col("v", 1) * 2.0, Col("v", 0)])   # reads its own components
    for name in EXPRS:
        same_bits(g, o, "out_" + name)
    same_bits(g, o, "v")
    assert g.get_state()["depth"] == o.get_state()["depth"] == len(EXPRS) + 1


def sv_filter(ctx, ys, ess, wait):
    """a nonlinear state-space model through the statements: the transition and the
    observation scale are general expressions (Assign), the kernels read them as columns
        x ~ Normal(0, 1); z .= 0
        for t: m .= 0.9 x + 0.5 sin(x);  x ~ Normal(m, 0.3);  s .= exp(0.5 x);
               z .= 0.5 z + x^2 (z read through the ancestors: rewritten to a fresh buffer);
               y_t => Normal(0, s);  Resample"""
    R = models.resolver(ctx)
    cx = ctx.col_create("x")
    ctx.sample(cx, Normal(0.0, 1.0).dist(R))
    ctx.col_create("m")
    ctx.col_create("s")
    assign(ctx, "z", 0.0 * Col("x"))
    for y in ys:
        assign(ctx, "m", 0.9 * Col("x") + 0.5 * sin(Col("x")))
        ctx.sample(cx, Normal(Col("m"), 0.3).dist(R))
        assign(ctx, "s", exp(0.5 * Col("x")))
        assign(ctx, "z", 0.5 * Col("z") + Col("x") ** 2)
        ctx.observe(Normal(0.0, Col("s")).dist(R), models._const([y]))
        ctx.resample(ess, abi.RESAMPLE_STRATIFIED, wait=wait)


@pytest.mark.parametrize("lazy", [True, False])
@pytest.mark.parametrize("ess", [1.0, 0.5])
def test_nonlinear_filter_through_expressions(gpu_available, lazy, ess):
    N = 4096
    ys = np.random.default_rng(8).normal(0.0, 1.5, 12)
    g, o = wsmc.Context(N, seed=21), Oracle(N, seed=21)
    g.store_set_lazy(lazy)
    sv_filter(g, ys, ess, wait=False)
    sv_filter(o, ys, ess, wait=True)
    g.store_materialize()
    for name in ("x", "m", "s", "z"):
        same_bits(g, o, name)
    np.testing.assert_array_equal(g.weights_download(), o.weights_download())
    sg, so = g.get_state(), o.get_state()
    for k in ("depth", "op_counter", "n_resamples", "n_terms"):
        assert sg[k] == so[k], k
    assert g.log_evidence() == o.log_evidence()


def test_expressions_on_the_multi_device_handle(gpu_available):
    N = 6000
    ys = np.random.default_rng(9).normal(0.0, 1.5, 6)
    g = wsmc.Context.multi(N, 2, seed=21, devices=[0, 0], transport=abi.TRANSPORT_HOST)
    o = Oracle(N, seed=21, shards=2)
    sv_filter(g, ys, 1.0, wait=True)
    sv_filter(o, ys, 1.0, wait=True)
    for name in ("x", "m", "s", "z"):
        same_bits(g, o, name)
    g.close()


def test_malformed_programs_are_refused(gpu_available):
    g = wsmc.Context(64, seed=1)
    fill(g, 64)
    out = g.col_create("out")

    def prog(ins):
        arr = (abi.XInst * len(ins))()
        for k, (op, col, comp, c) in enumerate(ins):
            arr[k].op, arr[k].col, arr[k].comp, arr[k].c = op, col, comp, c
        return arr

    for bad, lens in (([(abi.X_ADD, -1, 0, 0.0)], [1]),
                      ([(abi.X_COL, 99, 0, 0.0)], [1]),                  # unknown column
                      ([(abi.X_COL, g.col_find("a"), 1, 0.0)], [1]),      # component out of range
                      ([(abi.X_COL, 0, 0, 0.0), (abi.X_POWI, -1, 0, 1.5)], [2]),
                      ([(abi.X_CONST, -1, 0, 1.0)] * 97, [97])):
        with pytest.raises(wsmc.WSMCError) as e:
            g.assign_expr(out, prog(bad), lens)
        assert e.value.code == abi.WSMC_EARG
    assert g.get_state()["depth"] == 0   # nothing ran
