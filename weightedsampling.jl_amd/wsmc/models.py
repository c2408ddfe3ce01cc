"""The reference's example models as statement sequences over the context protocol.

Each function issues exactly the statements the reference's ``@model`` expansion
executes (including the auto-inserted ``Resample()`` after every ``~``/``=>``,
src/rewrites.jl:707-711), in the same order, against any object implementing the
context protocol (``wsmc.Context`` on the GPU). Column creation order, depth,
score-tape and RNG stream positions therefore match the fused runners.

    ssm1d_statements       examples/1D_ssm.jl:7-16
    lgssm1d_statements     benchmarks/ssm/WeightedSampling/lgssm1d.jl:18-24 (the reference's own CPU benchmark)
    ssm2d_statements       examples/2D_ssm.jl:7-17
    linreg_statements      examples/linear_regression.jl:17-27
    oscillator_statements  examples/damped_oscillator.jl:30-43
"""
from __future__ import annotations

import math

import numpy as np

from . import abi
from .abi import Operand
from .dsl import Col, HalfNormal, MvNormal, Normal, Oscillator, Uniform, value_operands


def resolver(ctx):
    def r(name: str) -> int:
        c = ctx.col_find(name)
        if c < 0:
            raise KeyError(f"unknown column {name!r}")
        return c
    return r


def _const(vals):
    return [Operand.const(float(v)) for v in vals]


# ---------------------------------------------------------------------------------------
def ssm2d_statements(ctx, obs, x0=(0.0, 0.0), v0=(1.0, 0.0), q_var=0.1, r_var=0.5,
                     ess_perc_min=0.5, scheme=abi.RESAMPLE_STRATIFIED, wait=True):
    """examples/2D_ssm.jl:7-17 (Σ's are covariances: 0.1·I₂ and 0.5·I₂), one C-ABI call per
    statement. The model has no `if resampled`: with wait=False no Resample returns its flag
    (the decisions stay on the device) and the function returns None."""
    R = resolver(ctx)
    obs = np.asarray(obs, dtype=float).reshape(-1, 2)
    cx1 = ctx.col_create("x_1", 2)
    ctx.assign(cx1, _const(x0))                       # x{1} .= [0.0, 0.0]
    cv = ctx.col_create("v", 2)
    ctx.assign(cv, _const(v0))                        # v .= [1.0, 0.0]
    I2 = np.eye(2)
    resampled = []
    cdv, v_next = -1, None
    dv_dist = MvNormal([0.0, 0.0], q_var * I2).dist(R)                      # the loop's kernels, built once
    for t, o in enumerate(obs, start=1):
        xt, xn = f"x_{t}", f"x_{t + 1}"
        cxn = ctx.col_create(xn, 2)
        if t == 1:   # @model's column order: x_1, v, x_2, dv, x_3, ...
            cdv = ctx.col_create("dv", 2)
            v_next = value_operands(Col("v") + Col("dv"), 2, R)
        ctx.assign(cxn, value_operands(Col(xt) + Col("v"), 2, R))            # x{t+1} .= x{t} + v
        ctx.sample(cdv, dv_dist)                                            # dv ~ MvNormal(0, 0.1 I)
        ctx.resample(ess_perc_min, scheme, wait=wait)                       # auto-inserted (no-op)
        ctx.assign(cv, v_next)                                              # v .= v + dv
        ctx.observe(MvNormal(Col(xn), r_var * I2).dist(R), _const(o))       # o => MvNormal(x{t+1}, 0.5 I)
        rs = ctx.resample(ess_perc_min, scheme, wait=wait)
        if wait:
            resampled.append(rs[0])
    return resampled if wait else None


def ssm1d_statements(ctx, obs, q_sd=0.1, r_sd=1.0, ess_perc_min=0.5, scheme=abi.RESAMPLE_STRATIFIED):
    """examples/1D_ssm.jl:7-16 (Normal's σ is a standard deviation)."""
    R = resolver(ctx)
    cx1 = ctx.col_create("x_1", 1)
    ctx.assign(cx1, _const([0.0]))
    cv = ctx.col_create("v", 1)
    ctx.assign(cv, _const([0.0]))
    resampled = []
    for t, o in enumerate(np.asarray(obs, dtype=float), start=1):
        xt, xn = f"x_{t}", f"x_{t + 1}"
        cxn = ctx.col_create(xn, 1)
        ctx.assign(cxn, value_operands(Col(xt) + Col("v"), 1, R))
        cdv = ctx.col_create("dv", 1)
        ctx.sample(cdv, Normal(0.0, q_sd).dist(R))
        ctx.resample(ess_perc_min, scheme)
        ctx.assign(cv, value_operands(Col("v") + Col("dv"), 1, R))
        ctx.observe(Normal(Col(xn), r_sd).dist(R), _const([o]))
        rs, _ = ctx.resample(ess_perc_min, scheme)
        resampled.append(rs)
    return resampled


def lgssm1d_statements(ctx, data, a=0.9, q=1.0, r=0.5, x0_std=1.0, ess_perc_min=1.0,
                       scheme=abi.RESAMPLE_STRATIFIED, wait=True):
    """The reference's own CPU benchmark model, benchmarks/ssm/WeightedSampling/lgssm1d.jl:18-24:
    x ~ Normal(0, x0_std); for y in data: x ~ Normal(a x, q); y => Normal(x, r); end.
    `x` is rebound, so the store keeps one column (no history), and every `~`/`=>` is
    followed by its auto-inserted Resample (a no-op after a Sample). The model has no `if
    resampled`, so with wait=False no Resample returns its flag to the host (the decisions
    stay on the device) and the function returns None."""
    R = resolver(ctx)
    cx = ctx.col_create("x", 1)
    ctx.sample(cx, Normal(0.0, x0_std).dist(R))
    ctx.resample(ess_perc_min, scheme, wait=wait)
    resampled = []
    transition = Normal(Col("x") * a, q).dist(R)       # the loop body's kernels (built once)
    likelihood = Normal(Col("x"), r).dist(R)
    for y in np.asarray(data, dtype=float):
        ctx.sample(cx, transition)                                          # x ~ Normal(a*x, q)
        ctx.resample(ess_perc_min, scheme, wait=wait)
        ctx.observe(likelihood, _const([y]))                                # y => Normal(x, r)
        rs = ctx.resample(ess_perc_min, scheme, wait=wait)
        if wait:
            resampled.append(rs[0])
    return resampled if wait else None


def linreg_statements(ctx, xs, ys, prior_sd=10.0, obs_sd=1.0, ess_perc_min=0.5,
                      scheme=abi.RESAMPLE_STRATIFIED, min_step=1e-3, wait_moves=True, gated=False,
                      block=True):
    """examples/linear_regression.jl:17-27: α, β ~ N(0,10); y => N(α + β x, 1);
    `if resampled; α << autoRW(); β << autoRW(); end`. gated=True lowers the `if resampled`
    block to device-gated Moves: no Resample returns its flag, nothing waits on the host inside
    the loop, and the function returns None. block=True issues the two Moves as one statement
    block (wsmc_move_block: one moments pass, one Move kernel), else as two wsmc_move_gated."""
    R = resolver(ctx)
    ca = ctx.col_create("α", 1)
    ctx.sample(ca, Normal(0.0, prior_sd).dist(R))
    ctx.resample(ess_perc_min, scheme)
    cb = ctx.col_create("β", 1)
    ctx.sample(cb, Normal(0.0, prior_sd).dist(R))
    ctx.resample(ess_perc_min, scheme)
    accepted = []
    for x, y in zip(xs, ys):
        ctx.observe(Normal(Col("α") + Col("β") * float(x), obs_sd).dist(R), _const([y]))
        if gated:
            ctx.resample(ess_perc_min, scheme, wait=False)
            if block:
                ctx.move_block([(abi.PROPOSAL_AUTORW, [ca], min_step), (abi.PROPOSAL_AUTORW, [cb], min_step)],
                               gated=True)
            else:
                ctx.move_gated(abi.PROPOSAL_AUTORW, [ca], min_step)
                ctx.move_gated(abi.PROPOSAL_AUTORW, [cb], min_step)
            continue
        rs, _ = ctx.resample(ess_perc_min, scheme)
        if rs:   # `if resampled` reads the flag; the moves need not return their counts
            a1 = ctx.move(abi.PROPOSAL_AUTORW, [ca], min_step, wait=wait_moves)
            a2 = ctx.move(abi.PROPOSAL_AUTORW, [cb], min_step, wait=wait_moves)
            accepted.append((a1, a2))
    return None if gated else accepted


def oscillator_statements(ctx, t_obs, y_obs, ess_perc_min=0.5, scheme=abi.RESAMPLE_STRATIFIED,
                          sweeps=1, diversity=0.9, min_step=1e-3, wait_moves=True, block=False):
    """examples/damped_oscillator.jl:30-43 with `sweeps` repetitions of the two moves. The model
    has no `if resampled`: no Resample returns its flag (the decisions stay on the device).
    Without a diversity gate each sweep's two Moves go as one statement block
    (wsmc_move_block) when block=True (off by default: for C5's 5-target sweep the block
    measured slower than the two Moves, 0.345 against 0.295 s a run)."""
    R = resolver(ctx)
    names = ["A", "ω", "γ", "ϕ", "σ"]
    priors = [HalfNormal(5.0), HalfNormal(5.0), HalfNormal(1.0), Uniform(-math.pi, math.pi), HalfNormal(1.0)]
    cols = {}
    for n, k in zip(names, priors):
        cols[n] = ctx.col_create(n, 1)
        ctx.sample(cols[n], k.dist(R))
        ctx.resample(ess_perc_min, scheme, wait=False)
    joint = [cols["A"], cols["ω"], cols["γ"], cols["σ"]]
    div = math.nan if diversity is None else float(diversity)
    accepted = []
    for t, y in zip(t_obs, y_obs):
        mean = Oscillator(float(t), Col("A"), Col("ω"), Col("γ"), Col("ϕ"))
        ctx.observe(Normal(mean, Col("σ")).dist(R), _const([y]))
        ctx.resample(ess_perc_min, scheme, wait=False)
        for _ in range(sweeps):
            if block and diversity is None:
                acc = ctx.move_block([(abi.PROPOSAL_AUTORW, joint, min_step, [0.0] * 4, [math.inf] * 4),
                                      (abi.PROPOSAL_AUTORW, [cols["ϕ"]], min_step, [-math.pi], [math.pi])],
                                     wait=wait_moves)
                accepted.append(tuple(acc) if wait_moves else (None, None))
                continue
            a1 = ctx.move(abi.PROPOSAL_AUTORW, joint, min_step, lo=[0.0] * 4, hi=[math.inf] * 4,
                          diversity=div, wait=wait_moves)
            a2 = ctx.move(abi.PROPOSAL_AUTORW, [cols["ϕ"]], min_step, lo=[-math.pi], hi=[math.pi],
                          diversity=div, wait=wait_moves)
            accepted.append((a1, a2))
    return accepted


# ---- data generators (the examples' recurrences, on numpy's Philox stream) -------------
def ssm2d_data(T: int, seed: int = 42):
    """examples/2D_ssm.jl:19-28: o_t = x_t + 0.5 z; x_{t+1} = x_t + v_t; v_{t+1} = v_t + 0.1 z."""
    rng = np.random.Generator(np.random.Philox(seed))
    x, v = np.zeros(2), np.array([1.0, 0.0])
    obs = np.empty((T, 2))
    for t in range(T):
        obs[t] = x + 0.5 * rng.standard_normal(2)
        x, v = x + v, v + 0.1 * rng.standard_normal(2)
    return obs


def ssm1d_data(T: int, seed: int = 7):
    """examples/1D_ssm.jl:18-27."""
    rng = np.random.Generator(np.random.Philox(seed))
    x, v = 0.0, 0.0
    obs = np.empty(T)
    for t in range(T):
        obs[t] = x + 1.0 * rng.standard_normal()
        x, v = x + v, v + 0.1 * rng.standard_normal()
    return obs


def lgssm1d_data(T: int, a=0.9, q=1.0, r=0.5, x0_std=1.0, seed: int = 42):
    """benchmarks/ssm/simulate.jl:21-31 (simulate_lgssm1d) on numpy's Philox stream."""
    rng = np.random.Generator(np.random.Philox(seed))
    x = x0_std * rng.standard_normal()
    obs = np.empty(T)
    for t in range(T):
        x = a * x + q * rng.standard_normal()
        obs[t] = x + r * rng.standard_normal()
    return obs


def linreg_data(seed: int = 42):
    """examples/linear_regression.jl:31-33: xs = 1:10, ys = 1 - 0.5 xs + 0.5 z."""
    rng = np.random.Generator(np.random.Philox(seed))
    xs = np.arange(1, 11, dtype=float)
    ys = 1.0 - 0.5 * xs + 0.5 * rng.standard_normal(10)
    return xs, ys


def oscillator_data(seed: int = 42, n: int = 60):
    """examples/damped_oscillator.jl:13-22."""
    rng = np.random.Generator(np.random.Philox(seed))
    t = np.linspace(0.0, 8.0, n)
    y = 3.0 * np.exp(-0.3 * t) * np.cos(2.5 * t + 0.5) + 1.0 * rng.standard_normal(n)
    return t, y
