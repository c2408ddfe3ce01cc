"""Host-side mirror of WeightedSampling.jl's ParticleTransformer / SMCState API.

Same names, argument meaning and error behaviour as the reference
(src/transformers.jl, src/types.jl, src/stores.jl, src/move_kernels.jl), with every
per-particle operation executed by the HIP library through the context protocol:

    reference (Julia)                      here
    SMCState(N; ess_perc_min)              SMCState(N, ess_perc_min=...)
    state[:x] / getcol(store, :x)          state["x"] / state.store.getcol("x")
    apply!(t, state) / run!(root, state)   apply(t, state) / run(root, state)
    Assign(:x, argfn)                      Assign("x", Col("y") + 1.0), Assign("p", ifelse(Col("f"), .9, .01))
    Sample(:x, kernel, argfn)              Sample("x", Normal(Col("x") * a, q))
    Observe(lhsfn, kernel, argfn)          Observe(y, Normal(Col("x"), r))
    Weight(kernel, argfn)                  Weight(Normal(Col("x"), r), y)
    Resample()                             Resample()
    Move(targets, RW|autoRW, argfn, div)   Move(["θ"], RW(0.3), diversity=0.9)
    Sequence / Loop / Cond                 Sequence / Loop / Cond (host control flow)

Julia closures (argfn) cannot run on the device; arguments are given as the affine
column expressions of ``dsl.py`` instead (the shapes @model's `vectorize` produces for
the supported kernels).
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Callable, Iterable, Sequence as Seq

import numpy as np

from . import abi
from .abi import Operand
from .context import Context
from .dsl import Expr, Kernel, _exprs, is_general, value_operands, xprogram


# ---------------------------------------------------------------------------------------
# store + state
# ---------------------------------------------------------------------------------------
class HipColumnStore:
    """AbstractParticleStore (src/stores.jl:1-35) over device columns."""

    def __init__(self, ctx):
        self.ctx = ctx

    def nparticles(self) -> int:
        return self.ctx.n

    def hascol(self, name: str) -> bool:
        return self.ctx.col_find(name) >= 0

    def getcol(self, name: str) -> np.ndarray:
        c = self.ctx.col_find(name)
        if c < 0:
            raise KeyError(name)
        return self.ctx.col_download(c)

    def colnames(self) -> list[str]:
        return self.ctx.col_names()

    def broadcast_setcol(self, name: str, values, dim: int | None = None) -> None:
        """broadcast_setcol!(store, name, identity, (values,)) — creates the column if needed."""
        v = np.asarray(values, dtype=np.float64)
        if dim is None:
            dim = 1 if v.ndim <= 1 else v.shape[0]
        c = self.ctx.col_create(name, dim)
        if v.size == 1 and self.ctx.n != 1:
            v = np.full(self.ctx.n * dim, float(v.reshape(-1)[0]))
        self.ctx.col_upload(c, v)

    def resample(self, indices) -> None:
        """resample!(store, indices) with 0-based indices (src/stores.jl:105-111)."""
        self.ctx.store_resample(indices)

    def resolve(self, name: str) -> int:
        c = self.ctx.col_find(name)
        if c < 0:
            raise KeyError(f"unknown particle variable {name!r}")
        return c

    def __repr__(self):
        return f"HipColumnStore(n={self.nparticles()}, columns={self.colnames()})"


class SMCState:
    """SMCState (src/types.jl:48-78): store + log-weights + flags, device-resident."""

    def __init__(self, n_particles: int, ess_perc_min: float = 0.5, seed: int = 42, device: int = 0,
                 scheme: int = abi.RESAMPLE_STRATIFIED):
        self._init(Context(n_particles, seed=seed, device=device), ess_perc_min, scheme)

    @classmethod
    def from_context(cls, ctx, ess_perc_min: float = 0.5, scheme: int = abi.RESAMPLE_STRATIFIED) -> "SMCState":
        s = cls.__new__(cls)
        s._init(ctx, ess_perc_min, scheme)
        return s

    def _init(self, ctx, ess_perc_min, scheme):
        self.ctx = ctx
        self.store = HipColumnStore(ctx)
        self.ess_perc_min = float(ess_perc_min)
        self.scheme = int(scheme)
        self.root = None

    # --- fields of the reference's SMCState ---
    @property
    def weights(self) -> np.ndarray:
        return self.ctx.weights_download()

    @weights.setter
    def weights(self, w) -> None:
        self.ctx.weights_upload(w)

    @property
    def resampled(self) -> bool:
        return bool(self.ctx.get_state()["resampled"])

    @property
    def weights_changed(self) -> bool:
        return bool(self.ctx.get_state()["weights_changed"])

    @property
    def depth(self) -> int:
        return self.ctx.get_state()["depth"]

    @depth.setter
    def depth(self, d: int) -> None:
        self.ctx.set_depth(int(d))

    def nparticles(self) -> int:
        return self.ctx.n

    def __getitem__(self, name: str) -> np.ndarray:
        return self.store.getcol(name)

    def log_evidence(self) -> float:
        """logsumexp(weights) - log(N) (src/utils.jl:21)."""
        return self.ctx.log_evidence()

    def __repr__(self):
        return f"SMCState(n_particles={self.nparticles()}, columns={self.store.colnames()})"


# ---------------------------------------------------------------------------------------
# transformers
# ---------------------------------------------------------------------------------------
class ParticleTransformer:
    def apply(self, state: SMCState) -> None:  # pragma: no cover - abstract
        raise NotImplementedError


def _ensure_col(state: SMCState, name: str, dim: int) -> int:
    return state.ctx.col_create(name, dim)


@dataclass
class Assign(ParticleTransformer):
    """x .= expr (src/transformers.jl:28-32); expr may be a constant, an Expr or a list."""
    lhs: str
    rhs: object

    def apply(self, state):
        dim = len(self.rhs) if isinstance(self.rhs, (list, tuple, np.ndarray)) else \
            (state.ctx.col_dim(state.ctx.col_find(self.lhs)) if state.store.hascol(self.lhs) else 1)
        if is_general(self.rhs):   # beyond the operand form: the general expression program
            comps = list(self.rhs) if isinstance(self.rhs, (list, tuple)) else [self.rhs]
            if len(comps) != dim:
                raise ValueError(f"{self.lhs}: give one expression per component ({dim})")
            c = _ensure_col(state, self.lhs, dim)
            prog, lens = xprogram(comps, state.store.resolve)
            state.ctx.assign_expr(c, prog, lens)
            return
        c = _ensure_col(state, self.lhs, dim)
        state.ctx.assign(c, value_operands(self.rhs, dim, state.store.resolve))


@dataclass
class ImportanceKernel:
    """importance_kernel(proposal, target) (src/default_kernels.jl:69-73)."""
    proposal: Kernel
    target: Kernel


def importance_kernel(proposal: Kernel, target: Kernel) -> ImportanceKernel:
    return ImportanceKernel(proposal, target)


@dataclass
class Sample(ParticleTransformer):
    """x ~ kernel (src/transformers.jl:172-182)."""
    lhs: str
    kernel: object

    def apply(self, state):
        R = state.store.resolve
        if isinstance(self.kernel, ImportanceKernel):
            c = _ensure_col(state, self.lhs, self.kernel.proposal.dim)
            state.ctx.sample_importance(c, self.kernel.proposal.dist(R), self.kernel.target.dist(R))
        else:
            c = _ensure_col(state, self.lhs, self.kernel.dim)
            state.ctx.sample(c, self.kernel.dist(R))


@dataclass
class Observe(ParticleTransformer):
    """value => kernel (src/transformers.jl:228-235)."""
    value: object
    kernel: Kernel

    def apply(self, state):
        R = state.store.resolve
        state.ctx.observe(self.kernel.dist(R), value_operands(self.value, self.kernel.dim, R))


@dataclass
class Weight(ParticleTransformer):
    """_ ~ f(args) (src/transformers.jl:283-289): adds logpdf(kernel, value)."""
    kernel: Kernel
    value: object

    def apply(self, state):
        R = state.store.resolve
        state.ctx.weight(self.kernel.dist(R), value_operands(self.value, self.kernel.dim, R))


@dataclass
class Resample(ParticleTransformer):
    """Resample() (src/transformers.jl:474-498); scheme: stratified (reference), systematic or
    multinomial."""
    scheme: int | None = None

    def apply(self, state):
        scheme = state.scheme if self.scheme is None else self.scheme
        state.ctx.resample(state.ess_perc_min, scheme)


@dataclass
class Proposal:
    kind: int
    step: float
    bounds: object = None

    def bounds_arrays(self, d: int):
        """_normalize_bounds (src/move_kernels.jl:23-28)."""
        if self.bounds is None:
            return None, None
        b = self.bounds
        if isinstance(b, tuple) and len(b) == 2 and not isinstance(b[0], (tuple, list)):
            return [float(b[0])] * d, [float(b[1])] * d
        b = list(b)
        if len(b) != d:
            raise ValueError(f"bounds must have length {d} (one (lo, hi) tuple per target), got {len(b)}")
        return [float(x[0]) for x in b], [float(x[1]) for x in b]


def RW(step_size: float, bounds=None) -> Proposal:
    """RW(state, targets, step_size, bounds) (src/move_kernels.jl:189-212); step_size is a std."""
    return Proposal(abi.PROPOSAL_RW, float(step_size), bounds)


def autoRW(min_step: float = 1e-3, bounds=None) -> Proposal:
    """autoRW(state, targets, min_step, bounds) (src/move_kernels.jl:232-253)."""
    return Proposal(abi.PROPOSAL_AUTORW, float(min_step), bounds)


@dataclass
class Move(ParticleTransformer):
    """targets << proposal (src/transformers.jl:588-623); depth- and score-neutral."""
    targets: Seq[str]
    proposal: Proposal
    diversity: float | None = None

    def apply(self, state):
        R = state.store.resolve
        cols = [R(t) for t in self.targets]
        lo, hi = self.proposal.bounds_arrays(len(cols))
        div = math.nan if self.diversity is None else float(self.diversity)
        state.ctx.move(self.proposal.kind, cols, self.proposal.step, lo, hi, -1, div)


class Sequence(ParticleTransformer):
    """Sequence(steps...) (src/transformers.jl:320-334)."""

    def __init__(self, *steps):
        self.steps = tuple(steps[0]) if len(steps) == 1 and isinstance(steps[0], (list, tuple)) else steps

    def apply(self, state):
        for s in self.steps:
            s.apply(state)


@dataclass
class Loop(ParticleTransformer):
    """for x in collection; body(x); end (src/transformers.jl:367-383)."""
    collection: Iterable
    body: Callable

    def apply(self, state):
        coll = self.collection(state) if callable(self.collection) else self.collection
        for x in coll:
            self.body(x).apply(state)


@dataclass
class Cond(ParticleTransformer):
    """if pred; body; end (src/transformers.jl:413-428); pred reads host state only."""
    pred: Callable
    body: ParticleTransformer

    def apply(self, state):
        if self.pred(state):
            self.body.apply(state)


def apply(t: ParticleTransformer, state: SMCState) -> SMCState:
    t.apply(state)
    return state


def run(root: ParticleTransformer, state: SMCState) -> SMCState:
    """run!(root, state) (src/types.jl:120-126)."""
    state.root = root
    root.apply(state)
    return state


def score_logpdf(state: SMCState, targets, target_depth: int) -> np.ndarray:
    """score_logpdf(state, targets, target_depth) (src/types.jl:185-206)."""
    return state.ctx.score(int(target_depth))


def marginal_diversity(store: HipColumnStore, targets) -> float:
    """marginal_diversity(store, targets) (src/transformers.jl:560-565)."""
    return store.ctx.marginal_diversity([store.resolve(t) for t in targets])


# ---------------------------------------------------------------------------------------
# analysis (src/utils.jl), reduced on the device
# ---------------------------------------------------------------------------------------
def expectation(state: SMCState, expr) -> float:
    """Weighted expectation under exp_norm(weights) (src/utils.jl:11; @E, :23-58) of an affine
    expression of particle variables, e.g. ``expectation(state, Col("x"))`` or
    ``Col("alpha") + 2.0 * Col("beta")``. Non-affine functions are evaluated on the host from
    ``state[name]``."""
    mean, _ = state.ctx.weighted_moments([Expr.lift(expr).operand(state.store.resolve)], want_cov=False)
    return float(mean[0])


def sample(state: SMCState, n: int, replace: bool = True) -> dict:
    """StatsBase.sample(state, n; replace) (src/utils.jl:92-118): n particles drawn by the
    normalised weights, one entry per column (``values[indices]``; vector columns [n, dim]).
    The indices are drawn and the rows gathered on the device."""
    idx = state.ctx.sample_particles(n, replace)
    out = {}
    for name in state.store.colnames():
        v = state.ctx.col_gather_rows(state.store.resolve(name), idx)
        out[name] = v if v.ndim == 1 else v.T
    return out


def dataframe(state: SMCState) -> dict:
    """DataFrame(state) (src/utils.jl:69-88): every column plus ``log_weight`` (the raw
    log-weights), unnormalised; a host copy of the whole population."""
    out = {}
    for name in state.store.colnames():
        v = state.ctx.col_download(state.store.resolve(name))
        out[name] = v if v.ndim == 1 else v.T
    out["log_weight"] = state.ctx.weights_download()
    return out


SPARK_CHARS = "▁▂▃▄▅▆▇█"


def describe(state: SMCState, cols=None) -> list[dict]:
    """describe(state; cols) (src/utils.jl:157-289): per numeric column its weighted mean,
    weighted median (StatsBase quantile 0.5), weighted std (StatsBase, corrected=false), min,
    max, the 8-bin weighted sparkline (scalar columns; "" for vector columns) and
    ESS = N * ess_perc; vector columns component-wise. Everything is reduced on the device
    (the median and histogram on the integer weights, include/wsmc_math.h)."""
    store = state.store
    names = store.colnames() if cols is None else list(cols)
    for n in names:
        if not store.hascol(n):
            raise ValueError(f"Column {n} not found in store")
    ess = state.nparticles() * state.ctx.ess()
    rows = []
    for n in names:
        c = store.resolve(n)
        d = state.ctx.col_dim(c)
        means, stds, mins, maxs, meds = [], [], [], [], []
        for k0 in range(0, d, 4):
            ks = list(range(k0, min(d, k0 + 4)))
            mean, cov = state.ctx.weighted_moments([Operand.column(c, k) for k in ks])
            means += list(mean)
            stds += [math.sqrt(cov[j, j]) for j in range(len(ks))]
        for k in range(d):
            mn, mx = state.ctx.col_minmax(c, k)
            mins.append(mn)
            maxs.append(mx)
            meds.append(state.ctx.weighted_median(c, k))
        one = d == 1
        hist = "".join(SPARK_CHARS[v - 1] for v in state.ctx.histogram(c, 0)) if one else ""
        rows.append(dict(variable=n, mean=means[0] if one else means, median=meds[0] if one else meds,
                         std=stds[0] if one else stds, min=mins[0] if one else mins,
                         max=maxs[0] if one else maxs, hist=hist, ess=ess))
    return rows


def resampled(state: SMCState) -> bool:
    """The `if resampled` predicate of @model bodies (src/rewrites.jl:360-368)."""
    return state.resampled


# ---------------------------------------------------------------------------------------
# fused model steps (one HIP graph per run)
# ---------------------------------------------------------------------------------------
@dataclass
class FusedSSM2D(ParticleTransformer):
    """The whole examples/2D_ssm.jl program as one device graph; same state as the
    statement-by-statement program (tests/test_gpu_parity.py)."""
    obs: object
    x0: tuple = (0.0, 0.0)
    v0: tuple = (1.0, 0.0)
    q_var: float = 0.1
    r_var: float = 0.5
    keep_history: bool = True

    def apply(self, state):
        state.ctx.ssm2d_run(self.obs, self.x0, self.v0, self.q_var, self.r_var, state.ess_perc_min,
                            state.scheme, self.keep_history, want_evidence=False)
