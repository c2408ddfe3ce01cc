"""Argument expressions and kernel descriptors.

The reference builds each statement's arguments with a Julia closure produced by
``vectorize`` (src/rewrites.jl:146-219) and resolves kernels from ``default_kernels``
(src/default_kernels.jl:83-102). The device path accepts the shapes those closures take
on the supported kernels: constants (``Ref(c)``), columns, and affine combinations of up
to two column components (``α + β * x``, ``a .* x``, ``x{t} + v``).

    Col("x")            column x (component 0)
    Col("x", 1)         component 1 of a vector column
    2.0 * Col("x") + 1  affine forms
    Normal(mu, sigma), MvNormal(mu, cov), HalfNormal(sigma), Uniform(a, b)
    Oscillator(t, A, ω, γ, ϕ)  the damped-oscillator mean (examples/damped_oscillator.jl:11)
"""
from __future__ import annotations

import ctypes as C
import math
from dataclasses import dataclass, field
from typing import Sequence, Union

import numpy as np

from . import abi
from .abi import Dist, Operand

Number = Union[int, float]


@dataclass(frozen=True)
class Expr:
    """c0 + sum coef * column[comp] over at most two (column, component) pairs."""
    c0: float = 0.0
    terms: tuple = ()   # ((name, comp, coef), ...)

    @staticmethod
    def lift(v) -> "Expr":
        if isinstance(v, Expr):
            return v
        if isinstance(v, (int, float, np.floating, np.integer)):
            return Expr(float(v), ())
        raise TypeError(f"cannot use {v!r} as a particle argument")

    def __add__(self, o):
        o = Expr.lift(o)
        return Expr(self.c0 + o.c0, self.terms + o.terms)._checked()

    __radd__ = __add__

    def __neg__(self):
        return Expr(-self.c0, tuple((n, c, -k) for n, c, k in self.terms))

    def __sub__(self, o):
        return self + (-Expr.lift(o))

    def __rsub__(self, o):
        return Expr.lift(o) + (-self)

    def __mul__(self, k):
        if isinstance(k, Expr):
            if not k.terms:
                k = k.c0
            elif not self.terms:
                return k * self.c0
            else:
                raise TypeError("products of two particle columns are not affine")
        k = float(k)
        return Expr(self.c0 * k, tuple((n, c, coef * k) for n, c, coef in self.terms))

    __rmul__ = __mul__

    def _checked(self) -> "Expr":
        if len(self.terms) > 2:
            raise ValueError("device argument forms support at most two column terms")
        return self

    def operand(self, resolve) -> Operand:
        o = Operand.const(self.c0)
        for k, (name, comp, coef) in enumerate(self.terms):
            o.col[k] = resolve(name)
            o.comp[k] = int(comp)
            o.coef[k] = float(coef)
        return o

    def columns(self):
        return [n for n, _, _ in self.terms]


def Col(name: str, comp: int = 0) -> Expr:
    return Expr(0.0, ((str(name), int(comp), 1.0),))


def _exprs(v, dim: int) -> list[Expr]:
    if isinstance(v, (list, tuple, np.ndarray)):
        vs = [Expr.lift(x) for x in v]
        if len(vs) != dim:
            raise ValueError(f"expected {dim} components, got {len(vs)}")
        return vs
    e = Expr.lift(v)
    if dim == 1:
        return [e]
    # a vector column referenced whole: component k of the same column(s)
    if e.terms and all(c == 0 for _, c, _ in e.terms):
        return [Expr(e.c0, tuple((n, k, coef) for n, _, coef in e.terms)) for k in range(dim)]
    return [e] * dim


@dataclass(frozen=True)
class Oscillator:
    """A * exp(-γ t) * cos(ω t + ϕ) (examples/damped_oscillator.jl:11)."""
    t: float
    A: object
    omega: object
    gamma: object
    phi: object


@dataclass(frozen=True)
class Kernel:
    """A device-supported WeightedKernel (weighter === nothing; src/types.jl:226-230)."""
    family: int
    dim: int
    mean: tuple = ()          # Exprs (or an Oscillator)
    scale: object = 1.0       # sigma (std) or variance (MvNormal iso)
    params: tuple = (0.0, 0.0)
    cov: tuple = ()           # FAM_MVNORMAL: Σ row-major (packed by the library)

    def dist(self, resolve) -> Dist:
        d = Dist()
        d.family = self.family
        d.dim = self.dim
        d.mean_fn = abi.MEAN_AFFINE
        for k in range(4):
            d.mu[k] = Operand.const(0.0)
        if isinstance(self.mean, Oscillator):
            d.mean_fn = abi.MEAN_OSCILLATOR
            o = self.mean
            for k, v in enumerate((o.A, o.omega, o.gamma, o.phi)):
                d.mu[k] = Expr.lift(v).operand(resolve)
            d.param[0] = float(o.t)
        else:
            for k, e in enumerate(self.mean):
                d.mu[k] = Expr.lift(e).operand(resolve)
        d.scale = Expr.lift(self.scale).operand(resolve)
        if self.family == abi.FAM_UNIFORM:
            d.param[0], d.param[1] = float(self.params[0]), float(self.params[1])
        if self.family == abi.FAM_MVNORMAL:
            S = (C.c_double * len(self.cov))(*self.cov)
            abi.check(abi.load_library().wsmc_dist_mvnormal_cov(C.byref(d), S))
        return d

    def columns(self):
        out = []
        means = self.mean
        if isinstance(means, Oscillator):
            means = (means.A, means.omega, means.gamma, means.phi)
        for e in list(means) + [self.scale]:
            out += Expr.lift(e).columns()
        return out


def Normal(mu=0.0, sigma=1.0) -> Kernel:
    """default_kernels.Normal(μ, σ) — σ is a standard deviation."""
    if isinstance(mu, Oscillator):
        return Kernel(abi.FAM_NORMAL, 1, mu, sigma)
    return Kernel(abi.FAM_NORMAL, 1, (Expr.lift(mu),), sigma)


def HalfNormal(sigma=1.0) -> Kernel:
    """Truncated(Normal(0, σ), 0, Inf) — the examples/damped_oscillator.jl:24-28 kernel."""
    return Kernel(abi.FAM_HALFNORMAL, 1, (Expr.lift(0.0),), sigma)


def Uniform(a: float, b: float) -> Kernel:
    """default_kernels.Uniform(a, b)."""
    return Kernel(abi.FAM_UNIFORM, 1, (Expr.lift(0.0),), 1.0, (float(a), float(b)))


def MvNormal(mu, cov) -> Kernel:
    """default_kernels.MvNormal(μ, Σ) — Σ is a COVARIANCE (src/default_kernels.jl:93). A scalar
    or Σ = v·I takes the isotropic family (dim ≤ 4); any other constant Σ (dim ≤ 3) takes the
    full-covariance family, its Cholesky factor packed once by wsmc_dist_mvnormal_cov."""
    if isinstance(cov, (int, float, np.floating)):
        var = float(cov)
        mus = mu if isinstance(mu, (list, tuple, np.ndarray)) else None
        dim = len(mus) if mus is not None else None
    else:
        S = np.asarray(cov, dtype=float)
        if S.ndim != 2 or S.shape[0] != S.shape[1]:
            raise ValueError("covariance must be square")
        var = float(S[0, 0])
        dim = S.shape[0]
        if not np.array_equal(S, var * np.eye(dim)):
            if not 1 <= dim <= 3:
                raise ValueError("MvNormal with a full covariance: dimension must be 1..3")
            return Kernel(abi.FAM_MVNORMAL, dim, tuple(_exprs(mu, dim)), 0.0, cov=tuple(S.ravel()))
    if dim is None:
        raise ValueError("MvNormal with a scalar variance needs an explicit mean vector")
    if not 1 <= dim <= 4:
        raise ValueError("MvNormal dimension must be 1..4")
    return Kernel(abi.FAM_MVNORMAL_ISO, dim, tuple(_exprs(mu, dim)), var)


def value_operands(v, dim: int, resolve) -> list[Operand]:
    return [e.operand(resolve) for e in _exprs(v, dim)]
