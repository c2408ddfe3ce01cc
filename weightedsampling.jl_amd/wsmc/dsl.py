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


def _pow2(k: float) -> bool:
    m, _ = math.frexp(k)
    return k != 0.0 and math.isfinite(k) and abs(m) == 0.5


@dataclass(frozen=True)
class Expr:
    """c0 + sum coef * column[comp] over at most two (column, component) pairs — the operand form,
    evaluated as (c0 + coef0 x0) + coef1 x1 (include/wsmc_terms.h wsmc_operand_eval). While that
    order rounds exactly as the user's own operations (Julia's broadcast) `fx` is None; an
    operation that would round differently in the merged form (a constant added after two terms,
    a sum scaled by a non power of two, ...) records the user's order in `fx`, and a program
    (wsmc_assign_expr) evaluates that instead. A distribution argument always takes the operand
    form (its value then within a rounding of the broadcast's)."""
    c0: float = 0.0
    terms: tuple = ()   # ((name, comp, coef), ...)
    fx: object = field(default=None, compare=False)

    @staticmethod
    def lift(v) -> "Expr":
        if isinstance(v, Expr):
            return v
        if isinstance(v, (int, float, np.floating, np.integer)):
            return Expr(float(v), ())
        if isinstance(v, Fx):
            raise TypeError("a distribution argument must be affine in at most two columns (the "
                            "operand form); assign the general expression to a column first")
        raise TypeError(f"cannot use {v!r} as a particle argument")

    def _sum_exact(self, o: "Expr") -> bool:
        """(self) + (o) rounds as the merged operand form does (signed zeros aside)"""
        if self.fx is not None or o.fx is not None:
            return False
        na, nb = len(self.terms), len(o.terms)
        if nb == 0:
            return o.c0 == 0.0 or (self.c0 == 0.0 and na <= 1)
        if na == 0:
            return self.c0 == 0.0 or (o.c0 == 0.0 and nb <= 1)
        return o.c0 == 0.0

    def __add__(self, o, swap=False):
        if isinstance(o, Fx):
            return o + Fx.lift(self) if swap else Fx.lift(self) + o
        o = Expr.lift(o)
        a, b = (o, self) if swap else (self, o)
        if len(a.terms) + len(b.terms) > 2:   # beyond the operand form: a general expression
            return Fx.lift(a) + Fx.lift(b)
        merged = Expr(a.c0 + b.c0, a.terms + b.terms)
        if a._sum_exact(b):
            return merged
        return Expr(merged.c0, merged.terms, Fx(abi.X_ADD, (Fx.lift(a), Fx.lift(b))))

    def __radd__(self, o):
        return self.__add__(o, swap=True)

    def __neg__(self):
        return Expr(-self.c0, tuple((n, c, -k) for n, c, k in self.terms),
                    None if self.fx is None else -self.fx)

    def __sub__(self, o):
        if isinstance(o, Fx):
            return Fx.lift(self) - o
        return self + (-Expr.lift(o))

    def __rsub__(self, o):
        return Expr.lift(o) + (-self)   # a - b is a + (-b) exactly

    # the non-affine operators give general expressions (Assign only: wsmc_assign_expr)
    def __truediv__(self, o):
        return Fx.lift(self) / o

    def __rtruediv__(self, o):
        return Fx.lift(o) / Fx.lift(self)

    def __pow__(self, o):
        return Fx.lift(self) ** o

    def __rpow__(self, o):
        return Fx.lift(o) ** Fx.lift(self)

    def __abs__(self):
        return abs(Fx.lift(self))

    def __lt__(self, o):
        return Fx.lift(self) < o

    def __le__(self, o):
        return Fx.lift(self) <= o

    def __gt__(self, o):
        return Fx.lift(self) > o

    def __ge__(self, o):
        return Fx.lift(self) >= o

    def __mul__(self, k):
        if isinstance(k, Fx):
            return Fx.lift(self) * k
        if isinstance(k, Expr):
            if not k.terms:
                k = k.c0
            elif not self.terms:
                return k * self.c0
            else:   # a product of two particle columns: a general expression
                return Fx.lift(self) * Fx.lift(k)
        k = float(k)
        scaled = Expr(self.c0 * k, tuple((n, c, coef * k) for n, c, coef in self.terms))
        # k (c0 + coef x + ...) distributes exactly for a constant, k = +-2^n, or k * x alone
        exact = self.fx is None and (not self.terms or _pow2(k) or
                                     (len(self.terms) == 1 and self.c0 == 0.0 and self.terms[0][2] == 1.0))
        if exact:
            return scaled
        return Expr(scaled.c0, scaled.terms, Fx(abi.X_MUL, (Fx.lift(self), Fx(abi.X_CONST, c=k))))

    __rmul__ = __mul__

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


def _scalar(fam, loc=0.0, scale=1.0) -> Kernel:
    return Kernel(fam, 1, (Expr.lift(loc),), scale)


def Bernoulli(p) -> Kernel:
    """default_kernels.Bernoulli(p): draws 1.0 / 0.0"""
    return _scalar(abi.FAM_BERNOULLI, p)


def BernoulliLogit(logitp) -> Kernel:
    return _scalar(abi.FAM_BERNOULLI_LOGIT, logitp)


def Exponential(theta=1.0) -> Kernel:
    """default_kernels.Exponential(θ) — θ is the scale (the mean)"""
    return _scalar(abi.FAM_EXPONENTIAL, 0.0, theta)


def LogNormal(mu=0.0, sigma=1.0) -> Kernel:
    return _scalar(abi.FAM_LOGNORMAL, mu, sigma)


def Laplace(mu=0.0, theta=1.0) -> Kernel:
    return _scalar(abi.FAM_LAPLACE, mu, theta)


def Cauchy(mu=0.0, sigma=1.0) -> Kernel:
    return _scalar(abi.FAM_CAUCHY, mu, sigma)


def Logistic(mu=0.0, theta=1.0) -> Kernel:
    return _scalar(abi.FAM_LOGISTIC, mu, theta)


def Gumbel(mu=0.0, theta=1.0) -> Kernel:
    return _scalar(abi.FAM_GUMBEL, mu, theta)


def Rayleigh(sigma=1.0) -> Kernel:
    return _scalar(abi.FAM_RAYLEIGH, 0.0, sigma)


def Geometric(p) -> Kernel:
    """default_kernels.Geometric(p): failures before the first success (0, 1, 2, ...)"""
    return _scalar(abi.FAM_GEOMETRIC, p)


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


# ---------------------------------------------------------------------------------------
# general expressions (wsmc_assign_expr)
# ---------------------------------------------------------------------------------------
_COMMUTATIVE = (abi.X_ADD, abi.X_MUL)


class Fx:
    """A general particle expression: the fused broadcast `vectorize` emits for an Assign's
    right-hand side (src/rewrites.jl:146-219) — calls, `cond ? a : b` (ifelse), `||` / `&&`,
    comparisons — as a tree over columns and constants, lowered to wsmc_assign_expr's postfix
    program. Booleans are 1.0 / 0.0 (the columns are Float64)."""

    __slots__ = ("op", "args", "c", "col", "comp")

    def __init__(self, op: int, args=(), c: float = 0.0, col=None, comp: int = 0):
        self.op, self.args, self.c, self.col, self.comp = int(op), tuple(args), float(c), col, int(comp)

    @staticmethod
    def lift(v) -> "Fx":
        if isinstance(v, Fx):
            return v
        if isinstance(v, (bool, np.bool_)):
            return Fx(abi.X_CONST, c=1.0 if v else 0.0)
        if isinstance(v, (int, float, np.floating, np.integer)):
            return Fx(abi.X_CONST, c=float(v))
        if isinstance(v, Expr):
            if v.fx is not None:   # the user's order (the merged form would round differently)
                return v.fx
            # the affine form in wsmc_operand_eval's order: its constant first when nonzero, then
            # the terms left to right (x, coef * x, -x), ((c0 + t0) + t1): the user's own order
            # whenever fx is None (Expr._sum_exact), so the value is the same bits as an operand
            # or inside a program
            e = Fx(abi.X_CONST, c=v.c0) if v.c0 != 0.0 else None
            for name, comp, coef in v.terms:
                x = Fx(abi.X_COL, col=name, comp=comp)
                t = x if coef == 1.0 else (Fx(abi.X_NEG, (x,)) if coef == -1.0 else
                                           Fx(abi.X_MUL, (Fx(abi.X_CONST, c=coef), x)))
                e = t if e is None else Fx(abi.X_ADD, (e, t))
            return e if e is not None else Fx(abi.X_CONST, c=v.c0)
        raise TypeError(f"cannot use {v!r} in a particle expression")

    def _bin(self, op, o, swap=False):
        a, b = (Fx.lift(o), self) if swap else (self, Fx.lift(o))
        return Fx(op, (a, b))

    __add__ = lambda s, o: s._bin(abi.X_ADD, o)
    __radd__ = lambda s, o: s._bin(abi.X_ADD, o, True)
    __sub__ = lambda s, o: s._bin(abi.X_SUB, o)
    __rsub__ = lambda s, o: s._bin(abi.X_SUB, o, True)
    __mul__ = lambda s, o: s._bin(abi.X_MUL, o)
    __rmul__ = lambda s, o: s._bin(abi.X_MUL, o, True)
    __truediv__ = lambda s, o: s._bin(abi.X_DIV, o)
    __rtruediv__ = lambda s, o: s._bin(abi.X_DIV, o, True)
    __lt__ = lambda s, o: s._bin(abi.X_LT, o)
    __le__ = lambda s, o: s._bin(abi.X_LE, o)
    __gt__ = lambda s, o: s._bin(abi.X_GT, o)
    __ge__ = lambda s, o: s._bin(abi.X_GE, o)
    __neg__ = lambda s: Fx(abi.X_NEG, (s,))
    __abs__ = lambda s: Fx(abi.X_ABS, (s,))

    def __pow__(self, o):
        if isinstance(o, (int, np.integer)) and not isinstance(o, bool):   # x^n (Base.literal_pow / pow_body)
            return Fx(abi.X_POWI, (self,), c=float(o))
        return self._bin(abi.X_POW, o)

    def __rpow__(self, o):
        return self._bin(abi.X_POW, o, True)

    def __bool__(self):
        raise TypeError("a particle expression has no truth value on the host; use ifelse / and_ / or_")

    # ---- lowering ----
    def _need(self) -> int:
        """stack values needed to evaluate (Sethi–Ullman, with the operand order _emit uses)"""
        if not self.args:
            return 1
        if self.op in _COMMUTATIVE:
            a, b = sorted((x._need() for x in self.args), reverse=True)
            return max(a, b + 1)
        return max(x._need() + k for k, x in enumerate(self.args))

    def _emit(self, resolve, out: list) -> None:
        args = self.args
        if self.op in _COMMUTATIVE and args[1]._need() > args[0]._need():
            args = (args[1], args[0])   # a + b == b + a, a * b == b * a bit for bit: the deeper first
        for a in args:
            a._emit(resolve, out)
        col = resolve(self.col) if self.op == abi.X_COL else -1
        out.append((self.op, col, self.comp if self.op == abi.X_COL else 0, self.c))

    def columns(self):
        if self.op == abi.X_COL:
            return [self.col]
        return [n for a in self.args for n in a.columns()]

    def __repr__(self):
        if self.op == abi.X_CONST:
            return repr(self.c)
        if self.op == abi.X_COL:
            return f"Col({self.col!r}, {self.comp})" if self.comp else f"Col({self.col!r})"
        return f"Fx({self.op}, {self.args!r}{', c=%r' % self.c if self.op == abi.X_POWI else ''})"


def _un(op):
    return lambda x: Fx(op, (Fx.lift(x),))


exp, log, log1p, sqrt, sin, cos, not_ = (_un(o) for o in (abi.X_EXP, abi.X_LOG, abi.X_LOG1P, abi.X_SQRT, abi.X_SIN,
                                                       abi.X_COS, abi.X_NOT))
exp.__doc__ = "exp.(x)"


def _bin2(op):
    return lambda a, b: Fx(op, (Fx.lift(a), Fx.lift(b)))


min_, max_, eq, ne, and_, or_ = (_bin2(o) for o in (abi.X_MIN, abi.X_MAX, abi.X_EQ, abi.X_NE, abi.X_AND, abi.X_OR))


def ifelse(cond, a, b) -> Fx:
    """cond ? a : b — ifelse.(cond, a, b): both sides evaluated (src/rewrites.jl:193-200)"""
    return Fx(abi.X_IFELSE, (Fx.lift(cond), Fx.lift(a), Fx.lift(b)))


def is_general(v) -> bool:
    """True when an Assign right-hand side needs wsmc_assign_expr (not the operand form)"""
    vs = v if isinstance(v, (list, tuple)) else [v]
    return any(isinstance(x, Fx) for x in vs)


def xprogram(components, resolve):
    """(XInst array, per-component lengths) for wsmc_assign_expr / the oracle's or_assign_expr"""
    ins = []
    lens = []
    for e in components:
        e = Fx.lift(e)
        if e._need() > abi.XSTACK_MAX:
            raise ValueError(f"expression needs more than {abi.XSTACK_MAX} stack values: {e!r}")
        n0 = len(ins)
        e._emit(resolve, ins)
        lens.append(len(ins) - n0)
    if len(ins) > abi.XPROG_MAX:
        raise ValueError(f"expression longer than {abi.XPROG_MAX} instructions")
    arr = (abi.XInst * max(1, len(ins)))()
    for k, (op, col, comp, c) in enumerate(ins):
        arr[k].op, arr[k].col, arr[k].comp, arr[k].c = op, col, comp, c
    return arr, lens
