"""General Assign expressions (wsmc_assign_expr) on the CPU: the oracle's program machine
(include/wsmc_terms.h wsmc_xeval over wsmc_xop1 / wsmc_xop2) against numpy's functions, the
Julia Base semantics the operators restate (min / max signed zeros and NaN, literal_pow, the
domain errors that become NaN), and the DSL's lowering to postfix programs. The HIP kernel is
compared with the oracle bit for bit in tests/test_gpu_expr.py."""
import math

import numpy as np
import pytest

from oracle import Oracle
from wsmc import abi, dsl
from wsmc.dsl import Col, Fx, and_, cos, eq, exp, ifelse, log, log1p, max_, min_, ne, not_, or_, sin, sqrt

N = 2000


def make(seed=3):
    rng = np.random.default_rng(seed)
    o = Oracle(N, seed=1)
    cols = {}
    for name, v in (("a", rng.normal(0.0, 2.0, N)), ("b", rng.uniform(0.1, 3.0, N)),
                    ("c", rng.integers(0, 2, N).astype(float)), ("d", rng.normal(0.0, 30.0, N))):
        cols[name] = v
        o.col_upload(o.col_create(name), v)
    vec = np.stack([rng.normal(size=N), rng.normal(size=N)])
    o.col_upload(o.col_create("v", 2), vec)
    cols["v"] = vec
    return o, cols


def run(o, exprs, out="out", dim=None):
    exprs = exprs if isinstance(exprs, list) else [exprs]
    c = o.col_create(out, dim or len(exprs))
    prog, lens = dsl.xprogram(exprs, o.col_find)
    o.assign_expr(c, prog, lens)
    return o.col_download(c)


@pytest.mark.parametrize("name,expr,ref,rtol", [
    ("exp", lambda: exp(Col("a")), lambda c: np.exp(c["a"]), 2e-16 * 4),
    ("log", lambda: log(Col("b")), lambda c: np.log(c["b"]), 2e-16 * 4),
    ("log1p", lambda: log1p(Col("b")), lambda c: np.log1p(c["b"]), 2e-16 * 8),
    ("sqrt", lambda: sqrt(Col("b")), lambda c: np.sqrt(c["b"]), 0.0),
    ("sin", lambda: sin(Col("d")), lambda c: np.sin(c["d"]), 1e-15),
    ("cos", lambda: cos(Col("d")), lambda c: np.cos(c["d"]), 1e-15),
    ("affine", lambda: 2.0 * Col("a") + Col("b") - 1.0, lambda c: (2.0 * c["a"] + c["b"]) - 1.0, 0.0),
    ("product", lambda: Col("a") * Col("b") / Col("d"), lambda c: c["a"] * c["b"] / c["d"], 0.0),
    ("powi", lambda: Col("a") ** 2 + Col("b") ** -2 + Col("a") ** 3, lambda c: (c["a"] * c["a"] + (1 / c["b"]) ** 2) +
     c["a"] * c["a"] * c["a"], 0.0),
    ("powi7", lambda: Col("b") ** 7, lambda c: c["b"] ** 7, 2e-16 * 2),
    ("powi-5", lambda: Col("b") ** -5, lambda c: c["b"] ** -5.0, 2e-16 * 2),
    ("pow", lambda: Col("b") ** (Col("a") * 0.5), lambda c: c["b"] ** (c["a"] * 0.5), 1e-14),
    ("minmax", lambda: min_(Col("a"), Col("d")) + max_(Col("a"), 0.0),
     lambda c: np.minimum(c["a"], c["d"]) + np.maximum(c["a"], 0.0), 0.0),
    ("compare", lambda: (Col("a") < Col("d")) + 2.0 * (Col("a") >= 0.5) + 4.0 * eq(Col("c"), 1.0),
     lambda c: (c["a"] < c["d"]) + 2.0 * (c["a"] >= 0.5) + 4.0 * (c["c"] == 1.0), 0.0),
    ("ifelse", lambda: ifelse(Col("c"), 0.9, 0.01), lambda c: np.where(c["c"] != 0, 0.9, 0.01), 0.0),
    ("logic", lambda: ifelse(or_(Col("c"), Col("a") > 1.0), 0.98, 0.01) + and_(Col("c"), not_(Col("c"))),
     lambda c: np.where((c["c"] != 0) | (c["a"] > 1.0), 0.98, 0.01), 0.0),
    ("oscillator", lambda: Col("b") * exp(-0.1 * Col("b") * 3.0) * cos(Col("a") * 3.0 + Col("d")),
     lambda c: c["b"] * np.exp(-0.1 * c["b"] * 3.0) * np.cos(c["a"] * 3.0 + c["d"]), 1e-14),
    ("component", lambda: Col("v", 1) * Col("v", 0), lambda c: c["v"][1] * c["v"][0], 0.0),
])
def test_oracle_expression_matches_numpy(name, expr, ref, rtol):
    o, c = make()
    got = run(o, expr())
    want = ref(c)
    if rtol == 0.0:
        np.testing.assert_array_equal(got, want)
    else:
        np.testing.assert_allclose(got, want, rtol=rtol, atol=0.0)
    assert o.get_state()["depth"] == 1


def test_julia_base_semantics():
    o = Oracle(8, seed=1)
    a = np.array([-0.0, 0.0, np.nan, 1.0, -2.0, -1.0, 2.0, np.inf])
    b = np.array([0.0, -0.0, 1.0, np.nan, 3.0, 0.5, -0.0, np.inf])
    o.col_upload(o.col_create("a"), a)
    o.col_upload(o.col_create("b"), b)

    def bits(x):
        return np.asarray(x, dtype=np.float64).view(np.uint64)

    mn = run(o, min_(Col("a"), Col("b")), "mn")
    mx = run(o, max_(Col("a"), Col("b")), "mx")
    # Base.min(-0.0, 0.0) = -0.0, min(0.0, -0.0) = -0.0; max the +0.0; NaN propagates
    assert bits(mn[0]) == bits(-0.0) and bits(mn[1]) == bits(-0.0)
    assert bits(mx[0]) == bits(0.0) and bits(mx[1]) == bits(0.0)
    assert np.isnan(mn[2]) and np.isnan(mn[3]) and np.isnan(mx[2]) and np.isnan(mx[3])
    assert mn[4] == -2.0 and mx[4] == 3.0 and mn[7] == np.inf
    p = run(o, Col("a") ** Col("b"), "p")
    assert p[4] == -8.0                      # a negative base to an integer power
    assert np.isnan(p[5])                    # (-1.0)^0.5: Julia's DomainError is NaN here
    assert p[6] == 1.0 and p[0] == 1.0       # x^0 = 1
    assert p[3] == 1.0                       # 1.0^NaN is 1 in Julia (a == 1 first)
    s = run(o, [sqrt(Col("a"))], "s")
    assert np.isnan(s[4]) and bits(s[0]) == bits(-0.0)
    lg = run(o, log(Col("a")), "lg")
    assert np.isnan(lg[4]) and lg[1] == -np.inf
    sn = run(o, sin(Col("a")), "sn")
    assert bits(sn[0]) == bits(-0.0) and np.isnan(sn[7])
    # Base.literal_pow: x^-1 = inv(x), x^-2 = inv(x)^2, x^3 = x*x*x
    q = run(o, [Col("b") ** -1 + Col("b") ** -2 * 0.0], "q")
    assert q[4] == 1.0 / 3.0


def test_julia_one_to_a_nan_power_is_one():
    o = Oracle(2, seed=1)
    o.col_upload(o.col_create("a"), np.array([1.0, 2.0]))
    o.col_upload(o.col_create("b"), np.array([np.nan, np.nan]))
    p = run(o, Col("a") ** Col("b"), "p")
    assert p[0] == 1.0 and np.isnan(p[1])


def test_vector_output_reads_its_own_components():
    """x .= [x[2], x[1]] : every component is evaluated before any is stored"""
    o, c = make()
    vid = o.col_find("v")
    prog, lens = dsl.xprogram([Col("v", 1), Col("v", 0)], o.col_find)
    o.assign_expr(vid, prog, lens)
    got = o.col_download(vid)
    np.testing.assert_array_equal(got[0], c["v"][1])
    np.testing.assert_array_equal(got[1], c["v"][0])


def test_program_shape_checks():
    o, _ = make()
    out = o.col_create("out")

    def prog(ins):
        arr = (abi.XInst * len(ins))()
        for k, (op, col, c) in enumerate(ins):
            arr[k].op, arr[k].col, arr[k].c = op, col, c
        return arr

    ok = prog([(abi.X_COL, 0, 0.0), (abi.X_EXP, -1, 0.0)])
    o.assign_expr(out, ok, [2])
    for bad, lens in (([(abi.X_ADD, -1, 0.0)], [1]),                                   # underflow
                      ([(abi.X_CONST, -1, 1.0), (abi.X_CONST, -1, 2.0)], [2]),          # two values left
                      ([(99, -1, 0.0)], [1]),                                          # unknown op
                      ([(abi.X_COL, 0, 0.0), (abi.X_POWI, -1, 0.5)], [2]),              # fractional POWI
                      ([(abi.X_CONST, -1, 1.0)] * 9 + [(abi.X_ADD, -1, 0.0)] * 8, [17])):  # stack > 8
        with pytest.raises(RuntimeError):
            o.assign_expr(out, prog(bad), lens)


def test_lowering_orders_commutative_operands_by_depth():
    # a right-deep sum of 12 columns needs 12 values left to right; swapping the commutative
    # operands (a + b == b + a bit for bit) evaluates it in 2
    names = [chr(ord("a") + k) for k in range(12)]
    e = Fx.lift(Col(names[-1]))
    for n in reversed(names[:-1]):
        e = Fx.lift(Col(n)) + e
    assert e._need() == 2
    prog, lens = dsl.xprogram([e], {n: k for k, n in enumerate(names)}.__getitem__)
    assert lens == [23]
    # a division chain cannot be reordered: too deep is refused on the host
    d = Fx.lift(Col("a"))
    for n in names[1:10]:
        d = Fx.lift(Col(n)) / d
    with pytest.raises(ValueError):
        dsl.xprogram([d], {n: k for k, n in enumerate(names)}.__getitem__)


def test_affine_stays_an_operand_and_general_forms_are_refused_in_distributions():
    e = 2.0 * Col("x") + Col("y")
    assert isinstance(e, dsl.Expr)
    assert not dsl.is_general(e)
    assert dsl.is_general(Col("x") * Col("y"))
    assert dsl.is_general([1.0, exp(Col("x"))])
    assert isinstance(Col("x") + Col("y") + Col("z"), Fx)   # three terms: beyond the operand form
    with pytest.raises(TypeError):
        dsl.Normal(Col("x") * Col("y"), 1.0).dist(lambda n: 0)
    with pytest.raises(TypeError):
        bool(Col("x") < 1.0)


def test_fire_alarm_probabilities_as_expressions():
    """examples/fire_alarm.jl's argument expressions: `fire ? 0.9 : 0.01` and
    `smoke || lever ? 0.98 : 0.01` as Assign programs over 0/1 columns"""
    o = Oracle(8, seed=1)
    bits = np.array([[f, s, l] for f in (0, 1) for s in (0, 1) for l in (0, 1)], dtype=float).T
    for k, n in enumerate(("fire", "smoke", "lever")):
        o.col_upload(o.col_create(n), bits[k])
    p = run(o, ifelse(Col("fire"), 0.9, 0.01), "p_smoke")
    np.testing.assert_array_equal(p, np.where(bits[0] == 1, 0.9, 0.01))
    q = run(o, ifelse(or_(Col("smoke"), Col("lever")), 0.98, 0.01), "p_alarm")
    np.testing.assert_array_equal(q, np.where((bits[1] == 1) | (bits[2] == 1), 0.98, 0.01))
    r = run(o, and_(Col("fire"), not_(Col("smoke"))), "fire_no_smoke")
    np.testing.assert_array_equal(r, (bits[0] == 1) & (bits[1] == 0))
    t = run(o, ne(Col("fire"), Col("smoke")), "xor")
    np.testing.assert_array_equal(t, bits[0] != bits[1])


def test_julia_pow_huge_and_edge_exponents():
    """Base.^(::Float64, ::Float64) clamps |y| to 1.5 2^62 before its integer test,
    so a negative base to a huge even exponent is the integer power (Inf / 0), not NaN; 0^y and
    Inf^y go by the sign of y (Julia 1.10 values, restated in include/wsmc_math.h wsmc_pow)."""
    o = Oracle(12, seed=1)
    a = np.array([-2.0, -2.0, -0.5, 2.0, 0.5, 0.0, 0.0, np.inf, np.inf, -np.inf, np.nan, -3.0])
    b = np.array([1e19, -1e19, 1e300, np.inf, np.inf, 0.5, -0.5, 0.5, -0.5, 1e19, 2.5, 2.5])
    o.col_upload(o.col_create("a"), a)
    o.col_upload(o.col_create("b"), b)
    p = run(o, Col("a") ** Col("b"), "p")
    assert p[0] == np.inf and p[1] == 0.0      # (-2.0)^1e19 = Inf, (-2.0)^-1e19 = 0.0
    assert p[2] == 0.0                         # (-0.5)^1e300 = 0.0
    assert p[3] == np.inf and p[4] == 0.0      # 2^Inf = Inf, 0.5^Inf = 0
    assert p[5] == 0.0 and p[6] == np.inf      # 0^0.5 = 0, 0^-0.5 = Inf
    assert p[7] == np.inf and p[8] == 0.0      # Inf^0.5 = Inf, Inf^-0.5 = 0
    assert p[9] == np.inf                      # (-Inf)^1e19: an even integer power
    assert np.isnan(p[10]) and np.isnan(p[11])  # NaN^2.5; (-3)^2.5 is Julia's DomainError


def test_affine_constant_keeps_the_operation_order():
    """an affine Expr that enters a program sums as ((c0 + t0) + t1) + ..., the order
    wsmc_operand_eval uses and, c0 + x being x + c0 exactly, Julia's ((x + 1) + y) + z."""
    rng = np.random.default_rng(4)
    n = 4096
    x, y, z = (rng.normal(0, 1, n) * 10.0 ** rng.integers(-8, 8, n) for _ in range(3))
    o = Oracle(n, seed=1)
    for name, v in (("x", x), ("y", y), ("z", z)):
        o.col_upload(o.col_create(name), v)
    got = run(o, Col("x") + 1.0 + Col("y") + Col("z"), "s")
    assert (got.view(np.uint64) == (((x + 1.0) + y) + z).view(np.uint64)).all()
    # two terms stay an operand; the same value through a program (a no-op max with itself)
    two = run(o, Col("x") * 3.0 + 1.5 + Col("y"), "t2")
    prog = run(o, max_(Col("x") * 3.0 + 1.5 + Col("y"), Col("x") * 3.0 + 1.5 + Col("y")), "t3")
    assert (two.view(np.uint64) == prog.view(np.uint64)).all()
    assert (two.view(np.uint64) == ((1.5 + 3.0 * x) + y).view(np.uint64)).all()
