"""Lazy genealogy of the generic store ("Lazy genealogy"): a Resample logs its
ancestors and gathers only the columns touched since the previous Resample; history columns
are brought up to date by one trace over the log when read. The reference gathers every
column at every resample (src/stores.jl:105-128); the values must be identical — checked
against the eager device store and the CPU oracle (whose store is the reference's eager
ColumnStore), bit for bit."""
import numpy as np
import pytest

import wsmc
from wsmc import abi, models
from oracle import Oracle
from test_gpu_parity import assert_same_state

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("scheme", [abi.RESAMPLE_STRATIFIED, abi.RESAMPLE_MULTINOMIAL])
@pytest.mark.parametrize("wait", [True, False])
def test_lazy_history_matches_oracle(gpu_available, scheme, wait):
    """C2's statements over T = 150 steps (> one trace launch's 96 log entries): the history
    columns x_1..x_T stay behind the log until downloaded, then match the eager oracle."""
    N, T = 3001, 150
    obs = models.ssm2d_data(T)
    g, o = wsmc.Context(N, seed=5), Oracle(N, seed=5)
    models.ssm2d_statements(g, obs, ess_perc_min=1.0, scheme=scheme, wait=wait)
    models.ssm2d_statements(o, obs, ess_perc_min=1.0, scheme=scheme)
    info = g.store_info()
    assert info["stale_columns"] >= T - 2          # x_1 .. x_{T-1}: left behind, never gathered
    assert T - 2 <= info["log_entries"] <= T + 1   # one ancestor row per resampling step
    np.testing.assert_array_equal(g.last_ancestors(), o.last_ancestors())
    assert_same_state(g, o)                        # downloads every column: one trace
    assert g.store_info()["stale_columns"] == 0
    assert g.log_evidence() == o.log_evidence()


def test_lazy_equals_eager_device_store(gpu_available):
    """The same run on a lazy and an eager (WSMC eager gathers) device store, bit for bit, at
    the example default ess 0.5 (some steps do not resample: gated identity entries)."""
    N, T = 5001, 40
    obs = models.ssm2d_data(T)
    a, b = wsmc.Context(N, seed=11), wsmc.Context(N, seed=11)
    b.store_set_lazy(False)
    models.ssm2d_statements(a, obs, ess_perc_min=0.5, wait=False)
    models.ssm2d_statements(b, obs, ess_perc_min=0.5, wait=False)
    assert b.store_info() == {"log_entries": 0, "stale_columns": 0}
    assert_same_state(a, b)


def test_lazy_log_stays_short_without_history(gpu_available):
    """The LGSSM rebinds one column, read at every step: it is never more than one entry behind,
    so the log keeps at most the newest row however long the run."""
    data = models.lgssm1d_data(60)
    g, o = wsmc.Context(2049, seed=3), Oracle(2049, seed=3)
    models.lgssm1d_statements(g, data, ess_perc_min=1.0, wait=False)
    models.lgssm1d_statements(o, data, ess_perc_min=1.0)
    assert g.store_info()["stale_columns"] <= 1    # x, one entry behind the last Resample
    g.get_state()                                   # folds the pending decisions in
    assert g.store_info()["log_entries"] <= 1
    assert_same_state(g, o)
    np.testing.assert_array_equal(g.last_ancestors(), o.last_ancestors())


def test_lazy_switch_to_eager_midrun(gpu_available):
    """Turning the lazy store off mid-run brings every column up to date first."""
    N = 2500
    obs = models.ssm2d_data(30)
    g, o = wsmc.Context(N, seed=9), Oracle(N, seed=9)
    models.ssm2d_statements(g, obs[:15], ess_perc_min=1.0)
    models.ssm2d_statements(o, obs[:15], ess_perc_min=1.0)
    assert g.store_info()["stale_columns"] > 0
    g.store_set_lazy(False)
    info = g.store_info()
    assert info["stale_columns"] == 0 and info["log_entries"] <= 1   # the newest row: last_ancestors
    assert_same_state(g, o)


def test_lazy_explicit_store_resample(gpu_available):
    """resample!(store, idx) with caller indices is logged like a Resample: a column the
    operators stopped touching picks it up when read."""
    N = 1000
    rng = np.random.default_rng(1)
    g, o = wsmc.Context(N, seed=2), Oracle(N, seed=2)
    for ctx in (g, o):
        a = ctx.col_create("a", 1)
        ctx.col_upload(a, np.arange(N, dtype=float))
        b = ctx.col_create("b", 2)
        ctx.col_upload(b, np.arange(2 * N, dtype=float) * 0.5)
    idx1 = rng.integers(0, N, N).astype(np.int32)
    idx2 = np.sort(rng.integers(0, N, N)).astype(np.int32)
    for ctx in (g, o):
        ctx.store_resample(idx1)                   # both left behind (one log entry)
        ctx.col_upload(ctx.col_find("b"), np.ones(2 * N))   # b rewritten: current again
        ctx.store_resample(idx2)                   # a two entries behind, b one
    assert g.store_info()["stale_columns"] == 2
    assert_same_state(g, o)
    np.testing.assert_array_equal(g.last_ancestors(), idx2)   # the last resample!'s indices


def _last_anc_program(c, switch, wait):
    """Resamples that do and do not resample around a store-mode switch. After a Resample
    the weights are equal; an Observe with no particle operand keeps them equal (exact ESS
    1), so the next Resample at 1.0 does not resample (strict <, src/transformers.jl:484)."""
    from wsmc.dsl import Normal
    R = models.resolver(c)
    a = c.col_create("a")
    c.sample(a, Normal(0.0, 1.0).dist(R))
    flags = []

    def step(y):   # varied weights: resamples
        c.observe(Normal(wsmc.Col("a"), 0.5).dist(R), models._const([y]))
        flags.append(c.resample(1.0, wait=wait))

    def flat():    # equal weights stay equal: no resample
        c.observe(Normal(0.0, 1.0).dist(R), models._const([0.3]))
        flags.append(c.resample(1.0, wait=wait))

    step(0.2)
    flat()
    switch(c)
    mid = c.last_ancestors()
    step(-0.1)
    flat()
    flat()
    return flags, mid


def _one_rank_exact(c):
    c.comm_init_host(lambda raw: [raw], 1, 0, 0, c.n)   # one rank: the all-gather is the identity
    c.comm_set_shard_mode(abi.SHARD_EXACT)


@pytest.mark.parametrize("switch", ["none", "eager", "eager_from_start", "exact", "store_resample"])
@pytest.mark.parametrize("wait", [True, False])
def test_last_ancestors_across_store_modes(gpu_available, switch, wait):
    """last_ancestors() is the newest Resample that resampled (the oracle's last_anc), also
    when the store turns eager or exact mid-run with asynchronous decisions still pending, when
    later Resamples do not resample, and when resample!(store, idx) follows pending ones."""
    N = 3000
    idx = np.arange(N, dtype=np.int32)[::-1].copy()
    sw = {
        "none": lambda c: None,
        "eager": lambda c: c.store_set_lazy(False),
        "eager_from_start": lambda c: None,
        "exact": _one_rank_exact,
        "store_resample": lambda c: c.store_resample(idx),
    }[switch]
    g, o = wsmc.Context(N, seed=17), Oracle(N, seed=17)
    if switch == "eager_from_start":
        g.store_set_lazy(False)
    _, mid_g = _last_anc_program(g, sw, wait)
    _, mid_o = _last_anc_program(o, (lambda c: c.store_resample(idx)) if switch == "store_resample"
                                 else (lambda c: None), True)
    np.testing.assert_array_equal(mid_g, mid_o)
    st = g.get_state()
    assert st["n_resamples"] == o.get_state()["n_resamples"]
    np.testing.assert_array_equal(g.last_ancestors(), o.last_ancestors())
    assert_same_state(g, o)


@pytest.mark.parametrize("ess", [1.0, 0.6])
def test_statement_batch_hazards(gpu_available, ess):
    """Statement batches (one kernel per run of Assign / Sample / Observe / Weight calls) against
    the oracle's one-statement-at-a-time path, bit for bit, over the cases the batch must get
    right: an Assign reading columns one Resample behind (through the ancestors) followed by an
    in-place Sample of one of them (the batch must end first), a weight term reading what a
    Sample of the same batch wrote (its LDS row), an Assign that reads its own output behind
    (a fresh buffer), two weight terms in one batch (the weight register), a 2-component
    column read by component, more statements than a batch holds, and a no-op Resample in the
    middle (the batch stays open)."""
    from wsmc.dsl import Col, MvNormal, Normal
    N = 3001
    res = []
    for ctx in (wsmc.Context(N, seed=5), Oracle(N, seed=5)):
        R = models.resolver(ctx)
        ca = ctx.col_create("a", 1)
        cb = ctx.col_create("b", 2)
        cc = ctx.col_create("c", 1)
        cd = ctx.col_create("d", 1)
        ctx.sample(ca, Normal(0.0, 1.0).dist(R))
        ctx.sample(cb, MvNormal([0.0, 0.0], np.eye(2)).dist(R))
        for t in range(6):
            ctx.assign(cc, models.value_operands(Col("a") + Col("b", 1) * 0.5, 1, R))   # a, b behind
            ctx.resample(ess, wait=False)                                               # a no-op: weights unchanged
            ctx.sample(ca, Normal(Col("c"), 1.0).dist(R))                              # a in place
            ctx.observe(Normal(Col("a"), 1.0).dist(R), models._const([0.1 * t]))       # a from the batch
            if t % 2:
                ctx.resample(ess, wait=False)                                           # a Resample mid-step
            ctx.assign(cb, models.value_operands([Col("b", 0) + Col("a"), Col("b", 1) - Col("c")], 2, R))
            ctx.weight(Normal(Col("b", 1), 2.0).dist(R), models._const([0.3]))        # b's new buffer
            ctx.assign(cd, models.value_operands(Col("c") * 2.0 + Col("d"), 1, R))
            ctx.assign(cc, models.value_operands(Col("d") - Col("a"), 1, R))           # a seventh statement
            ctx.resample(ess, wait=False)
        res.append(ctx)
    g, o = res
    assert_same_state(g, o)
    assert g.log_evidence() == o.log_evidence()
