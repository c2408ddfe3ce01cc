"""World-2 device path on one GPU: two processes, each a shard (HIP context) of one
population, exchanging their shard records through the host (wsmc_comm_init_host) instead
of RCCL — RCCL refuses two ranks on one device, and the box has one. Everything else on
the device is the multi-GPU path: per-shard records, rank-order global decision, island
resampling, shard log-mean reset, record-combined evidence. Results must equal the
single-process sharded oracle bit for bit."""
import os
import pathlib
import socket
import sys

import numpy as np
import pytest

REPO = pathlib.Path(__file__).resolve().parents[1]
pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, N, T, ess, scheme, outdir):
    sys.path[:0] = [str(REPO / "weightedsampling.jl_amd")]
    import wsmc
    from wsmc.hostcomm import HostComm
    comm = HostComm(rank, world, "127.0.0.1", port, tag="ms", timeout=120)
    n = N // world
    obs2 = wsmc.models.ssm2d_data(T)
    out = {}
    # statement-by-statement (generic operators)
    c = wsmc.Context(n, seed=21, device=0)
    c.comm_init_host(comm.allgather, world, rank, rank * n, N)
    flags = wsmc.models.ssm2d_statements(c, obs2, ess_perc_min=ess, scheme=scheme)
    out["flags"] = np.array(flags)
    out["w"] = c.weights_download()
    out["ev"] = np.array([c.log_evidence()])
    for name in c.col_names():
        out["s_" + name] = c.col_download(c.col_find(name))
    c.close()
    # fused run
    f = wsmc.Context(n, seed=21, device=0)
    f.comm_init_host(comm.allgather, world, rank, rank * n, N)
    out["fev"] = np.array([f.ssm2d_run(obs2, ess_perc_min=ess, scheme=scheme, keep_history=True)])
    out["fw"] = f.weights_download()
    for name in f.col_names():
        out["f_" + name] = f.col_download(f.col_find(name))
    f.close()
    comm.barrier()
    comm.close()
    np.savez(os.path.join(outdir, f"rank{rank}.npz"), **out)


@pytest.mark.parametrize("N,ess,scheme", [(4096, 1.0, 0), (4096, 0.5, 1), (4096, 1.0, 2), (140002, 1.0, 0),
                                          (140002, 0.5, 0)])
def test_two_shards_one_gpu_match_sharded_oracle(gpu_available, tmp_path, N, ess, scheme):
    import multiprocessing as mp
    sys.path.insert(0, str(REPO / "oracle"))
    from oracle import Oracle
    import wsmc
    T, world = 10, 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    ps = [ctx.Process(target=_worker, args=(r, world, port, N, T, ess, scheme, str(tmp_path))) for r in range(world)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(300)
    codes = [p.exitcode for p in ps]
    for p in ps:
        if p.is_alive():
            p.kill()
    assert codes == [0] * world, codes
    ref = Oracle(N, seed=21, shards=world)
    flags = wsmc.models.ssm2d_statements(ref, wsmc.models.ssm2d_data(T), ess_perc_min=ess, scheme=scheme)
    n = N // world
    for r in range(world):
        p = np.load(tmp_path / f"rank{r}.npz")
        sl = slice(r * n, (r + 1) * n)
        assert list(p["flags"]) == flags
        np.testing.assert_array_equal(p["w"], ref.weights_download()[sl])
        np.testing.assert_array_equal(p["fw"], ref.weights_download()[sl])
        for name in ref.col_names():
            full = ref.col_download(ref.col_find(name))
            np.testing.assert_array_equal(p["s_" + name], full[..., sl], err_msg=name)
            np.testing.assert_array_equal(p["f_" + name], full[..., sl], err_msg=name)
        assert p["ev"][0] == ref.log_evidence()
        assert p["fev"][0] == ref.log_evidence()



def _move_program(ctx, which):
    import wsmc
    if which == "c3":
        xs, ys = wsmc.models.linreg_data()
        return wsmc.models.linreg_statements(ctx, xs[:6], ys[:6], ess_perc_min=1.0)
    if which == "c5g":   # the example's gated moves (ess 0.5): the population-wide unique count;
        t, y = wsmc.models.oscillator_data(n=8)          # at 0.7 the gate both skips and runs
        return wsmc.models.oscillator_statements(ctx, t, y, ess_perc_min=0.5, sweeps=2, diversity=0.7)
    t, y = wsmc.models.oscillator_data(n=5)
    return wsmc.models.oscillator_statements(ctx, t, y, ess_perc_min=1.0, scheme=wsmc.RESAMPLE_SYSTEMATIC,
                                             sweeps=2, diversity=None)


def _move_worker(rank, world, port, N, which, outdir, exact=False):
    sys.path[:0] = [str(REPO / "weightedsampling.jl_amd")]
    import wsmc
    from wsmc import abi
    from wsmc.hostcomm import HostComm
    comm = HostComm(rank, world, "127.0.0.1", port, tag="mv", timeout=120)
    n = N // world
    c = wsmc.Context(n, seed=33, device=0)
    c.comm_init_host(comm.allgather, world, rank, rank * n, N)
    if exact:
        c.comm_set_shard_mode(abi.SHARD_EXACT)
    acc = _move_program(c, which)
    out = {"acc": np.array(acc), "w": c.weights_download(), "ev": np.array([c.log_evidence()])}
    for name in c.col_names():
        out["c_" + name] = c.col_download(c.col_find(name))
    c.close()
    comm.barrier()
    comm.close()
    np.savez(os.path.join(outdir, f"mv{rank}.npz"), **out)


@pytest.mark.parametrize("exact", [False, True])
@pytest.mark.parametrize("which", ["c3", "c5", "c5g"])
def test_two_shards_moves_match_sharded_oracle(gpu_available, tmp_path, which, exact):
    """Sharded autoRW: global max, per-rank canonical moment totals combined in rank order;
    with exact sharding the Resamples are population-wide (the oracle's exact flag)."""
    import multiprocessing as mp
    sys.path.insert(0, str(REPO / "oracle"))
    from oracle import Oracle
    import wsmc
    N, world = 6002, 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    ps = [ctx.Process(target=_move_worker, args=(r, world, port, N, which, str(tmp_path), exact))
          for r in range(world)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(300)
    codes = [p.exitcode for p in ps]
    for p in ps:
        if p.is_alive():
            p.kill()
    assert codes == [0] * world, codes
    ref = Oracle(N, seed=33, shards=world, exact=exact)
    acc = _move_program(ref, which)
    n = N // world
    parts = [np.load(tmp_path / f"mv{r}.npz") for r in range(world)]
    # accepted counts are per shard; their sum is the single-process count
    np.testing.assert_array_equal(sum(p["acc"] for p in parts), np.array(acc))
    for r, p in enumerate(parts):
        sl = slice(r * n, (r + 1) * n)
        np.testing.assert_array_equal(p["w"], ref.weights_download()[sl])
        for name in ref.col_names():
            np.testing.assert_array_equal(p["c_" + name], ref.col_download(ref.col_find(name))[..., sl], err_msg=name)
        assert p["ev"][0] == ref.log_evidence()


# ---- exact sharding: the shards together give the single-context bits ---------------------
def _exact_worker(rank, world, port, sizes, T, ess, scheme, outdir):
    sys.path[:0] = [str(REPO / "weightedsampling.jl_amd")]
    import wsmc
    from wsmc import abi
    from wsmc.hostcomm import HostComm
    comm = HostComm(rank, world, "127.0.0.1", port, tag="ex", timeout=120)
    n, goff, N = sizes[rank], sum(sizes[:rank]), sum(sizes)
    c = wsmc.Context(n, seed=21, device=0)
    c.comm_init_host(comm.allgather, world, rank, goff, N)
    c.comm_set_shard_mode(abi.SHARD_EXACT)
    flags = wsmc.models.ssm2d_statements(c, wsmc.models.ssm2d_data(T), ess_perc_min=ess, scheme=scheme)
    out = {"flags": np.array(flags), "w": c.weights_download(), "anc": c.last_ancestors(),
           "ev": np.array([c.log_evidence()]), "ess": np.array([c.ess()])}
    for name in c.col_names():
        out["s_" + name] = c.col_download(c.col_find(name))
    # what exact shards refuse rather than silently doing island work
    refused = []
    try:
        c.resample(2.0, abi.RESAMPLE_MULTINOMIAL)
    except wsmc.WSMCError:
        refused.append("multinomial")
    try:
        c.ssm2d_run(wsmc.models.ssm2d_data(2), ess_perc_min=ess, scheme=abi.RESAMPLE_MULTINOMIAL)
    except wsmc.WSMCError:
        refused.append("fused multinomial")
    out["refused"] = np.array(refused)
    c.close()
    # the fused run on exact shards: the same bits (history traced back across ranks)
    for keep in (True, False):
        f = wsmc.Context(n, seed=21, device=0)
        f.comm_init_host(comm.allgather, world, rank, goff, N)
        f.comm_set_shard_mode(abi.SHARD_EXACT)
        tag = "fk" if keep else "fn"
        out[tag + "ev"] = np.array([f.ssm2d_run(wsmc.models.ssm2d_data(T), ess_perc_min=ess, scheme=scheme,
                                                keep_history=keep)])
        out[tag + "w"] = f.weights_download()
        out[tag + "anc"] = f.last_ancestors()
        for name in f.col_names():
            out[tag + "_" + name] = f.col_download(f.col_find(name))
        f.close()
    comm.barrier()
    comm.close()
    np.savez(os.path.join(outdir, f"ex{rank}.npz"), **out)


@pytest.mark.parametrize("sizes,ess,scheme", [((2048, 2048), 1.0, 0), ((2048, 2048), 0.5, 1),
                                              ((3000, 1096), 1.0, 0), ((70001, 70001), 1.0, 0),
                                              ((70001, 70001), 0.5, 1), ((1, 1), 1.0, 0), ((1, 2, 1), 1.0, 1)])
def test_exact_shards_match_single_context_oracle(gpu_available, tmp_path, sizes, ess, scheme):
    """WSMC_SHARD_EXACT: two shards (one ragged layout) == the unsharded oracle: flags,
    weights, every column, global ancestor indices, log-evidence and ESS, bit for bit."""
    import multiprocessing as mp
    sys.path.insert(0, str(REPO / "oracle"))
    from oracle import Oracle
    import wsmc
    T, world = 8, len(sizes)
    port = _free_port()
    ctx = mp.get_context("spawn")
    ps = [ctx.Process(target=_exact_worker, args=(r, world, port, sizes, T, ess, scheme, str(tmp_path)))
          for r in range(world)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(300)
    codes = [p.exitcode for p in ps]
    for p in ps:
        if p.is_alive():
            p.kill()
    assert codes == [0] * world, codes
    N = sum(sizes)
    ref = Oracle(N, seed=21)
    flags = wsmc.models.ssm2d_statements(ref, wsmc.models.ssm2d_data(T), ess_perc_min=ess, scheme=scheme)
    for r in range(world):
        p = np.load(tmp_path / f"ex{r}.npz")
        sl = slice(sum(sizes[:r]), sum(sizes[:r + 1]))
        assert list(p["flags"]) == flags
        np.testing.assert_array_equal(p["w"], ref.weights_download()[sl])
        np.testing.assert_array_equal(p["anc"], ref.last_ancestors()[sl])
        for name in ref.col_names():
            np.testing.assert_array_equal(p["s_" + name], ref.col_download(ref.col_find(name))[..., sl],
                                          err_msg=name)
        assert p["ev"][0] == ref.log_evidence()
        assert p["ess"][0] == ref.ess()
        assert list(p["refused"]) == ["multinomial", "fused multinomial"]
        for tag in ("fk", "fn"):
            assert p[tag + "ev"][0] == ref.log_evidence(), tag
            np.testing.assert_array_equal(p[tag + "w"], ref.weights_download()[sl])
            np.testing.assert_array_equal(p[tag + "anc"], ref.last_ancestors()[sl])
            for name in ("v", "dv"):
                np.testing.assert_array_equal(p[tag + "_" + name], ref.col_download(ref.col_find(name))[..., sl],
                                              err_msg=tag + name)
        for name in ref.col_names():                       # the traced-back history
            np.testing.assert_array_equal(p["fk_" + name], ref.col_download(ref.col_find(name))[..., sl],
                                          err_msg=name)
        np.testing.assert_array_equal(p["fn_x"], ref.col_download(ref.col_find(f"x_{T + 1}"))[..., sl])


def _exact_skew_worker(rank, world, port, sizes, kind, outdir):
    sys.path[:0] = [str(REPO / "weightedsampling.jl_amd")]
    import wsmc
    from wsmc import abi
    from wsmc.dsl import Normal
    from wsmc.hostcomm import HostComm
    comm = HostComm(rank, world, "127.0.0.1", port, tag="xs", timeout=120)
    n, goff, N = sizes[rank], sum(sizes[:rank]), sum(sizes)
    c = wsmc.Context(n, seed=8, device=0)
    c.comm_init_host(comm.allgather, world, rank, goff, N)
    c.comm_set_shard_mode(abi.SHARD_EXACT)
    w = _skew(kind, N)[goff:goff + n]
    cx = c.col_create("x")
    c.col_upload(cx, np.arange(goff, goff + n, dtype=float))
    c.weights_upload(w)
    c.weight(Normal(0.0, 1.0).dist(c.col_find), [abi.Operand.const(0.0)])
    rs, ess = c.resample(2.0, abi.RESAMPLE_STRATIFIED)
    out = {"rs": np.array([rs, ess]), "w": c.weights_download(), "anc": c.last_ancestors(),
           "x": c.col_download(cx), "ev": np.array([c.log_evidence()])}
    c.close()
    comm.barrier()
    comm.close()
    np.savez(os.path.join(outdir, f"xs{rank}.npz"), **out)


def _skew(kind, N):
    w = np.full(N, -np.inf)
    if kind == "last_shard":          # every slot's ancestor lives on the last rank
        w[N - 50:] = np.linspace(-1.0, 0.0, 50)
    elif kind == "one_particle":      # one dominant particle on rank 0
        w[:] = -200.0
        w[7] = 0.0
    else:                             # alternating mass: many short windows
        w[::3] = 0.0
    return w


@pytest.mark.parametrize("kind", ["last_shard", "one_particle", "alternating"])
def test_exact_shards_skewed_windows(gpu_available, tmp_path, kind):
    """Exact sharding with all weight on one shard (full migration, empty windows) or one
    particle: the unsharded oracle's ancestors, columns, weights and evidence."""
    import multiprocessing as mp
    sys.path.insert(0, str(REPO / "oracle"))
    from oracle import Oracle
    from wsmc import abi
    from wsmc.dsl import Normal
    sizes = (3000, 1096, 2001)
    port = _free_port()
    ctx = mp.get_context("spawn")
    ps = [ctx.Process(target=_exact_skew_worker, args=(r, len(sizes), port, sizes, kind, str(tmp_path)))
          for r in range(len(sizes))]
    for p in ps:
        p.start()
    for p in ps:
        p.join(300)
    codes = [p.exitcode for p in ps]
    for p in ps:
        if p.is_alive():
            p.kill()
    assert codes == [0] * len(sizes), codes
    N = sum(sizes)
    o = Oracle(N, seed=8)
    cx = o.col_create("x")
    o.col_upload(cx, np.arange(N, dtype=float))
    o.weights_upload(_skew(kind, N))
    o.weight(Normal(0.0, 1.0).dist(o.col_find), [abi.Operand.const(0.0)])
    rs, ess = o.resample(2.0, abi.RESAMPLE_STRATIFIED)
    for r in range(len(sizes)):
        p = np.load(tmp_path / f"xs{r}.npz")
        sl = slice(sum(sizes[:r]), sum(sizes[:r + 1]))
        assert bool(p["rs"][0]) == rs and p["rs"][1] == ess
        np.testing.assert_array_equal(p["anc"], o.last_ancestors()[sl])
        np.testing.assert_array_equal(p["x"], o.col_download(cx)[sl])
        np.testing.assert_array_equal(p["w"], o.weights_download()[sl])
        assert p["ev"][0] == o.log_evidence()


def _rccl1_worker(mode, outdir):
    """One process, a one-rank RCCL communicator: every exchange of the sharded paths goes
    through ncclAllGather / ncclSend / ncclRecv for real (with one rank), and one shard is
    the whole population, so the results must equal the unsharded oracle."""
    os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")     # the rendezvous of a lone rank
    sys.path[:0] = [str(REPO / "weightedsampling.jl_amd")]
    import wsmc
    from wsmc import abi
    N, T = 5001, 12
    obs2 = wsmc.models.ssm2d_data(T)
    out = {}

    def ctx(seed):
        c = wsmc.Context(N, seed=seed, device=0)
        c.comm_init(wsmc.Context.comm_unique_id(), 1, 0, 0, N)   # a fresh rendezvous per communicator
        if mode == "exact":
            c.comm_set_shard_mode(abi.SHARD_EXACT)
        return c
    c = ctx(21)                                           # statements
    out["flags"] = np.array(wsmc.models.ssm2d_statements(c, obs2, ess_perc_min=0.5))
    out["w"] = c.weights_download()
    out["ev"] = np.array([c.log_evidence()])
    for name in c.col_names():
        out["s_" + name] = c.col_download(c.col_find(name))
    c.close()
    f = ctx(22)                                           # the fused run
    out["fev"] = np.array([f.ssm2d_run(obs2, ess_perc_min=1.0, keep_history=True)])
    out["fw"] = f.weights_download()
    for name in f.col_names():
        out["f_" + name] = f.col_download(f.col_find(name))
    f.close()
    m = ctx(23)                                           # autoRW moves (moment exchange)
    xs, ys = wsmc.models.linreg_data()
    out["acc"] = np.array(wsmc.models.linreg_statements(m, xs[:6], ys[:6], ess_perc_min=1.0))
    out["mw"] = m.weights_download()
    for name in m.col_names():
        out["m_" + name] = m.col_download(m.col_find(name))
    m.close()
    g = ctx(24)                                           # diversity-gated moves (global_unique)
    out["gacc"] = np.array(_move_program(g, "c5g"))
    for name in g.col_names():
        out["g_" + name] = g.col_download(g.col_find(name))
    g.close()
    np.savez(os.path.join(outdir, f"rccl1_{mode}.npz"), **out)


@pytest.mark.parametrize("mode", ["island", "exact"])
def test_one_rank_rccl_matches_unsharded_oracle(gpu_available, tmp_path, mode):
    """The RCCL calls of the multi-GPU path on the box's one GPU (a one-rank communicator)."""
    import multiprocessing as mp
    sys.path.insert(0, str(REPO / "oracle"))
    from oracle import Oracle
    import wsmc
    p = mp.get_context("spawn").Process(target=_rccl1_worker, args=(mode, str(tmp_path)))
    p.start()
    p.join(100)
    if p.is_alive():
        p.kill()
    assert p.exitcode == 0, p.exitcode
    r = np.load(tmp_path / f"rccl1_{mode}.npz")
    N, T = 5001, 12
    obs2 = wsmc.models.ssm2d_data(T)
    o = Oracle(N, seed=21)
    assert list(r["flags"]) == wsmc.models.ssm2d_statements(o, obs2, ess_perc_min=0.5)
    np.testing.assert_array_equal(r["w"], o.weights_download())
    for name in o.col_names():
        np.testing.assert_array_equal(r["s_" + name], o.col_download(o.col_find(name)), err_msg=name)
    assert r["ev"][0] == o.log_evidence()
    o = Oracle(N, seed=22)
    wsmc.models.ssm2d_statements(o, obs2, ess_perc_min=1.0)
    np.testing.assert_array_equal(r["fw"], o.weights_download())
    for name in o.col_names():
        np.testing.assert_array_equal(r["f_" + name], o.col_download(o.col_find(name)), err_msg=name)
    assert r["fev"][0] == o.log_evidence()
    o = Oracle(N, seed=23)
    xs, ys = wsmc.models.linreg_data()
    assert [tuple(a) for a in r["acc"]] == wsmc.models.linreg_statements(o, xs[:6], ys[:6], ess_perc_min=1.0)
    np.testing.assert_array_equal(r["mw"], o.weights_download())
    for name in o.col_names():
        np.testing.assert_array_equal(r["m_" + name], o.col_download(o.col_find(name)), err_msg=name)
    o = Oracle(N, seed=24)
    assert [tuple(a) for a in r["gacc"]] == _move_program(o, "c5g")
    for name in o.col_names():
        np.testing.assert_array_equal(r["g_" + name], o.col_download(o.col_find(name)), err_msg=name)


def _analysis_worker(rank, world, port, sizes, outdir):
    sys.path[:0] = [str(REPO / "weightedsampling.jl_amd")]
    import wsmc
    from wsmc.abi import Operand
    from wsmc.hostcomm import HostComm
    comm = HostComm(rank, world, "127.0.0.1", port, tag="an", timeout=120)
    n, goff, N = sizes[rank], sum(sizes[:rank]), sum(sizes)
    c = wsmc.Context(n, seed=44, device=0)
    c.comm_init_host(comm.allgather, world, rank, goff, N)
    xs, ys = wsmc.models.linreg_data()
    wsmc.models.linreg_statements(c, xs[:5], ys[:5], ess_perc_min=0.3)
    a, b = c.col_find("α"), c.col_find("β")
    mean, cov = c.weighted_moments([Operand.column(a), Operand.column(b, coef=2.0, c0=1.0)])
    out = {"mean": np.asarray(mean), "cov": np.asarray(cov), "ess": np.array([c.ess()]),
           "ev": np.array([c.log_evidence()])}
    for k, col in (("a", a), ("b", b)):
        out["mm" + k] = np.array(c.col_minmax(col))
        out["h" + k] = c.histogram(col)
        out["md" + k] = np.array([c.weighted_median(col)])
    out["sr"] = c.sample_particles(257, replace=True)
    out["sn"] = c.sample_particles(300, replace=False)
    out["sall"] = c.sample_particles(N, replace=False)       # every particle, zero weights last
    c.close()
    comm.barrier()
    comm.close()
    np.savez(os.path.join(outdir, f"an{rank}.npz"), **out)


@pytest.mark.parametrize("sizes", [(3000, 3000), (70001, 70001)])
def test_two_shards_analysis_match_single_context(gpu_available, tmp_path, sizes):
    """describe / @E on island shards: min/max, the sparkline histogram (integer weights
    relative to the population's max: bit-identical bins), the weighted median (over the
    all-gathered (value, q) union), sample(state, n; replace) (global indices) and ESS equal
    the sharded oracle's
    population-wide values exactly; the weighted moments are rank-order combinations of
    per-shard canonical sums, equal to the population's up to summation order."""
    import multiprocessing as mp
    sys.path.insert(0, str(REPO / "oracle"))
    from oracle import Oracle
    import wsmc
    from wsmc.abi import Operand
    world = len(sizes)
    port = _free_port()
    ctx = mp.get_context("spawn")
    ps = [ctx.Process(target=_analysis_worker, args=(r, world, port, sizes, str(tmp_path))) for r in range(world)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(300)
    codes = [p.exitcode for p in ps]
    for p in ps:
        if p.is_alive():
            p.kill()
    assert codes == [0] * world, codes
    # island shards resample within themselves: the reference population is the sharded oracle's
    o = Oracle(sum(sizes), seed=44, shards=world)
    xs, ys = wsmc.models.linreg_data()
    wsmc.models.linreg_statements(o, xs[:5], ys[:5], ess_perc_min=0.3)
    a, b = o.col_find("α"), o.col_find("β")
    mean, cov = o.weighted_moments([Operand.column(a), Operand.column(b, coef=2.0, c0=1.0)])
    parts = [np.load(tmp_path / f"an{r}.npz") for r in range(world)]
    # each sample() consumes one op counter: draw in the workers' order, once
    sr = o.sample_particles(257, replace=True)
    sn = o.sample_particles(300, replace=False)
    sall = o.sample_particles(sum(sizes), replace=False)
    assert sorted(sall) == list(range(sum(sizes)))
    for p in parts:
        for k, col in (("a", a), ("b", b)):
            np.testing.assert_array_equal(p["mm" + k], np.array(o.col_minmax(col)))
            np.testing.assert_array_equal(p["h" + k], o.histogram(col))
            assert p["md" + k][0] == o.weighted_median(col)
        assert p["ess"][0] == o.ess()
        np.testing.assert_array_equal(p["sr"], sr)
        np.testing.assert_array_equal(p["sn"], sn)
        np.testing.assert_array_equal(p["sall"], sall)
        assert p["ev"][0] == o.log_evidence()
        np.testing.assert_allclose(p["mean"], mean, rtol=1e-12)
        np.testing.assert_allclose(p["cov"], cov, rtol=1e-10)


# ---- one handle over several shards (wsmc_create_multi) -------------------------------------
def _multi_program(ctx):
    import wsmc
    obs = wsmc.models.ssm2d_data(10)
    flags = wsmc.models.ssm2d_statements(ctx, obs, ess_perc_min=1.0)
    xs, ys = wsmc.models.linreg_data()
    cx = ctx.col_create("alpha", 1)
    ctx.sample(cx, wsmc.dsl.Normal(0.0, 10.0).dist(wsmc.models.resolver(ctx)))
    acc = ctx.move(wsmc.PROPOSAL_AUTORW, [cx], 1e-3)
    return flags, acc


@pytest.mark.parametrize("shards,transport,mode", [(1, 0, "island"), (1, 0, "exact"), (2, 1, "island"),
                                                   (2, 1, "exact"), (3, 1, "island")])
def test_multi_handle_matches_oracle(gpu_available, shards, transport, mode):
    """SMCState over several shards in one handle: one communicator from
    ncclCommInitAll (one shard: the RCCL exchange paths on one GPU), or two / three shards on
    the one device with the in-process exchange; every call fans out to the shards' threads.
    Island shards equal the sharded oracle; exact shards one context, bit for bit."""
    sys.path.insert(0, str(REPO / "oracle"))
    from oracle import Oracle
    import wsmc
    from wsmc import abi
    from test_gpu_parity import assert_same_state
    N = 3001
    g = wsmc.Context.multi(N, shards, seed=13, devices=[0] * shards, transport=transport)
    if mode == "exact":
        g.comm_set_shard_mode(abi.SHARD_EXACT)
    o = Oracle(N, seed=13, shards=shards, exact=(mode == "exact")) if shards > 1 else Oracle(N, seed=13)
    fg, ag = _multi_program(g)
    fo, ao = _multi_program(o)
    assert fg == fo
    assert ag == ao
    assert_same_state(g, o)
    assert g.log_evidence() == o.log_evidence()
    assert g.ess() == o.ess()
    rows = np.array([0, N - 1, N // 2, 7, N // 3 + 1])
    np.testing.assert_array_equal(g.col_gather_rows(g.col_find("v"), rows),
                                  o.col_download(o.col_find("v"))[:, rows])
    g.close()


def test_comm_info_reports_the_communicator(gpu_available):
    """wsmc_comm_info (bench.py's `ranks` object): a plain context is unsharded; a one-rank
    RCCL communicator reports ncclCommCount = 1; a multi-device handle reports its shards, their
    devices and sizes (one RCCL shard on GPU 0, and three host-exchange shards sharing it)."""
    import wsmc
    from wsmc import abi
    c = wsmc.Context(1000, seed=1)
    i = c.comm_info()
    assert (i["shards"], i["world"], i["rccl_ranks"], i["transport"]) == (1, 1, 0, "none")
    assert i["devices"] == [0] and i["shard_n"] == [1000]
    c.comm_init(wsmc.Context.comm_unique_id(), 1, 0, 0, 1000)
    i = c.comm_info()
    assert (i["world"], i["rank"], i["rccl_ranks"], i["transport"]) == (1, 0, 1, "rccl")
    c.close()
    g = wsmc.Context.multi(1001, 1, seed=1, devices=[0], transport=abi.TRANSPORT_RCCL)
    i = g.comm_info()
    assert (i["shards"], i["rccl_ranks"], i["transport"], i["devices"], i["shard_n"]) == (1, 1, "rccl", [0], [1001])
    g.close()
    g = wsmc.Context.multi(1001, 3, seed=1, devices=[0] * 3, transport=abi.TRANSPORT_HOST)
    g.comm_set_shard_mode(abi.SHARD_EXACT)
    i = g.comm_info()
    assert (i["shards"], i["world"], i["rccl_ranks"], i["transport"], i["shard_mode"]) == (3, 3, 0, "host", "exact")
    assert i["devices"] == [0, 0, 0] and i["shard_n"] == [333, 334, 334]
    g.close()


def test_one_rank_rccl_autorw_not_pd(gpu_available):
    """Sharded autoRW combines the ranks' moment totals on the device (k_autorw_combine): a
    singular covariance sets the device flag, the Move leaves the state untouched and the call
    raises PosDefException (src/move_kernels.jl:150), as on one GPU — through a one-rank RCCL
    communicator, so the sharded path runs."""
    import numpy as np
    import wsmc
    from oracle import Oracle
    from wsmc import abi, models
    from test_gpu_parity import assert_same_state, not_pd_seed, rank1_case
    N = 2048
    seed = not_pd_seed(lambda s: Oracle(N, seed=s))
    g = wsmc.Context(N, seed=seed)
    g.comm_init(wsmc.Context.comm_unique_id(), 1, 0, 0, N)
    res = []
    for c in (g, Oracle(N, seed=seed)):
        a, b = rank1_case(c)                               # b = 2a: rank-1 covariance
        with pytest.raises(np.linalg.LinAlgError):
            c.move(abi.PROPOSAL_AUTORW, [a, b], 1e-3)
        acc = c.move(abi.PROPOSAL_AUTORW, [a], 1e-3)
        res.append((c, acc))
    assert res[0][1] == res[1][1]
    assert_same_state(res[0][0], res[1][0])


@pytest.mark.parametrize("mode", ["island", "exact"])
def test_multi_handle_eight_shards_c4_partition(gpu_available, mode):
    """C4's partition through one handle: SMCState(HipColumnStore(N; gpus=8)) as
    INTEGRATION.md binds it, here 8 shards x 20k on device 0 with the in-process exchange.
    Statement path and fused run, against the eight-shard oracle (island) or the unsharded
    oracle (exact), bit for bit."""
    sys.path.insert(0, str(REPO / "oracle"))
    from oracle import Oracle
    import wsmc
    from wsmc import abi, models
    from test_gpu_parity import assert_same_state
    G, n, T = 8, 20_000, 12
    N = G * n
    obs = models.ssm2d_data(T)
    exact = mode == "exact"

    def oracle():
        return Oracle(N, seed=42, shards=G, exact=True) if exact else Oracle(N, seed=42, shards=G)

    g = wsmc.Context.multi(N, G, seed=42, devices=[0] * G, transport=abi.TRANSPORT_HOST)
    if exact:
        g.comm_set_shard_mode(abi.SHARD_EXACT)
    o = oracle()
    assert models.ssm2d_statements(g, obs, ess_perc_min=0.5) == models.ssm2d_statements(o, obs, ess_perc_min=0.5)
    assert_same_state(g, o)
    np.testing.assert_array_equal(g.last_ancestors(), o.last_ancestors())
    assert g.log_evidence() == o.log_evidence()
    g.close()

    f = wsmc.Context.multi(N, G, seed=42, devices=[0] * G, transport=abi.TRANSPORT_HOST)
    if exact:
        f.comm_set_shard_mode(abi.SHARD_EXACT)
    ev = f.ssm2d_run(obs, ess_perc_min=1.0, keep_history=True)
    o = oracle()
    models.ssm2d_statements(o, obs, ess_perc_min=1.0)
    assert_same_state(f, o)
    assert ev == o.log_evidence()
    f.close()


@pytest.mark.parametrize("transport", [0, 1])
def test_multi_handle_shard_failure_returns_error(gpu_available, transport):
    """A shard that fails mid-call must not leave the others waiting for it (in the host
    exchange or in an RCCL collective): the call returns the failing shard's error, and a
    handle whose shards diverged refuses later calls instead of hanging."""
    import wsmc
    from wsmc import abi, models
    shards = 3 if transport == abi.TRANSPORT_HOST else 1
    N = 3000
    g = wsmc.Context.multi(N, shards, seed=5, devices=[0] * shards, transport=transport)
    obs = models.ssm2d_data(4)
    models.ssm2d_statements(g, obs[:2], ess_perc_min=1.0)
    g.debug_inject_failure(shards - 1, 1)
    with pytest.raises(wsmc.WSMCError, match="injected"):
        models.ssm2d_statements(g, obs[2:], ess_perc_min=1.0)
    if shards > 1:   # the others were released by the abort: states diverged
        with pytest.raises(wsmc.WSMCError, match="failed in an earlier call"):
            g.get_state()
    else:            # one shard: nothing diverged, the handle stays usable
        g.get_state()
    g.close()


def test_multi_handle_lone_argument_error_returns_promptly(gpu_available):
    """an argument error one shard meets alone after an exchange of the call (an
    exact Resample's record exchange follows its max exchange) must not be taken for a symmetric
    error: the shard requests the abort at once — the call returns within seconds, not after the
    30 s peer wait — and the diverged handle refuses later calls."""
    import time
    import wsmc
    from wsmc import abi, models
    g = wsmc.Context.multi(3000, 3, seed=5, devices=[0] * 3, transport=abi.TRANSPORT_HOST)
    g.comm_set_shard_mode(abi.SHARD_EXACT)
    obs = models.ssm2d_data(4)
    models.ssm2d_statements(g, obs[:2], ess_perc_min=1.0)
    g.debug_inject_failure(2, 1001)
    t0 = time.perf_counter()
    with pytest.raises(wsmc.WSMCError, match="injected shard argument error"):
        models.ssm2d_statements(g, obs[2:], ess_perc_min=1.0)
    assert time.perf_counter() - t0 < 10.0
    with pytest.raises(wsmc.WSMCError, match="failed in an earlier call"):
        g.get_state()
    g.close()


@pytest.mark.parametrize("mode", ["island", "exact"])
def test_multi_handle_symmetric_errors_keep_the_handle(gpu_available, mode):
    """Errors every shard meets at the same point do not abort the handle: an
    argument error (before any exchange) and a population-wide not-positive-definite autoRW
    covariance (after the same exchanges on every shard) return the error, the shards keep
    one state, and later calls work — bit for bit against the three-shard oracle."""
    sys.path.insert(0, str(REPO / "oracle"))
    from oracle import Oracle
    import wsmc
    from wsmc import abi, models
    from test_gpu_parity import assert_same_state, not_pd_seed, rank1_case
    G, N = 3, 3000
    exact = mode == "exact"
    seed = not_pd_seed(lambda s: Oracle(N, seed=s, shards=G, exact=exact))
    g = wsmc.Context.multi(N, G, seed=seed, devices=[0] * G, transport=abi.TRANSPORT_HOST)
    if exact:
        g.comm_set_shard_mode(abi.SHARD_EXACT)
    o = Oracle(N, seed=seed, shards=G, exact=exact)
    res = []
    for c in (g, o):
        a, b = rank1_case(c)                               # b = 2a: rank-1 covariance
        with pytest.raises(np.linalg.LinAlgError):
            c.move(abi.PROPOSAL_AUTORW, [a, b], 1e-3)
        acc = c.move(abi.PROPOSAL_AUTORW, [a], 1e-3)
        res.append(acc)
    assert res[0] == res[1]
    with pytest.raises(wsmc.WSMCError):
        g.assign(999, abi.Operand.column(0))             # an unknown column on every shard
    g.get_state()                                        # still one state: the handle works
    assert_same_state(g, o)
    g.close()


@pytest.mark.parametrize("sizes", [(2600, 2600), (1700, 2101, 1500)])
@pytest.mark.parametrize("small", [False, True, "windows"])
@pytest.mark.parametrize("peer", [True, False])
def test_exact_fused_run_without_host_round_trips(gpu_available, sizes, small, peer, monkeypatch):
    """The exact-sharded fused run as it now runs: no host read inside the
    run, particles moved between neighbours through fixed-size blocks and the lineages traced
    through fixed trace windows. With the default sizes nothing overflows; with blocks and
    windows of a few slots every run overflows and is re-done on the eager path; with windows
    alone of a few ids the filter stands and only the history is traced across ranks. Shards of
    one handle that can read each other's memory (peer) trace lineages in their owners' buffers
    instead: tiny windows then cost nothing. All must equal one context holding the whole
    population, bit for bit, on ragged shards too."""
    if not peer:
        monkeypatch.setenv("WSMC_DIAG_NO_PEER", "1")
    sys.path.insert(0, str(REPO / "oracle"))
    from oracle import Oracle
    import wsmc
    from wsmc import abi, models
    from test_gpu_parity import assert_same_state
    N, T = sum(sizes), 14
    obs = models.ssm2d_data(T)
    for ess, keep in ((1.0, True), (0.5, True), (1.0, False)):
        o = Oracle(N, seed=21)
        models.ssm2d_statements(o, obs, ess_perc_min=ess)
        f = wsmc.Context.multi(N, len(sizes), seed=21, devices=[0] * len(sizes), transport=abi.TRANSPORT_HOST)
        f.comm_set_shard_mode(abi.SHARD_EXACT)
        if small == "windows":
            f.debug_exact(ctr=2)
        elif small:
            f.debug_exact(cap=3, ctr=2)
        ev = f.ssm2d_run(obs, ess_perc_min=ess, keep_history=keep)
        st = f.debug_exact()
        assert (st["eager_reruns"] >= 1) == (small is True), st
        if small == "windows" and keep:
            assert (st["history_traces"] >= 1) == (not peer), st
        assert ev == o.log_evidence()
        np.testing.assert_array_equal(f.weights_download(), o.weights_download())
        np.testing.assert_array_equal(f.last_ancestors(), o.last_ancestors())
        names = ["v", "dv"] + ([f"x_{t}" for t in range(1, T + 2)] if keep else [])
        for nm in names:
            np.testing.assert_array_equal(f.col_download(f.col_find(nm)), o.col_download(o.col_find(nm)), err_msg=nm)
        if not keep:
            np.testing.assert_array_equal(f.col_download(f.col_find("x")), o.col_download(o.col_find(f"x_{T + 1}")))
        f.close()


def test_global_population_limit(gpu_available):
    """ancestor ids are int32 and the exact fill ranks slots in 32 bits, so a sharded
    population of 2^31 particles or more is refused at the boundary (wsmc_comm_init_host /
    wsmc_comm_init / wsmc_create_multi) instead of truncating slots silently."""
    import wsmc
    from wsmc import abi
    c = wsmc.Context(1024, seed=1)
    with pytest.raises(abi.WSMCError):
        c.comm_init_host(lambda mine: [mine, mine], 2, 0, 0, 1 << 31)
    c.comm_init_host(lambda mine: [mine, mine], 2, 0, 0, 2048)   # a valid shard still initialises
    c.close()
    with pytest.raises(abi.WSMCError):
        wsmc.Context.multi(1 << 31, 2, devices=[0, 0])
