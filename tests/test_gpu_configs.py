"""The configs at their own shapes (BASELINE.json configs):

* C5 (examples/damped_oscillator.jl:20, 30-43): all 60 observations, the canonical five
  ungated sweeps of the bounded 4-D + 1-D autoRW moves, 50k particles — the longest score
  folds (5 + 60 terms per particle, twice per move) bit for bit against the oracle.
* C5 at its 4-GPU partition: four shards of 12.5k in one handle, island and exact.
* C4 (C2 sharded): eight shards on the one GPU of a test box (eight processes, records
  exchanged through the host in place of RCCL, which refuses two ranks on one device), and
  C4's own population of 8M as two shards of 4M, island and exact, T = 100, every traced-back
  column against the bit-exact CPU port (oracle/wsmc_port_mt.c: one island shard per port
  run with its global offset, or one context holding all 8M for exact shards).
"""
import os
import pathlib
import sys

import numpy as np
import pytest

REPO = pathlib.Path(__file__).resolve().parents[1]
pytestmark = pytest.mark.gpu


# ---- C5 over its full horizon --------------------------------------------------------------
@pytest.mark.parametrize("scheme", [0, 1])   # stratified (the reference's), systematic (the bench's)
def test_c5_full_horizon_matches_oracle(gpu_available, scheme):
    import wsmc
    from oracle import Oracle
    from test_gpu_parity import assert_same_state
    N = 50_000
    t, y = wsmc.models.oscillator_data(n=60)
    g, o = wsmc.Context(N, seed=4), Oracle(N, seed=4)
    ag = wsmc.models.oscillator_statements(g, t, y, ess_perc_min=1.0, scheme=scheme, sweeps=5, diversity=None)
    ao = wsmc.models.oscillator_statements(o, t, y, ess_perc_min=1.0, scheme=scheme, sweeps=5, diversity=None)
    assert len(ag) == 60 * 5
    assert ag == ao                      # accepted counts of all 600 moves
    assert_same_state(g, o)
    assert g.log_evidence() == o.log_evidence()


@pytest.mark.timeout(300)
def test_c5_per_gpu_shard_size_matches_oracle(gpu_available):
    """C5 at its per-GPU size (configs[4]: 4M particles over 4 GPUs, 1M a GPU), which no other
    test reaches: 1M particles, the first 5 observations, the canonical five
    ungated sweeps, systematic resampling — every column, weight, accepted count and the
    evidence bit for bit against the oracle (about 16 s of CPU for the oracle)."""
    import wsmc
    from oracle import Oracle
    from test_gpu_parity import assert_same_state
    N = 1_000_000
    t, y = wsmc.models.oscillator_data(n=60)
    t, y = t[:5], y[:5]
    kw = dict(ess_perc_min=1.0, scheme=1, sweeps=5, diversity=None)
    g = wsmc.Context(N, seed=42)
    ag = wsmc.models.oscillator_statements(g, t, y, **kw)
    o = Oracle(N, seed=42)
    ao = wsmc.models.oscillator_statements(o, t, y, **kw)
    assert len(ag) == 5 * 5 and ag == ao
    assert_same_state(g, o)
    assert g.log_evidence() == o.log_evidence()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("mode", ["island", "exact"])
@pytest.mark.parametrize("scheme", [0, 1])
def test_c5_four_shards_full_horizon(gpu_available, mode, scheme):
    """C5 at its 4-GPU partition (BASELINE configs[4]) on one GPU: SMCState over 4 shards of
    12.5k in one handle (wsmc_create_multi, the in-process exchange standing in for RCCL), all
    60 observations, 5 ungated sweeps of the bounded 4-D + 1-D autoRW moves (600 moves, the
    sharded autoRW combine at every one). Island shards against the four-shard oracle, exact
    shards against it in exact mode (one population's bits), accepted counts and every column
    bit for bit."""
    import wsmc
    from oracle import Oracle
    from wsmc import abi
    from test_gpu_parity import assert_same_state
    G, N = 4, 50_000
    exact = mode == "exact"
    t, y = wsmc.models.oscillator_data(n=60)
    g = wsmc.Context.multi(N, G, seed=4, devices=[0] * G, transport=abi.TRANSPORT_HOST)
    if exact:
        g.comm_set_shard_mode(abi.SHARD_EXACT)
    o = Oracle(N, seed=4, shards=G, exact=exact)
    ag = wsmc.models.oscillator_statements(g, t, y, ess_perc_min=1.0, scheme=scheme, sweeps=5, diversity=None)
    ao = wsmc.models.oscillator_statements(o, t, y, ess_perc_min=1.0, scheme=scheme, sweeps=5, diversity=None)
    assert len(ag) == 60 * 5
    assert ag == ao
    assert_same_state(g, o)
    assert g.log_evidence() == o.log_evidence()
    g.close()


# ---- C4's partition ----------------------------------------------------------------------
def _digest(a):
    import xxhash
    return xxhash.xxh3_128_hexdigest(np.ascontiguousarray(a).tobytes())


def _c4_worker(rank, world, port, n, T, mode, outdir):
    sys.path[:0] = [str(REPO / "weightedsampling.jl_amd")]
    import json
    import wsmc
    from wsmc import abi
    from wsmc.hostcomm import HostComm
    comm = HostComm(rank, world, "127.0.0.1", port, tag="c4", timeout=300)
    obs = wsmc.models.ssm2d_data(T)
    c = wsmc.Context(n, seed=42, device=0)
    c.comm_init_host(comm.allgather, world, rank, rank * n, world * n)
    if mode == "exact":
        c.comm_set_shard_mode(abi.SHARD_EXACT)
    ev = c.ssm2d_run(obs, ess_perc_min=1.0, keep_history=True)
    out = {"ev": ev, "w": _digest(c.weights_download()), "flags": c.get_state()["n_resamples"]}
    for name in c.col_names():
        out["c_" + name] = _digest(c.col_download(c.col_find(name)))
    c.close()
    comm.barrier()
    comm.close()
    with open(os.path.join(outdir, f"rank{rank}.json"), "w") as f:
        json.dump(out, f)


def _run_ranks(world, target, args, tmp_path):
    import multiprocessing as mp
    from test_gpu_multishard import _free_port
    port = _free_port()
    ctx = mp.get_context("spawn")
    ps = [ctx.Process(target=target, args=(r, world, port) + args + (str(tmp_path),)) for r in range(world)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(600)
    codes = [p.exitcode for p in ps]
    for p in ps:
        if p.is_alive():
            p.kill()
    assert codes == [0] * world, codes


@pytest.mark.timeout(600)
@pytest.mark.parametrize("mode", ["island", "exact"])
def test_c4_population_as_two_shards(gpu_available, tmp_path, mode):
    """C4's 8M particles as two 4M shards (the per-GPU size of C4 on two GPUs), T = 100,
    forced resampling: every traced-back column and the weights, bit for bit."""
    import json
    import oracle
    import wsmc
    world, n, T = 2, 4_000_000, 100
    _run_ranks(world, _c4_worker, (n, T, mode), tmp_path)
    res = [json.load(open(tmp_path / f"rank{r}.json")) for r in range(world)]
    obs = wsmc.models.ssm2d_data(T)
    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    if mode == "exact":   # the shards together hold one context's bits
        p = oracle.ssm2d_run_mt(world * n, obs, seed=42, ess_perc_min=1.0, threads=threads)
        for r in range(world):
            sl = slice(r * n, (r + 1) * n)
            assert res[r]["w"] == _digest(p["weights"][sl])
            for k, v in p.items():
                if k.startswith("x_") or k in ("v", "dv"):
                    assert res[r]["c_" + k] == _digest(v[..., sl]), (r, k)
            assert res[r]["ev"] == p["log_evidence"]
        return
    for r in range(world):   # island: shard r is one port run with its global offset
        p = oracle.ssm2d_run_mt(n, obs, seed=42, ess_perc_min=1.0, threads=threads, goff=r * n)
        assert res[r]["w"] == _digest(p["weights"])
        for k, v in p.items():
            if k.startswith("x_") or k in ("v", "dv"):
                assert res[r]["c_" + k] == _digest(v), (r, k)
        del p


@pytest.mark.timeout(600)
def test_eight_shards_one_gpu_island(gpu_available, tmp_path):
    """C4's partition (eight ranks) at 8 x 20k, T = 100: the statement path and the fused
    run of every rank against the eight-shard oracle."""
    import wsmc
    from oracle import Oracle
    from test_gpu_multishard import _worker
    world, N, T = 8, 160_000, 100
    _run_ranks(world, _worker, (N, T, 1.0, 0), tmp_path)
    ref = Oracle(N, seed=21, shards=world)
    flags = wsmc.models.ssm2d_statements(ref, wsmc.models.ssm2d_data(T), ess_perc_min=1.0)
    n = N // world
    w = ref.weights_download()
    cols = {name: ref.col_download(ref.col_find(name)) for name in ref.col_names()}
    for r in range(world):
        p = np.load(tmp_path / f"rank{r}.npz")
        sl = slice(r * n, (r + 1) * n)
        assert list(p["flags"]) == flags
        np.testing.assert_array_equal(p["w"], w[sl])
        np.testing.assert_array_equal(p["fw"], w[sl])
        for name, full in cols.items():
            np.testing.assert_array_equal(p["s_" + name], full[..., sl], err_msg=name)
            np.testing.assert_array_equal(p["f_" + name], full[..., sl], err_msg=name)
        assert p["ev"][0] == ref.log_evidence()
        assert p["fev"][0] == ref.log_evidence()
