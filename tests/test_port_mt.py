"""The all-cores CPU port of the fused 2D SSM run (oracle/wsmc_port_mt.c, bench.py's
cpu_baseline): bit for bit the statement oracle (every traced-back column, the weights, the
flags, the evidence) for every thread count, so the baseline times the same computation
the device's wsmc_ssm2d_run does."""
import numpy as np
import pytest

import oracle
import wsmc
from oracle import Oracle
from wsmc import abi


@pytest.mark.parametrize("N,T,ess,scheme", [
    (1, 4, 1.0, abi.RESAMPLE_STRATIFIED),
    (5, 6, 1.0, abi.RESAMPLE_STRATIFIED),
    (1025, 12, 1.0, abi.RESAMPLE_SYSTEMATIC),
    (3001, 8, 0.5, abi.RESAMPLE_STRATIFIED),
    (4096, 10, 0.9, abi.RESAMPLE_SYSTEMATIC),
])
def test_port_mt_matches_statement_oracle(N, T, ess, scheme):
    obs = wsmc.models.ssm2d_data(T)
    o = Oracle(N, seed=123)
    flags = wsmc.models.ssm2d_statements(o, obs, ess_perc_min=ess, scheme=scheme)
    for threads in (1, 3, 8):
        r = oracle.ssm2d_run_mt(N, obs, seed=123, ess_perc_min=ess, scheme=scheme, threads=threads)
        for name in o.col_names():
            np.testing.assert_array_equal(r[name], o.col_download(o.col_find(name)), err_msg=f"{name} t={threads}")
        np.testing.assert_array_equal(r["weights"], o.weights_download())
        assert list(r["flags"]) == [bool(f) for f in flags]
        assert r["log_evidence"] == o.log_evidence()


def test_port_mt_without_history_is_the_last_column():
    obs = wsmc.models.ssm2d_data(9)
    a = oracle.ssm2d_run_mt(2000, obs, seed=5, ess_perc_min=1.0, threads=4, keep_history=True)
    b = oracle.ssm2d_run_mt(2000, obs, seed=5, ess_perc_min=1.0, threads=2, keep_history=False)
    np.testing.assert_array_equal(b["x"], a["x_10"])
    for k in ("v", "dv", "weights"):
        np.testing.assert_array_equal(b[k], a[k])
    assert a["log_evidence"] == b["log_evidence"]


def test_port_mt_degenerate_weights():
    # a NaN observation: NaN log-weights never resample (ESS is NaN, the strict test fails),
    # exactly as the statements do
    obs = wsmc.models.ssm2d_data(6).copy()
    obs[3, 0] = np.nan
    o = Oracle(777, seed=9)
    flags = wsmc.models.ssm2d_statements(o, obs, ess_perc_min=1.0)
    r = oracle.ssm2d_run_mt(777, obs, seed=9, ess_perc_min=1.0, threads=4)
    assert list(r["flags"]) == [bool(f) for f in flags]
    np.testing.assert_array_equal(r["weights"], o.weights_download())
    for name in o.col_names():
        np.testing.assert_array_equal(r[name], o.col_download(o.col_find(name)), err_msg=name)


@pytest.mark.parametrize("world", [2, 3])
def test_port_mt_goff_is_one_island_shard(world):
    """With the global offset (RNG index and stratum slot base) the port runs one island shard
    of a sharded population: under forced resampling (every step resamples, whatever the
    global ESS; the first step's weights are all equal everywhere) shard r's columns and weights equal the sharded oracle's slice — the
    reference the C4 shard tests hold the device against at 4M particles a shard."""
    n, T = 1500, 12
    obs = wsmc.models.ssm2d_data(T)
    o = Oracle(n * world, seed=77, shards=world)
    flags = wsmc.models.ssm2d_statements(o, obs, ess_perc_min=1.0)
    assert all(flags[1:])                   # step 1: x_2 = x0 + v0 for all, equal weights, ESS = 1
    for r in range(world):
        p = oracle.ssm2d_run_mt(n, obs, seed=77, ess_perc_min=1.0, threads=4, goff=r * n)
        assert list(p["flags"]) == [bool(f) for f in flags]
        sl = slice(r * n, (r + 1) * n)
        for name in o.col_names():
            np.testing.assert_array_equal(p[name], o.col_download(o.col_find(name))[..., sl], err_msg=name)
        np.testing.assert_array_equal(p["weights"], o.weights_download()[sl])
