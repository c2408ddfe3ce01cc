"""The reference-speed CPU ports (oracle/wsmc_port_fast.c, bench.py's cpu_baseline legs):
the reference's algorithm with a fast non-canonical RNG (xoshiro256++ + ziggurat) and libm,
so not bit-exact — checked statistically against the exact Kalman filters, like the
reference's own filter tests (test/transformers_test.jl:158-190)."""
import numpy as np
import pytest

import oracle
import wsmc
from backends import kalman_2d_ssm, kalman_filter_evidence


@pytest.mark.parametrize("threads", [1, 4])
def test_fast_lgssm1d_matches_kalman(threads):
    data = wsmc.models.lgssm1d_data(200)
    exact_mean, exact_ev = kalman_filter_evidence(data, 0.9, 1.0, 0.5)
    ev, pm, nrs = oracle.fast_lgssm1d_run(50_000, data, ess_perc_min=1.0, threads=threads)
    assert nrs == 200
    assert abs(ev - exact_ev) < 1.0
    assert abs(pm - exact_mean) < 0.05


def test_fast_lgssm1d_ess_gate():
    data = wsmc.models.lgssm1d_data(100)
    _, _, never = oracle.fast_lgssm1d_run(2000, data, ess_perc_min=0.0)    # strict <: ESS% < 0 never
    assert never == 0
    _, _, some = oracle.fast_lgssm1d_run(2000, data, ess_perc_min=0.5)
    assert 0 < some <= 100


@pytest.mark.parametrize("threads", [1, 3])
def test_fast_ssm2d_matches_kalman(threads):
    T = 20
    obs = wsmc.models.ssm2d_data(T)
    ev_exact, m_exact, v_exact = kalman_2d_ssm(obs)
    ev, nrs, xs = oracle.fast_ssm2d_run(100_000, obs, ess_perc_min=1.0, threads=threads, outputs=True)
    assert nrs == T - 1        # step 1 observes x_2 = x_1 + v0 for every particle: ESS% = 1, not < 1
    assert abs(ev - ev_exact) < 1.0
    # forced resampling leaves equal weights: the posterior mean is the plain column mean
    np.testing.assert_array_less(np.abs(xs[T].mean(axis=1) - m_exact), 4 * np.sqrt(v_exact) / np.sqrt(2000) + 0.05)
    np.testing.assert_array_equal(xs[0], np.zeros((2, 100_000)))          # x_1 = [0, 0]


def test_fast_ssm2d_history_is_a_lineage():
    """The traced-back history is a set of lineages: x_{t+1} - x_t is the lineage's v, which
    changes by one dv draw per step (σ = √0.1; selection by the observations only narrows
    it), never by a jump between particles."""
    T, N = 12, 4096
    obs = wsmc.models.ssm2d_data(T)
    _, _, xs = oracle.fast_ssm2d_run(N, obs, ess_perc_min=1.0, threads=2, outputs=True)
    v = np.diff(xs, axis=0)                       # [T, 2, N]: v_1 .. v_T of each lineage
    np.testing.assert_array_equal(v[0], np.tile(np.array([[1.0], [0.0]]), (1, N)))
    dv = np.diff(v, axis=0)
    assert abs(dv.mean()) < 0.05 and 0.15 < dv.std() < np.sqrt(0.1) + 0.02
