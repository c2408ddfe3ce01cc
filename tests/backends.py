"""Backend factories for tests: the same SMCState/transformer programs run on the CPU
oracle (oracle/, test infrastructure) or on the HIP library (gpu-marked tests)."""
import numpy as np
import pytest

import wsmc
from oracle import Oracle

BACKENDS = [pytest.param("oracle", id="oracle"), pytest.param("hip", id="hip", marks=pytest.mark.gpu)]


def make_ctx(backend: str, n: int, seed: int = 42):
    if backend == "oracle":
        return Oracle(n, seed=seed)
    return wsmc.Context(n, seed=seed)


def make_state(backend: str, n: int, seed: int = 42, ess_perc_min: float = 0.5, scheme: int = 0):
    return wsmc.SMCState.from_context(make_ctx(backend, n, seed), ess_perc_min=ess_perc_min, scheme=scheme)


def normlogpdf(mu, sigma, x):
    z = (np.asarray(x, float) - mu) / sigma
    return -(z * z + np.log(2 * np.pi)) / 2 - np.log(sigma)


def exp_norm(lw):
    w = np.exp(lw - np.max(lw))
    return w / w.sum()


def logsumexp(lw):
    m = np.max(lw)
    return m + np.log(np.sum(np.exp(lw - m)))


def kalman_filter_evidence(data, a, q, r):
    """test/models.jl:272-288 (1D, x0 ~ N(0,1))."""
    mu, P, ev = 0.0, 1.0, 0.0
    for y in data:
        mu_p, P_p = a * mu, a * a * P + q * q
        S = P_p + r * r
        res = y - mu_p
        ev += -0.5 * (np.log(2 * np.pi) + np.log(S) + res * res / S)
        K = P_p / S
        mu, P = mu_p + K * res, (1 - K) * P_p
    return mu, ev


def kalman_2d_ssm(obs, x0=(0.0, 0.0), v0=(1.0, 0.0), q_var=0.1, r_var=0.5):
    """Exact filter for examples/2D_ssm.jl: per axis s=(x_{t+1}, v_{t+1}) = F s + (0, dv),
    dv ~ N(0, q_var), o_t ~ N(x_{t+1}, r_var), start at the point mass (x0, v0).
    Returns (log evidence, final posterior mean of x_{T+1} per axis, its variance)."""
    F = np.array([[1.0, 1.0], [0.0, 1.0]])
    Qm = np.diag([0.0, q_var])
    ev = 0.0
    means, vars_ = [], []
    obs = np.asarray(obs, float)
    for ax in range(2):
        m = np.array([x0[ax], v0[ax]])
        P = np.zeros((2, 2))
        for t in range(len(obs)):
            # the step's x{t+1} uses the pre-update v; the observation sees x{t+1}
            m = F @ m
            P = F @ P @ F.T + Qm
            S = P[0, 0] + r_var
            y = obs[t, ax] - m[0]
            ev += -0.5 * (np.log(2 * np.pi) + np.log(S) + y * y / S)
            K = P[:, 0] / S
            m = m + K * y
            P = P - np.outer(K, P[0, :])
        means.append(m[0])
        vars_.append(P[0, 0])
    return ev, np.array(means), np.array(vars_)


def conjugate_linreg(xs, ys, prior_sd=10.0, obs_sd=1.0):
    """Exact posterior of α, β ~ N(0, prior_sd²), y ~ N(α + β x, obs_sd²) and the evidence."""
    X = np.column_stack([np.ones(len(xs)), np.asarray(xs, float)])
    y = np.asarray(ys, float)
    S0 = prior_sd ** 2 * np.eye(2)
    prec = np.linalg.inv(S0) + X.T @ X / obs_sd ** 2
    cov = np.linalg.inv(prec)
    mean = cov @ (X.T @ y) / obs_sd ** 2
    C = X @ S0 @ X.T + obs_sd ** 2 * np.eye(len(y))
    sign, logdet = np.linalg.slogdet(C)
    ev = -0.5 * (len(y) * np.log(2 * np.pi) + logdet + y @ np.linalg.solve(C, y))
    return mean, cov, ev
