"""Golden fixtures (tests/golden/make_golden.py): the oracle must reproduce them exactly
(regression pin of the restatement); under -m gpu the HIP path must match them bit for bit."""
import pathlib

import numpy as np
import pytest

import wsmc
from backends import BACKENDS, make_ctx

G = pathlib.Path(__file__).resolve().parent / "golden"


def check(ctx, path, flags):
    f = np.load(path)
    assert list(ctx.col_names()) == list(f["colnames"])
    for n in f["colnames"]:
        np.testing.assert_array_equal(ctx.col_download(ctx.col_find(str(n))), f[f"col__{n}"], err_msg=str(n))
    np.testing.assert_array_equal(ctx.weights_download(), f["weights"])
    np.testing.assert_array_equal(ctx.last_ancestors(), f["ancestors"])
    if flags is not None:
        assert list(np.asarray(flags, dtype=np.int8).reshape(-1)) == list(f["resampled"].reshape(-1))
    assert ctx.log_evidence() == f["log_evidence"][0]
    st = ctx.get_state()
    assert [st["depth"], st["n_terms"], st["op_counter"], st["n_resamples"]] == list(f["state"])


@pytest.mark.parametrize("backend", BACKENDS)
@pytest.mark.parametrize("tag", ["05", "10"])
def test_golden_ssm1d(backend, tag):
    path = G / f"c1_ssm1d_ess{tag}.npz"
    f = np.load(path)
    c = make_ctx(backend, 1000, seed=7)
    flags = wsmc.models.ssm1d_statements(c, f["obs"], ess_perc_min=int(tag) / 10)
    check(c, path, flags)


@pytest.mark.parametrize("backend", BACKENDS)
@pytest.mark.parametrize("tag", ["05", "10"])
def test_golden_ssm2d(backend, tag):
    path = G / f"c2_ssm2d_ess{tag}.npz"
    f = np.load(path)
    c = make_ctx(backend, 1024, seed=42)
    flags = wsmc.models.ssm2d_statements(c, f["obs"], ess_perc_min=int(tag) / 10)
    check(c, path, flags)


@pytest.mark.gpu
@pytest.mark.parametrize("tag", ["05", "10"])
def test_golden_ssm2d_fused(tag):
    path = G / f"c2_ssm2d_ess{tag}.npz"
    f = np.load(path)
    c = wsmc.Context(1024, seed=42)
    c.ssm2d_run(f["obs"], ess_perc_min=int(tag) / 10, keep_history=True)
    for n in f["colnames"]:
        np.testing.assert_array_equal(c.col_download(c.col_find(str(n))), f[f"col__{n}"], err_msg=str(n))
    np.testing.assert_array_equal(c.weights_download(), f["weights"])
    assert c.log_evidence() == f["log_evidence"][0]


@pytest.mark.parametrize("backend", BACKENDS)
def test_golden_linreg(backend):
    path = G / "c3_linreg_ess10.npz"
    f = np.load(path)
    c = make_ctx(backend, 2048, seed=42)
    acc = wsmc.models.linreg_statements(c, f["xs"], f["ys"], ess_perc_min=1.0)
    np.testing.assert_array_equal(np.array(acc), f["accepted"])
    check(c, path, None)


@pytest.mark.parametrize("backend", BACKENDS)
def test_golden_oscillator(backend):
    path = G / "c5_oscillator_ess10.npz"
    f = np.load(path)
    c = make_ctx(backend, 2048, seed=42)
    acc = wsmc.models.oscillator_statements(c, f["t"], f["y"], ess_perc_min=1.0,
                                            scheme=wsmc.RESAMPLE_SYSTEMATIC, sweeps=2, diversity=None)
    np.testing.assert_array_equal(np.array(acc), f["accepted"])
    check(c, path, None)
