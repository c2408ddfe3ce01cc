"""The Move acceptance screen (csrc/wsmc_kernels.hip `move_accept`).

The reference accepts a proposal when `log(rand()) < lpr + s_new - s_old`
(/root/reference/src/transformers.jl:615). The device decides it from a single-precision
log of u wherever that settles the comparison, and falls back to the restated double log
(include/wsmc_math.h wsmc_log, the oracle's) inside a band around the estimate. The decision
bits equal the oracle's exactly when the estimate lies within the band's half-width
2^-13 + 2^-16 |L| of the double log for every u >= 2^-60 (smaller u always take the double
log). This checks that bound on the device, with a factor of 8 to spare, over random
uniforms on the 2^-53 grid, log-uniform values down to 2^-60, and the neighbourhoods of 1 and
of every power of two. The Move parity tests check the decisions themselves bit for bit.
"""
import ctypes as C

import numpy as np
import pytest

from wsmc import abi


def _screen(u):
    u = np.ascontiguousarray(u, dtype=np.float64)
    out = np.empty(2 * u.size, dtype=np.float64)
    abi.check(abi.load_library().wsmc_debug_log_screen(u.ctypes.data_as(C.c_void_p), u.size,
                                                        out.ctypes.data_as(C.c_void_p)))
    return out[0::2], out[1::2]


@pytest.mark.gpu
def test_log_screen_band_bound(gpu_available):
    rng = np.random.default_rng(20261017)
    grid = (rng.integers(1, 2**53, size=2_000_000, dtype=np.int64).astype(np.float64)) * 2.0**-53
    logu = np.exp2(-rng.uniform(0.0, 60.0, size=2_000_000))
    near1 = 1.0 - np.arange(1, 200_001, dtype=np.float64) * 2.0**-53
    pw = []
    for k in range(1, 61):
        b = 2.0**-k
        pw.append(b + np.arange(-64, 65) * np.spacing(b))
    u = np.concatenate([grid, logu, near1, np.concatenate(pw)])
    u = u[(u >= 2.0**-60) & (u < 1.0)]
    L, exact = _screen(u)
    band = 2.0**-13 + 2.0**-16 * np.abs(L)
    err = np.abs(L - exact)
    worst = float(np.max(err / band))
    assert np.all(np.isfinite(L))
    assert worst < 0.125, f"screen estimate within {worst:.3g} of its band (bound 1/8)"
