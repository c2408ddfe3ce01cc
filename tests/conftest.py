"""Test configuration: repo paths, the `gpu` marker, and backend factories.

`-m "not gpu"` tests run on CPU only (oracle vs golden vectors / analytic oracles, host
logic, ABI symbol checks). `-m gpu` tests call the HIP library through the C ABI and
compare against the CPU oracle (oracle/) bit for bit.
"""
import pathlib
import sys

import pytest

REPO = pathlib.Path(__file__).resolve().parents[1]
for p in (REPO / "weightedsampling.jl_amd", REPO / "oracle", REPO):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and libwsmc.so")
    config.addinivalue_line("markers", "slow: long-running statistical test")


@pytest.fixture(scope="session")
def gpu_available():
    import wsmc
    try:
        n = wsmc.device_count()
    except Exception as e:  # library missing is a hard failure for gpu tests
        pytest.fail(f"libwsmc.so unusable: {e}")
    if n < 1:
        pytest.fail("no HIP device visible")
    return n
