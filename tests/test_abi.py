"""CPU checks of the drop-in boundary: libwsmc.so loads, exports every symbol declared in
include/wsmc.h, and the ctypes layouts match the C structs. No compute without a GPU."""
import ctypes as C
import pathlib
import re

import pytest

import oracle as O
import wsmc
from wsmc import abi

REPO = pathlib.Path(__file__).resolve().parents[1]


def declared_functions():
    src = (REPO / "include" / "wsmc.h").read_text()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(wsmc_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    lib = wsmc.load_library()
    names = declared_functions()
    assert len(names) >= 30
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    # and every declared function has a bound signature on the Python side
    assert set(names) <= set(abi.SIGNATURES), set(names) - set(abi.SIGNATURES)


def test_struct_layouts_match_c():
    L = O.lib()
    assert C.sizeof(abi.Term) == L.or_sizeof_term()
    assert C.sizeof(abi.Dist) == L.or_sizeof_dist()
    assert C.sizeof(abi.Operand) == 40
    assert C.sizeof(abi.CommInfo) == 120   # 6 int32, devices[8] int32, shard_n[8] int64


def test_version_and_error_channel():
    lib = wsmc.load_library()
    ma, mi = C.c_int32(), C.c_int32()
    assert lib.wsmc_version(C.byref(ma), C.byref(mi)) == 0
    # an invalid call reports through wsmc_last_error, no exception across the ABI
    rc = lib.wsmc_nparticles(None, None)
    assert rc == abi.WSMC_EARG
    assert b"null" in lib.wsmc_last_error()


def test_product_fails_loudly_without_device_or_library(tmp_path):
    # (no torch import here: torch's bundled HIP runtime must never share a process with libwsmc)
    try:
        if wsmc.device_count() > 0:
            pytest.skip("GPU present")
    except wsmc.WSMCError:
        pass
    with pytest.raises(wsmc.WSMCError):
        wsmc.Context(16)
    with pytest.raises(ImportError):
        abi.load_library(tmp_path / "missing.so")


def test_statement_batch_jit_compiles_without_a_device():
    """The run-time compiled statement batches (csrc/wsmc_jit.hip): hiprtc builds a
    representative signature (the 2D SSM step) from the headers embedded in the library,
    for gfx950, with no device — the build check of the code the GPU path compiles."""
    lib = wsmc.load_library()
    rc = lib.wsmc_debug_jit_selfcheck()
    assert rc == abi.WSMC_OK, lib.wsmc_last_error().decode()
    st = abi.jit_stats()
    assert set(st) == {"compiled", "failed", "launched", "interpreted", "compile_s"}


def test_move_block_jit_compiles_without_a_device():
    """The run-time compiled Move blocks (csrc/wsmc_mv_body.h): hiprtc builds C3's block shape
    (two 1-D unbounded autoRW moves over two Normal priors and an affine Normal run) from the
    headers embedded in the library, for gfx950, with no device."""
    lib = wsmc.load_library()
    rc = lib.wsmc_debug_mv_jit_selfcheck()
    assert rc == abi.WSMC_OK, lib.wsmc_last_error().decode()
    st = abi.mv_jit_stats()
    assert set(st) == {"compiled", "failed", "launched", "interpreted", "compile_s"}
