"""ctypes view of the C ABI in include/wsmc.h (the drop-in boundary).

Loads ``libwsmc.so`` built in-tree by ``weightedsampling.jl_amd/build.py``. There is no
fallback: if the library is missing or fails to load, importing the operators raises.
"""
from __future__ import annotations

import ctypes as C
import os
import pathlib

_PKG_DIR = pathlib.Path(__file__).resolve().parent
LIB_PATH = _PKG_DIR / "libwsmc.so"

# ---- enums (include/wsmc.h) ---------------------------------------------------------
WSMC_OK, WSMC_EARG, WSMC_EHIP, WSMC_ENOTPD, WSMC_ERCCL, WSMC_ESTATE, WSMC_ENOMEM = range(7)
FAM_NORMAL, FAM_HALFNORMAL, FAM_UNIFORM, FAM_MVNORMAL_ISO, FAM_MVNORMAL = range(5)
(FAM_BERNOULLI, FAM_BERNOULLI_LOGIT, FAM_EXPONENTIAL, FAM_LOGNORMAL, FAM_LAPLACE, FAM_CAUCHY, FAM_LOGISTIC,
 FAM_GUMBEL, FAM_RAYLEIGH, FAM_GEOMETRIC) = range(5, 15)
MEAN_AFFINE, MEAN_OSCILLATOR = range(2)
TERM_SAMPLE, TERM_OBSERVE, TERM_WEIGHT = range(3)
RESAMPLE_STRATIFIED, RESAMPLE_SYSTEMATIC, RESAMPLE_MULTINOMIAL = range(3)
SHARD_ISLAND, SHARD_EXACT = range(2)
TRANSPORT_RCCL, TRANSPORT_HOST = range(2)
PROPOSAL_RW, PROPOSAL_AUTORW = range(2)


class Operand(C.Structure):
    """value(i) = c0 + coef[0]*col[0][comp[0]][i] + coef[1]*col[1][comp[1]][i]"""
    _fields_ = [("c0", C.c_double), ("col", C.c_int32 * 2), ("comp", C.c_int32 * 2),
                ("coef", C.c_double * 2)]

    @classmethod
    def const(cls, v: float) -> "Operand":
        o = cls()
        o.c0 = float(v)
        o.col[0] = o.col[1] = -1
        return o

    @classmethod
    def column(cls, col: int, comp: int = 0, coef: float = 1.0, c0: float = 0.0) -> "Operand":
        o = cls()
        o.c0 = float(c0)
        o.col[0], o.comp[0], o.coef[0] = int(col), int(comp), float(coef)
        o.col[1] = -1
        return o


class XInst(C.Structure):
    """wsmc_xinst: one instruction of a wsmc_assign_expr postfix program"""
    _fields_ = [("op", C.c_int32), ("col", C.c_int32), ("comp", C.c_int32), ("reserved", C.c_int32),
                ("c", C.c_double)]


# wsmc_xop (include/wsmc.h)
X_CONST, X_COL, X_NEG, X_ABS, X_SQRT, X_EXP, X_LOG, X_LOG1P, X_SIN, X_COS, X_POWI, X_NOT = range(12)
X_ADD, X_SUB, X_MUL, X_DIV, X_MIN, X_MAX, X_POW, X_LT, X_LE, X_GT, X_GE, X_EQ, X_NE, X_AND, X_OR, \
    X_IFELSE = range(16, 32)
XPROG_MAX, XSTACK_MAX = 96, 8


class Dist(C.Structure):
    _fields_ = [("family", C.c_int32), ("mean_fn", C.c_int32), ("dim", C.c_int32),
                ("reserved", C.c_int32), ("mu", Operand * 4), ("scale", Operand),
                ("param", C.c_double * 2)]


class Term(C.Structure):
    _fields_ = [("dist", Dist), ("x", Operand * 4), ("kind", C.c_int32), ("depth", C.c_int32)]


class State(C.Structure):
    _fields_ = [("resampled", C.c_int32), ("weights_changed", C.c_int32), ("depth", C.c_int32),
                ("n_terms", C.c_int32), ("last_ess_perc", C.c_double),
                ("op_counter", C.c_uint64), ("n_resamples", C.c_int64)]


class CommInfo(C.Structure):
    """wsmc_comm_info_t: what a context or multi-device handle is sharded over"""
    _fields_ = [("shards", C.c_int32), ("world", C.c_int32), ("rank", C.c_int32),
                ("rccl_ranks", C.c_int32), ("transport", C.c_int32), ("shard_mode", C.c_int32),
                ("devices", C.c_int32 * 8), ("shard_n", C.c_int64 * 8)]


class MoveSpec(C.Structure):
    """wsmc_move_spec: one Move of a wsmc_move_block statement block"""
    _fields_ = [("proposal", C.c_int32), ("d", C.c_int32), ("targets", C.c_int32 * 4),
                ("bounded", C.c_int32), ("target_depth", C.c_int32), ("step", C.c_double),
                ("lo", C.c_double * 4), ("hi", C.c_double * 4)]


class RunTiming(C.Structure):
    _fields_ = [("total_ms", C.c_double), ("propagate_ms", C.c_double),
                ("reduce_ms", C.c_double), ("resample_ms", C.c_double),
                ("finalize_ms", C.c_double), ("steps", C.c_int32), ("n_resamples", C.c_int32)]


# ---- exported symbols (name -> (restype, argtypes)); tests check every one loads ----
_P = C.c_void_p
_D = C.POINTER(C.c_double)
_I32P = C.POINTER(C.c_int32)
SIGNATURES = {
    "wsmc_last_error": (C.c_char_p, []),
    "wsmc_version": (C.c_int, [_I32P, _I32P]),
    "wsmc_device_count": (C.c_int, [_I32P]),
    "wsmc_dist_mvnormal_cov": (C.c_int, [C.c_void_p, _D]),
    "wsmc_create": (C.c_int, [C.POINTER(_P), C.c_int64, C.c_int32, C.c_uint64]),
    "wsmc_destroy": (C.c_int, [_P]),
    "wsmc_create_multi": (C.c_int, [C.POINTER(_P), C.c_int64, C.c_int32, _I32P, C.c_uint64, C.c_int32]),
    "wsmc_sync": (C.c_int, [_P]),
    "wsmc_nparticles": (C.c_int, [_P, C.POINTER(C.c_int64)]),
    "wsmc_get_state": (C.c_int, [_P, C.POINTER(State)]),
    "wsmc_set_depth": (C.c_int, [_P, C.c_int32]),
    "wsmc_set_op_counter": (C.c_int, [_P, C.c_uint64]),
    "wsmc_comm_unique_id": (C.c_int, [C.POINTER(C.c_uint8)]),
    "wsmc_comm_init": (C.c_int, [_P, C.POINTER(C.c_uint8), C.c_int32, C.c_int32, C.c_int64,
                                 C.c_int64]),
    "wsmc_comm_set_shard_mode": (C.c_int, [_P, C.c_int32]),
    "wsmc_comm_info": (C.c_int, [_P, C.POINTER(CommInfo)]),
    "wsmc_comm_init_host": (C.c_int, [_P, C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_int64,
                                      C.c_int64]),
    "wsmc_col_create": (C.c_int, [_P, C.c_char_p, C.c_int32, _I32P]),
    "wsmc_col_find": (C.c_int, [_P, C.c_char_p, _I32P]),
    "wsmc_col_count": (C.c_int, [_P, _I32P]),
    "wsmc_col_info": (C.c_int, [_P, C.c_int32, C.c_char_p, C.c_int32, _I32P]),
    "wsmc_col_download": (C.c_int, [_P, C.c_int32, _D]),
    "wsmc_col_upload": (C.c_int, [_P, C.c_int32, _D]),
    "wsmc_col_device_ptr": (C.c_int, [_P, C.c_int32, C.POINTER(_D)]),
    "wsmc_store_resample": (C.c_int, [_P, _I32P]),
    "wsmc_store_set_lazy": (C.c_int, [_P, C.c_int32]),
    "wsmc_store_materialize": (C.c_int, [_P]),
    "wsmc_store_info": (C.c_int, [_P, C.POINTER(C.c_int64), _I32P]),
    "wsmc_weights_upload": (C.c_int, [_P, _D]),
    "wsmc_weights_download": (C.c_int, [_P, _D]),
    "wsmc_log_evidence": (C.c_int, [_P, _D]),
    "wsmc_weighted_moments": (C.c_int, [_P, C.POINTER(Operand), C.c_int32, _D, _D]),
    "wsmc_col_minmax": (C.c_int, [_P, C.c_int32, C.c_int32, _D, _D]),
    "wsmc_ess": (C.c_int, [_P, _D]),
    "wsmc_weighted_median": (C.c_int, [_P, C.c_int32, C.c_int32, _D]),
    "wsmc_histogram": (C.c_int, [_P, C.c_int32, C.c_int32, C.POINTER(C.c_int32)]),
    "wsmc_sample_particles": (C.c_int, [_P, C.c_int64, C.c_int32, C.POINTER(C.c_int64)]),
    "wsmc_col_gather_rows": (C.c_int, [_P, C.c_int32, C.POINTER(C.c_int64), C.c_int64, _D]),
    "wsmc_assign": (C.c_int, [_P, C.c_int32, C.POINTER(Operand)]),
    "wsmc_assign_expr": (C.c_int, [_P, C.c_int32, C.POINTER(XInst), _I32P]),
    "wsmc_sample": (C.c_int, [_P, C.c_int32, C.POINTER(Dist)]),
    "wsmc_sample_importance": (C.c_int, [_P, C.c_int32, C.POINTER(Dist), C.POINTER(Dist)]),
    "wsmc_observe": (C.c_int, [_P, C.POINTER(Dist), C.POINTER(Operand)]),
    "wsmc_weight": (C.c_int, [_P, C.POINTER(Dist), C.POINTER(Operand)]),
    "wsmc_resample": (C.c_int, [_P, C.c_double, C.c_int32, _I32P, _D]),
    "wsmc_move": (C.c_int, [_P, C.c_int32, _I32P, C.c_int32, C.c_double, _D, _D, C.c_int32,
                            C.c_double, C.POINTER(C.c_int64)]),
    "wsmc_move_gated": (C.c_int, [_P, C.c_int32, _I32P, C.c_int32, C.c_double, _D, _D, C.c_int32, C.c_double]),
    "wsmc_move_block": (C.c_int, [_P, C.c_int32, C.POINTER(MoveSpec), C.c_int32, C.POINTER(C.c_int64)]),
    "wsmc_score": (C.c_int, [_P, C.c_int32, _D]),
    "wsmc_marginal_diversity": (C.c_int, [_P, _I32P, C.c_int32, _D]),
    "wsmc_last_ancestors": (C.c_int, [_P, _I32P]),
    "wsmc_ssm2d_run": (C.c_int, [_P, _D, C.c_int32, _D, _D, C.c_double, C.c_double, C.c_double,
                                 C.c_int32, C.c_int32, _D]),
    "wsmc_run_set_timing": (C.c_int, [_P, C.c_int32]),
    "wsmc_run_get_timing": (C.c_int, [_P, C.POINTER(RunTiming)]),
    "wsmc_debug_kernel_bench": (C.c_int, [_P, C.c_int32, C.c_int32, C.c_int32, _D]),
    "wsmc_debug_inject_failure": (C.c_int, [_P, C.c_int32, C.c_int32]),
    "wsmc_debug_exact": (C.c_int, [_P, C.c_int64, C.c_int64, C.POINTER(C.c_int64)]),
    "wsmc_debug_jit_stats": (C.c_int, [C.POINTER(C.c_int64)]),
    "wsmc_debug_jit_selfcheck": (C.c_int, []),
    "wsmc_debug_log_screen": (C.c_int, [C.c_void_p, C.c_int64, C.c_void_p]),
    "wsmc_debug_mv_jit_stats": (C.c_int, [C.POINTER(C.c_int64)]),
    "wsmc_debug_mv_jit_selfcheck": (C.c_int, []),
    "wsmc_debug_run_stats": (C.c_int, [C.c_void_p, C.POINTER(C.c_int64)]),
    "wsmc_comm_set_timeout": (C.c_int, [C.c_void_p, C.c_double]),
}


def jit_stats() -> dict:
    """Process-wide counters of the statement batches compiled for their shape (csrc/wsmc_jit.hip)."""
    st = (C.c_int64 * 5)()
    check(load_library().wsmc_debug_jit_stats(st))
    return {"compiled": st[0], "failed": st[1], "launched": st[2], "interpreted": st[3],
            "compile_s": st[4] / 1e6}


def mv_jit_stats() -> dict:
    """Process-wide counters of the Move blocks compiled for their shape (csrc/wsmc_mv_body.h)."""
    st = (C.c_int64 * 5)()
    check(load_library().wsmc_debug_mv_jit_stats(st))
    return {"compiled": st[0], "failed": st[1], "launched": st[2], "interpreted": st[3],
            "compile_s": st[4] / 1e6}


# int exchange(void* user, const uint64_t* mine, int32_t words, uint64_t* all)
EXCHANGE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_uint64), C.c_int32, C.POINTER(C.c_uint64))


class WSMCError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"wsmc error {code}: {msg}")
        self.code = code


_lib = None


def load_library(path: os.PathLike | None = None) -> C.CDLL:
    """Load libwsmc.so and bind every signature. Raises if it is absent (no fallback)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    # WSMC_LIB: an alternative build of the same library (block-size experiments, tools/)
    p = pathlib.Path(path) if path is not None else pathlib.Path(os.environ.get("WSMC_LIB", LIB_PATH))
    if not p.exists():
        raise ImportError(
            f"{p} not found: the HIP library is required (build it with "
            f"`python weightedsampling.jl_amd/build.py` or __graft_entry__.build()); "
            f"there is no CPU fallback")
    lib = C.CDLL(str(p), mode=C.RTLD_GLOBAL)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _lib = lib
    return lib


def check(code: int) -> None:
    if code != WSMC_OK:
        msg = load_library().wsmc_last_error()
        raise WSMCError(code, msg.decode() if msg else "")
