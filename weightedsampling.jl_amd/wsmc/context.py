"""Low-level context: one particle shard on one GPU, driven through the C ABI.

Each method is a thin, typed wrapper of one include/wsmc.h entry point. The same method
set ("the context protocol") is what the high-level operators in ``transformers.py``
call, so they are agnostic of how a context is implemented; tests drive the CPU oracle
through the identical protocol to compare results bit for bit.
"""
from __future__ import annotations

import ctypes as C
import sys
import math

import numpy as np

from . import abi
from .abi import Dist, Operand, RunTiming, State, check, load_library

_D = C.POINTER(C.c_double)
_I32P = C.POINTER(C.c_int32)


def _dptr(a: np.ndarray):
    return a.ctypes.data_as(_D)


def _operands4(exprs) -> C.Array:
    ops = list(exprs) if isinstance(exprs, (list, tuple)) else [exprs]
    arr = (Operand * 4)()
    for k in range(4):
        arr[k] = ops[k] if k < len(ops) else ops[0]
    return arr


class Context:
    """A shard of ``n_particles`` particles on HIP device ``device`` (SMCState's storage)."""

    is_oracle = False

    def __init__(self, n_particles: int, seed: int = 42, device: int = 0):
        self._L = load_library()
        h = C.c_void_p()
        check(self._L.wsmc_create(C.byref(h), int(n_particles), int(device), int(seed) & (2**64 - 1)))
        self._h = h
        self.n = int(n_particles)
        self.seed = int(seed)
        self.device = int(device)
        self.world = 1
        self.rank = 0

    @classmethod
    def multi(cls, n_particles: int, n_gpus: int, seed: int = 42, devices=None,
              transport: int = abi.TRANSPORT_RCCL) -> "Context":
        """One handle over n_gpus shards (wsmc_create_multi): every call fans out to the
        shards; host arrays cover all n_particles."""
        self = cls.__new__(cls)
        self._L = load_library()
        h = C.c_void_p()
        devs = None
        if devices is not None:
            devs = (C.c_int32 * n_gpus)(*[int(d) for d in devices])
        check(self._L.wsmc_create_multi(C.byref(h), int(n_particles), int(n_gpus),
                                        C.cast(devs, _I32P) if devs is not None else None,
                                        int(seed) & (2**64 - 1), int(transport)))
        self._h = h
        self.n = int(n_particles)
        self.seed = int(seed)
        self.device = int(devices[0]) if devices is not None else 0
        self.world = 1
        self.rank = 0
        return self

    # ---- lifetime ----
    def close(self) -> None:
        if getattr(self, "_h", None):
            self._L.wsmc_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def sync(self) -> None:
        check(self._L.wsmc_sync(self._h))

    # ---- multi-GPU ----
    @staticmethod
    def comm_unique_id() -> bytes:
        buf = (C.c_uint8 * 128)()
        check(load_library().wsmc_comm_unique_id(buf))
        return bytes(buf)

    def comm_init(self, uid: bytes, world: int, rank: int, global_offset: int, global_n: int) -> None:
        buf = (C.c_uint8 * 128).from_buffer_copy(uid)
        check(self._L.wsmc_comm_init(self._h, buf, int(world), int(rank), int(global_offset), int(global_n)))
        self.world, self.rank = int(world), int(rank)

    def comm_init_host(self, allgather, world: int, rank: int, global_offset: int, global_n: int) -> None:
        """Shard this context with a host-side record exchange: ``allgather(list_of_u64)`` must
        return every rank's list in rank order (e.g. wsmc.hostcomm.HostComm.allgather)."""
        def _exchange(_user, mine, words, out):
            try:
                nb = 8 * int(words)
                recs = allgather(C.string_at(mine, nb))        # raw u64 words of this rank
                for r, rec in enumerate(recs):
                    if len(rec) != nb:   # the ranks are at different exchanges: a desync
                        sys.stderr.write(f"wsmc host exchange: rank {rank} sent {nb} B, rank {r} {len(rec)} B\n")
                        return 1
                    C.memmove(C.addressof(out.contents) + r * nb, rec, nb)
                return 0
            except Exception as e:   # the reason goes to stderr; the ABI call fails with ERCCL
                sys.stderr.write(f"wsmc host exchange: rank {rank}: {type(e).__name__}: {e}\n")
                return 1
        self._exchange_cb = abi.EXCHANGE_FN(_exchange)   # keep alive as long as the context
        check(self._L.wsmc_comm_init_host(self._h, C.cast(self._exchange_cb, C.c_void_p), None, int(world),
                                          int(rank), int(global_offset), int(global_n)))
        self.world, self.rank = int(world), int(rank)

    def comm_set_timeout(self, seconds: float) -> None:
        """wsmc_comm_set_timeout: abort the communicator when a stream wait exceeds `seconds`."""
        check(self._L.wsmc_comm_set_timeout(self._h, float(seconds)))

    def comm_info(self) -> dict:
        """wsmc_comm_info: shards, world/rank, the RCCL communicator's own rank count
        (ncclCommCount), transport, shard mode, and each shard's device and size."""
        ci = abi.CommInfo()
        check(self._L.wsmc_comm_info(self._h, C.byref(ci)))
        k = min(int(ci.shards), 8)
        return {"shards": int(ci.shards), "world": int(ci.world), "rank": int(ci.rank),
                "rccl_ranks": int(ci.rccl_ranks),
                "transport": {abi.TRANSPORT_RCCL: "rccl", abi.TRANSPORT_HOST: "host"}.get(int(ci.transport), "none"),
                "shard_mode": "exact" if ci.shard_mode == abi.SHARD_EXACT else "island",
                "devices": [int(ci.devices[g]) for g in range(k)],
                "shard_n": [int(ci.shard_n[g]) for g in range(k)]}

    @staticmethod
    def device_count() -> int:
        n = C.c_int32()
        check(load_library().wsmc_device_count(C.byref(n)))
        return int(n.value)

    def comm_set_shard_mode(self, mode: int) -> None:
        """abi.SHARD_ISLAND (default) or abi.SHARD_EXACT: sharded Resample over the whole
        population, bit-identical to one context holding every particle (include/wsmc.h)."""
        check(self._L.wsmc_comm_set_shard_mode(self._h, int(mode)))

    # ---- store (AbstractParticleStore) ----
    def col_find(self, name: str) -> int:
        c = C.c_int32()
        check(self._L.wsmc_col_find(self._h, name.encode(), C.byref(c)))
        return int(c.value)

    def col_create(self, name: str, dim: int = 1) -> int:
        c = C.c_int32()
        check(self._L.wsmc_col_create(self._h, name.encode(), int(dim), C.byref(c)))
        return int(c.value)

    def col_dim(self, col: int) -> int:
        d = C.c_int32()
        check(self._L.wsmc_col_info(self._h, int(col), None, 0, C.byref(d)))
        return int(d.value)

    def col_names(self) -> list[str]:
        n = C.c_int32()
        check(self._L.wsmc_col_count(self._h, C.byref(n)))
        out = []
        buf = C.create_string_buffer(256)
        for k in range(n.value):
            check(self._L.wsmc_col_info(self._h, k, buf, 256, None))
            out.append(buf.value.decode())
        return out

    def col_download(self, col: int) -> np.ndarray:
        d = self.col_dim(col)
        a = np.empty(d * self.n)
        check(self._L.wsmc_col_download(self._h, int(col), _dptr(a)))
        return a.reshape(d, self.n) if d > 1 else a

    def col_upload(self, col: int, values) -> None:
        d = self.col_dim(col)
        v = np.ascontiguousarray(np.asarray(values, dtype=np.float64).reshape(d * self.n))
        check(self._L.wsmc_col_upload(self._h, int(col), _dptr(v)))

    def store_resample(self, indices) -> None:
        idx = np.ascontiguousarray(np.asarray(indices, dtype=np.int32))
        check(self._L.wsmc_store_resample(self._h, idx.ctypes.data_as(_I32P)))

    def store_set_lazy(self, lazy: bool) -> None:
        """Lazy genealogy (default) or the eager ColumnStore gather of every column."""
        check(self._L.wsmc_store_set_lazy(self._h, 1 if lazy else 0))

    def store_materialize(self) -> None:
        """Bring every column up to date (one trace over the Resample log)."""
        check(self._L.wsmc_store_materialize(self._h))

    def store_info(self) -> dict:
        e = C.c_int64()
        st = C.c_int32()
        check(self._L.wsmc_store_info(self._h, C.byref(e), C.byref(st)))
        return {"log_entries": e.value, "stale_columns": st.value}

    # ---- weights / state ----
    def weights_download(self) -> np.ndarray:
        a = np.empty(self.n)
        check(self._L.wsmc_weights_download(self._h, _dptr(a)))
        return a

    def weights_upload(self, w) -> None:
        a = np.ascontiguousarray(np.asarray(w, dtype=np.float64).reshape(self.n))
        check(self._L.wsmc_weights_upload(self._h, _dptr(a)))

    def log_evidence(self) -> float:
        v = C.c_double()
        check(self._L.wsmc_log_evidence(self._h, C.byref(v)))
        return float(v.value)

    # ---- analysis reductions (src/utils.jl) ----
    def weighted_moments(self, exprs, want_cov: bool = True):
        """Means (and uncorrected covariance) of up to 4 operand expressions under
        exp_norm(weights): expectation / @E and describe's mean / std."""
        ex = list(exprs) if isinstance(exprs, (list, tuple)) else [exprs]
        d = len(ex)
        arr = (Operand * 4)()
        for k in range(4):
            arr[k] = ex[k] if k < d else ex[0]
        mean = np.zeros(d)
        cov = np.zeros(d * d)
        check(self._L.wsmc_weighted_moments(self._h, arr, d, _dptr(mean), _dptr(cov) if want_cov else None))
        return mean, (cov.reshape(d, d) if want_cov else None)

    def col_minmax(self, col: int, comp: int = 0):
        mn, mx = C.c_double(), C.c_double()
        check(self._L.wsmc_col_minmax(self._h, int(col), int(comp), C.byref(mn), C.byref(mx)))
        return float(mn.value), float(mx.value)

    def ess(self) -> float:
        v = C.c_double()
        check(self._L.wsmc_ess(self._h, C.byref(v)))
        return float(v.value)

    def weighted_median(self, col: int, comp: int = 0) -> float:
        """StatsBase.quantile(v, Weights(w), 0.5) of a column component (describe's median)."""
        v = C.c_double()
        check(self._L.wsmc_weighted_median(self._h, int(col), int(comp), C.byref(v)))
        return float(v.value)

    def histogram(self, col: int, comp: int = 0) -> np.ndarray:
        """describe's 8-bin weighted sparkline as levels 1..8 (src/utils.jl:120-141)."""
        lv = np.zeros(8, dtype=np.int32)
        check(self._L.wsmc_histogram(self._h, int(col), int(comp), lv.ctypes.data_as(C.POINTER(C.c_int32))))
        return lv

    def sample_particles(self, n: int, replace: bool = True) -> np.ndarray:
        """sample(state, n; replace) indices (0-based), src/utils.jl:92-118."""
        out = np.zeros(max(int(n), 0), dtype=np.int64)
        check(self._L.wsmc_sample_particles(self._h, int(n), int(bool(replace)),
                                            out.ctypes.data_as(C.POINTER(C.c_int64))))
        return out

    def col_gather_rows(self, col: int, idx) -> np.ndarray:
        """getcol(store, c)[idx] on the device: [n] (scalar column) or [dim][n]."""
        ix = np.ascontiguousarray(np.asarray(idx, dtype=np.int64))
        dim = self.col_dim(col)
        out = np.zeros((dim, len(ix)))
        check(self._L.wsmc_col_gather_rows(self._h, int(col), ix.ctypes.data_as(C.POINTER(C.c_int64)), len(ix),
                                           _dptr(out)))
        return out[0] if dim == 1 else out

    def get_state(self) -> dict:
        s = State()
        check(self._L.wsmc_get_state(self._h, C.byref(s)))
        return dict(resampled=int(s.resampled), weights_changed=int(s.weights_changed), depth=int(s.depth),
                    n_terms=int(s.n_terms), last_ess_perc=float(s.last_ess_perc),
                    op_counter=int(s.op_counter), n_resamples=int(s.n_resamples))

    def set_depth(self, d: int) -> None:
        check(self._L.wsmc_set_depth(self._h, int(d)))

    def set_op_counter(self, op: int) -> None:
        check(self._L.wsmc_set_op_counter(self._h, int(op)))

    def last_ancestors(self) -> np.ndarray:
        a = np.empty(self.n, dtype=np.int32)
        check(self._L.wsmc_last_ancestors(self._h, a.ctypes.data_as(_I32P)))
        return a

    # ---- operators ----
    def assign(self, out: int, exprs) -> None:
        check(self._L.wsmc_assign(self._h, int(out), _operands4(exprs)))

    def assign_expr(self, out: int, prog, lens) -> None:
        """wsmc_assign_expr: prog a ctypes XInst array (wsmc.dsl.xprogram), lens the
        per-component program lengths"""
        ln = (C.c_int32 * 4)(*(list(lens) + [0] * (4 - len(lens))))
        check(self._L.wsmc_assign_expr(self._h, int(out), prog, ln))

    def sample(self, out: int, dist: Dist) -> None:
        check(self._L.wsmc_sample(self._h, int(out), C.byref(dist)))

    def sample_importance(self, out: int, proposal: Dist, target: Dist) -> None:
        check(self._L.wsmc_sample_importance(self._h, int(out), C.byref(proposal), C.byref(target)))

    def observe(self, dist: Dist, x) -> None:
        check(self._L.wsmc_observe(self._h, C.byref(dist), _operands4(x)))

    def weight(self, dist: Dist, x) -> None:
        check(self._L.wsmc_weight(self._h, C.byref(dist), _operands4(x)))

    def resample(self, ess_perc_min: float, scheme: int = abi.RESAMPLE_STRATIFIED, wait: bool = True):
        """Resample.apply!; returns (resampled, ESS%). wait=False leaves the decision on the
        device (no host round trip; the gather and weight reset are gated there) and returns
        None; get_state() folds it in later."""
        if not wait:
            check(self._L.wsmc_resample(self._h, float(ess_perc_min), int(scheme), None, None))
            return None
        r = C.c_int32()
        e = C.c_double()
        check(self._L.wsmc_resample(self._h, float(ess_perc_min), int(scheme), C.byref(r), C.byref(e)))
        return bool(r.value), float(e.value)

    def move(self, proposal: int, targets, step: float, lo=None, hi=None, target_depth: int = -1,
             diversity: float = math.nan, wait: bool = True):
        """Move.apply!; returns the accepted count. wait=False: asynchronous (returns None; a
        PosDefException surfaces at the next synchronizing call)."""
        t = np.ascontiguousarray(np.asarray(targets, dtype=np.int32))
        d = len(t)
        lo_a = None if lo is None else np.ascontiguousarray(np.asarray(lo, float).reshape(d))
        hi_a = None if hi is None else np.ascontiguousarray(np.asarray(hi, float).reshape(d))
        acc = C.c_int64()
        rc = self._L.wsmc_move(self._h, int(proposal), t.ctypes.data_as(_I32P), d, float(step),
                               None if lo_a is None else _dptr(lo_a), None if hi_a is None else _dptr(hi_a),
                               int(target_depth), float(diversity), C.byref(acc) if wait else None)
        if rc == abi.WSMC_ENOTPD:
            raise np.linalg.LinAlgError(self._L.wsmc_last_error().decode())
        check(rc)
        return int(acc.value) if wait else None

    def move_gated(self, proposal: int, targets, step: float, lo=None, hi=None, target_depth: int = -1,
                   diversity: float = math.nan) -> None:
        """Move.apply! inside `if resampled` decided on the device (wsmc_move_gated): runs only
        if the last Resample resampled; consumes its two op counters either way."""
        t = np.ascontiguousarray(np.asarray(targets, dtype=np.int32))
        d = len(t)
        lo_a = None if lo is None else np.ascontiguousarray(np.asarray(lo, float).reshape(d))
        hi_a = None if hi is None else np.ascontiguousarray(np.asarray(hi, float).reshape(d))
        rc = self._L.wsmc_move_gated(self._h, int(proposal), t.ctypes.data_as(_I32P), d, float(step),
                                     None if lo_a is None else _dptr(lo_a), None if hi_a is None else _dptr(hi_a),
                                     int(target_depth), float(diversity))
        if rc == abi.WSMC_ENOTPD:
            raise np.linalg.LinAlgError(self._L.wsmc_last_error().decode())
        check(rc)

    def move_block(self, moves, gated: bool = False, wait: bool = False):
        """A statement block of consecutive Moves (wsmc_move_block): `moves` is a list of
        (proposal, targets, step) or (proposal, targets, step, lo, hi[, target_depth]); the
        same results as calling move / move_gated for each in order. wait=True returns the
        accepted counts (a list), else None (asynchronous)."""
        n = len(moves)
        specs = (abi.MoveSpec * max(n, 1))()
        for m, mv in enumerate(moves):
            proposal, targets, step = mv[0], mv[1], mv[2]
            lo = mv[3] if len(mv) > 3 else None
            hi = mv[4] if len(mv) > 4 else None
            depth = mv[5] if len(mv) > 5 else -1
            t = [int(x) for x in np.asarray(targets).reshape(-1)]
            if not 1 <= len(t) <= 4:
                raise ValueError("a Move has 1..4 targets")
            sp = specs[m]
            sp.proposal, sp.d, sp.step, sp.target_depth = int(proposal), len(t), float(step), int(depth)
            sp.bounded = 0 if (lo is None and hi is None) else 1
            for k in range(4):
                sp.targets[k] = t[k] if k < len(t) else -1
                sp.lo[k] = float(lo[k]) if lo is not None and k < len(t) else -math.inf
                sp.hi[k] = float(hi[k]) if hi is not None and k < len(t) else math.inf
        acc = (C.c_int64 * max(n, 1))()
        rc = self._L.wsmc_move_block(self._h, n, specs, 1 if gated else 0, acc if wait else None)
        if rc == abi.WSMC_ENOTPD:
            raise np.linalg.LinAlgError(self._L.wsmc_last_error().decode())
        check(rc)
        return [int(acc[m]) for m in range(n)] if wait else None

    def score(self, target_depth: int) -> np.ndarray:
        out = np.empty(self.n)
        check(self._L.wsmc_score(self._h, int(target_depth), _dptr(out)))
        return out

    def marginal_diversity(self, targets) -> float:
        t = np.ascontiguousarray(np.asarray(targets, dtype=np.int32))
        v = C.c_double()
        check(self._L.wsmc_marginal_diversity(self._h, t.ctypes.data_as(_I32P), len(t), C.byref(v)))
        return float(v.value)

    # ---- fused runners ----
    def run_stats(self) -> dict:
        """The fused run's Resample statistics (wsmc_debug_run_stats): steps whose statistics
        were recomputed against the exact reference point (cumulative), and where they are taken."""
        st = (C.c_int64 * 4)()
        check(self._L.wsmc_debug_run_stats(self._h, st))
        return {"missed_steps": st[0], "qstat_mode": st[1], "replays": st[2], "batch_statistics": st[3]}

    def ssm2d_run(self, obs, x0=(0.0, 0.0), v0=(1.0, 0.0), q_var=0.1, r_var=0.5, ess_perc_min=0.5,
                  scheme: int = abi.RESAMPLE_STRATIFIED, keep_history: bool = True,
                  want_evidence: bool = True):
        o = np.ascontiguousarray(np.asarray(obs, dtype=np.float64).reshape(-1, 2))
        x0a = np.asarray(x0, dtype=np.float64)
        v0a = np.asarray(v0, dtype=np.float64)
        ev = C.c_double()
        check(self._L.wsmc_ssm2d_run(self._h, _dptr(o), len(o), _dptr(x0a), _dptr(v0a), float(q_var),
                                     float(r_var), float(ess_perc_min), int(scheme), int(bool(keep_history)),
                                     C.byref(ev) if want_evidence else None))
        return float(ev.value) if want_evidence else None

    def set_timing(self, enabled: bool) -> None:
        check(self._L.wsmc_run_set_timing(self._h, int(bool(enabled))))

    def debug_kernel_bench(self, kernel: int, mode: int = 0, iters: int = 50) -> float:
        v = C.c_double()
        check(self._L.wsmc_debug_kernel_bench(self._h, int(kernel), int(mode), int(iters), C.byref(v)))
        return float(v.value)

    def debug_exact(self, cap: int = -1, ctr: int = -1) -> dict:
        """Exact-sharded fused run: set the neighbour block / trace window sizes (> 0 sets, 0
        restores the defaults, < 0 keeps) and return the last run's statistics."""
        st = (C.c_int64 * 6)()
        check(self._L.wsmc_debug_exact(self._h, int(cap), int(ctr), st))
        return {"need": st[0], "excursion": st[1], "eager_reruns": st[2], "cap": st[3],
                "history_traces": st[4], "no_windows": st[5]}

    def debug_inject_failure(self, shard: int, nth: int) -> None:
        """Test hook: shard `shard` fails its nth next record exchange (include/wsmc.h)."""
        check(self._L.wsmc_debug_inject_failure(self._h, int(shard), int(nth)))

    def timing(self) -> dict:
        t = RunTiming()
        check(self._L.wsmc_run_get_timing(self._h, C.byref(t)))
        return {f: getattr(t, f) for f, _ in RunTiming._fields_}


def device_count() -> int:
    n = C.c_int32()
    check(load_library().wsmc_device_count(C.byref(n)))
    return int(n.value)
