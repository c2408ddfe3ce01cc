"""Multi-process (world_size 2) CPU tests of the N > 1 path.

1. The island-resampling protocol over torch.distributed (gloo): each rank owns one
   shard (an oracle shard with its global offset), exchanges the 8-word shard record per
   Resample with all_gather, and applies the global decision locally — exactly what the
   GPU ranks do with ncclAllGather inside libwsmc. The result must equal the
   single-process run with the same shard layout, bit for bit.
2. The sharded autoRW protocol: global max, per-rank canonical moment totals exchanged
   and combined in rank order, the factor on every rank, the move applied locally — the
   sequence libwsmc's sharded Move runs over RCCL.
3. Exact sharding: global max, integer record sums, the shard's window of global slots,
   the particles moved to their owners — the device ranks' WSMC_SHARD_EXACT protocol.
   Two gloo ranks must reproduce the unsharded oracle bit for bit.
4. The torch-free TCP rendezvous bench.py ranks use (wsmc.hostcomm).
"""
import os
import pathlib
import socket
import sys

import numpy as np
import pytest

REPO = pathlib.Path(__file__).resolve().parents[1]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _spawn(fn, nprocs, args, timeout=300):
    # stdlib spawn: the test process itself never imports torch (its bundled HIP runtime
    # must not share a process with libwsmc, which other tests load)
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    ps = [ctx.Process(target=fn, args=(r,) + tuple(args)) for r in range(nprocs)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(timeout)
    codes = [p.exitcode for p in ps]
    for p in ps:
        if p.is_alive():
            p.kill()
    assert codes == [0] * nprocs, codes


class ShardCtx:
    """Context-protocol adapter: an oracle shard whose resample() exchanges records."""

    def __init__(self, oracle, exchange, rank, global_n=None):
        self.o, self.exchange, self.rank = oracle, exchange, rank
        self.gN = global_n

    def __getattr__(self, k):
        return getattr(self.o, k)

    def resample(self, ess_perc_min, scheme=0, wait=True):
        recs = self.exchange(self.o.shard_record())
        r = self.o.resample_records(ess_perc_min, scheme, np.stack(recs), self.rank)
        return r if wait else None

    def _global_unique(self, col):
        x = self.o.col_download(col)
        keys = np.unique(np.where(np.isnan(x), np.nan, x).view(np.uint64))   # canonical NaN, bitwise
        counts = [int(c[0]) for c in self.exchange(np.array([len(keys)], dtype=np.uint64))]
        pad = np.zeros(max(max(counts), 1), dtype=np.uint64)
        pad[:len(keys)] = keys
        parts = self.exchange(pad)
        return len(np.unique(np.concatenate([p[:c] for p, c in zip(parts, counts)])))

    def _allgather_f64(self, vals):
        words = np.ascontiguousarray(np.asarray(vals, float)).view(np.uint64)
        return [r.view(np.float64) for r in self.exchange(words)]

    def move(self, proposal, targets, step, lo=None, hi=None, target_depth=-1, diversity=float("nan"), wait=True):
        acc = self._move(proposal, targets, step, lo, hi, target_depth, diversity)
        return acc if wait else None

    def move_block(self, moves, gated=False, wait=False):
        """wsmc_move_block: the block's Moves one after the other, each through the protocol"""
        out = []
        for mv in moves:
            lo = mv[3] if len(mv) > 3 else None
            hi = mv[4] if len(mv) > 4 else None
            depth = mv[5] if len(mv) > 5 else -1
            out.append(self._move(mv[0], mv[1], mv[2], lo, hi, depth))
        return out if wait else None

    def _move(self, proposal, targets, step, lo=None, hi=None, target_depth=-1, diversity=float("nan")):
        import math
        from wsmc import abi
        if not math.isnan(diversity):
            # the gate's population-wide unique count (the device's
            # global_unique): counts, then every rank's unique keys padded to the largest
            # count, all-gathered; every rank counts the union
            div = min(self._global_unique(t) for t in targets) / self.gN
            if div >= diversity:
                # skip exactly as the shard itself would: same op-counter consumption
                return self.o.move(proposal, targets, step, lo, hi, target_depth, diversity=-math.inf)
        if proposal != abi.PROPOSAL_AUTORW:
            return self.o.move(proposal, targets, step, lo, hi, target_depth)
        d = len(targets)
        bounded = any(math.isfinite(b) for bb in (lo or [], hi or []) for b in bb)
        lo, hi = (lo, hi) if bounded else (None, None)
        # global max (NaN if any rank holds a NaN weight, as the device's ordered max)
        w = self.o.weights_download()
        m = np.array([np.nan if np.isnan(w).any() else (w.max() if len(w) else -np.inf)])
        ms = np.concatenate(self._allgather_f64(m))
        M = np.nan if np.isnan(ms).any() else float(ms.max())

        def rank_order_sum(parts):
            acc = parts[0].copy()
            for x in parts[1:]:
                acc = acc + x
            return acc
        # the pivot: rank 0's particle 0 (all-gathered with the max on the device)
        pivot = self._allgather_f64(self.o.autorw_pivot(targets, lo, hi))[0]
        tot = rank_order_sum(self._allgather_f64(self.o.moment_totals(targets, M, pivot, lo=lo, hi=hi)))
        L = self.o.factor(tot, d, step)
        if L is None:
            self.o.skip_move()
            raise np.linalg.LinAlgError("proposal covariance not positive definite")
        return self.o.move_factor(targets, L, lo, hi, target_depth)


def _gloo_worker(rank, world, port, N, T, ess, scheme, outdir):
    sys.path[:0] = [str(REPO / "weightedsampling.jl_amd"), str(REPO / "oracle")]
    import torch
    import torch.distributed as dist
    from oracle import Oracle, log_evidence_records
    import wsmc
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def exchange(rec):
        t = torch.from_numpy(rec.view(np.int64).copy())
        out = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(out, t)
        return [o.numpy().view(np.uint64) for o in out]

    n = N // world
    o = Oracle(n, seed=11, global_offset=rank * n)
    ctx = ShardCtx(o, exchange, rank)
    obs = wsmc.models.ssm2d_data(T)
    flags = wsmc.models.ssm2d_statements(ctx, obs, ess_perc_min=ess, scheme=scheme)
    ev = log_evidence_records(np.stack(exchange(o.shard_record())))
    cols = {name: o.col_download(o.col_find(name)) for name in o.col_names()}
    np.savez(os.path.join(outdir, f"rank{rank}.npz"), w=o.weights_download(), flags=np.array(flags),
             ev=np.array([ev]), **{k.replace("_", "U"): v for k, v in cols.items()})
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("ess,scheme", [(1.0, 0), (0.5, 1), (1.0, 2)])
def test_island_protocol_gloo_world2(tmp_path, ess, scheme):
    from oracle import Oracle
    import wsmc
    N, T, world = 4096, 10, 2
    _spawn(_gloo_worker, world, (world, _free_port(), N, T, ess, scheme, str(tmp_path)))
    ref = Oracle(N, seed=11, shards=world)
    flags = wsmc.models.ssm2d_statements(ref, wsmc.models.ssm2d_data(T), ess_perc_min=ess, scheme=scheme)
    parts = [np.load(tmp_path / f"rank{r}.npz") for r in range(world)]
    n = N // world
    for r, p in enumerate(parts):
        assert list(p["flags"]) == flags
        np.testing.assert_array_equal(p["w"], ref.weights_download()[r * n:(r + 1) * n])
        for name in ref.col_names():
            full = ref.col_download(ref.col_find(name))
            np.testing.assert_array_equal(p[name.replace("_", "U")], full[..., r * n:(r + 1) * n])
        assert p["ev"][0] == ref.log_evidence()


def _move_worker(rank, world, port, N, which, outdir):
    sys.path[:0] = [str(REPO / "weightedsampling.jl_amd"), str(REPO / "oracle")]
    import torch
    import torch.distributed as dist
    from oracle import Oracle
    import wsmc
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def exchange(rec):
        t = torch.from_numpy(np.ascontiguousarray(rec).view(np.int64).copy())
        out = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(out, t)
        return [o.numpy().view(np.uint64) for o in out]

    n = N // world
    o = Oracle(n, seed=33, global_offset=rank * n)
    ctx = ShardCtx(o, exchange, rank, global_n=N)
    acc = _move_program(ctx, which)
    cols = {"c_" + name: o.col_download(o.col_find(name)) for name in o.col_names()}
    np.savez(os.path.join(outdir, f"mv{rank}.npz"), acc=np.array(acc), w=o.weights_download(), **cols)
    dist.barrier()
    dist.destroy_process_group()


def _move_program(ctx, which):
    import wsmc
    if which == "c3":
        xs, ys = wsmc.models.linreg_data()
        return wsmc.models.linreg_statements(ctx, xs[:6], ys[:6], ess_perc_min=1.0)
    if which == "c5g":   # the example's gated moves (ess 0.5); at 0.7 the gate both skips and runs
        t, y = wsmc.models.oscillator_data(n=8)
        return wsmc.models.oscillator_statements(ctx, t, y, ess_perc_min=0.5, sweeps=2, diversity=0.7)
    t, y = wsmc.models.oscillator_data(n=4)
    return wsmc.models.oscillator_statements(ctx, t, y, ess_perc_min=1.0, scheme=wsmc.RESAMPLE_SYSTEMATIC,
                                             sweeps=2, diversity=None)


@pytest.mark.parametrize("which", ["c3", "c5", "c5g"])
def test_sharded_autorw_protocol_gloo_world2(tmp_path, which):
    """C3 (1-d autoRW) and C5 (bounded 4-d + 1-d autoRW) on two gloo ranks == the sharded oracle."""
    from oracle import Oracle
    N, world = 3002, 2
    _spawn(_move_worker, world, (world, _free_port(), N, which, str(tmp_path)))
    ref = Oracle(N, seed=33, shards=world)
    acc = _move_program(ref, which)
    n = N // world
    parts = [np.load(tmp_path / f"mv{r}.npz") for r in range(world)]
    np.testing.assert_array_equal(sum(p["acc"] for p in parts), np.array(acc))
    for r, p in enumerate(parts):
        sl = slice(r * n, (r + 1) * n)
        np.testing.assert_array_equal(p["w"], ref.weights_download()[sl])
        for name in ref.col_names():
            np.testing.assert_array_equal(p["c_" + name], ref.col_download(ref.col_find(name))[..., sl],
                                          err_msg=name)


class ExactShardCtx(ShardCtx):
    """Context-protocol adapter: an oracle shard whose Resample / log_evidence follow the
    exact-sharding protocol (include/wsmc.h WSMC_SHARD_EXACT)."""

    def __init__(self, oracle, exchange, gather_obj, rank, world, goff, gN):
        super().__init__(oracle, exchange, rank)
        self.gather_obj, self.world, self.goff, self.gN = gather_obj, world, goff, gN
        self.last_anc = np.zeros(oracle.n, dtype=np.int32)

    def _records(self):
        from oracle import Oracle
        w = self.o.weights_download()
        m = np.nan if np.isnan(w).any() else float(w.max())
        ms = np.concatenate(self._allgather_f64(np.array([m])))
        M = np.nan if np.isnan(ms).any() else float(ms.max())
        recs = self.exchange(self.o.exact_record(M, self.gN))
        return M, recs, Oracle.combine_records(np.stack(recs))

    def log_evidence(self):
        from oracle import Oracle
        return Oracle.record_summary(self._records()[2])[2]

    def last_ancestors(self):
        return self.last_anc

    def resample(self, ess_perc_min, scheme=0, wait=True):
        r = self._resample(ess_perc_min, scheme)
        return r if wait else None

    def _resample(self, ess_perc_min, scheme=0):
        from oracle import Oracle
        st = self.o.get_state()
        op = st["op_counter"]
        self.o.set_op_counter(op + 1)                       # a Resample consumes one op, even a no-op
        if not st["weights_changed"]:
            return bool(st["resampled"]), st["last_ess_perc"]
        M, recs, comb = self._records()
        ess, mean, _ = Oracle.record_summary(comb)
        if not ess < ess_perc_min:
            self.o.set_resample_flags(False, False, ess)
            return False, ess
        Q = int(comb[1])
        cbase = sum(int(r[1]) for r in recs[:self.rank])
        a, b, anc = self.o.exact_window(M, self.gN, Q, cbase, scheme, op)
        names = self.o.col_names()
        data = {nm: self.o.col_download(self.o.col_find(nm))[..., anc] for nm in names}
        parts = self.gather_obj((a, b, data, self.goff + anc))
        lo, hi = self.goff, self.goff + self.o.n
        new = {nm: np.empty_like(self.o.col_download(self.o.col_find(nm))) for nm in names}
        gid = np.empty(self.o.n, dtype=np.int64)
        for pa, pb, pdata, pgid in parts:
            s0, s1 = max(pa, lo), min(pb, hi)
            if s1 <= s0:
                continue
            gid[s0 - lo:s1 - lo] = pgid[s0 - pa:s1 - pa]
            for nm in names:
                new[nm][..., s0 - lo:s1 - lo] = pdata[nm][..., s0 - pa:s1 - pa]
        for nm in names:
            self.o.col_upload(self.o.col_find(nm), new[nm])
        self.o.weights_upload(np.full(self.o.n, mean))
        self.o.set_resample_flags(True, False, ess)
        self.last_anc = gid.astype(np.int32)
        return True, ess


def _exact_worker(rank, world, port, sizes, T, ess, scheme, outdir):
    sys.path[:0] = [str(REPO / "weightedsampling.jl_amd"), str(REPO / "oracle")]
    import torch
    import torch.distributed as dist
    from oracle import Oracle
    import wsmc
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def exchange(rec):
        t = torch.from_numpy(np.ascontiguousarray(rec).view(np.int64).copy())
        out = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(out, t)
        return [o.numpy().view(np.uint64) for o in out]

    def gather_obj(obj):
        out = [None] * world
        dist.all_gather_object(out, obj)
        return out

    n, goff, N = sizes[rank], sum(sizes[:rank]), sum(sizes)
    o = Oracle(n, seed=13, global_offset=goff)
    ctx = ExactShardCtx(o, exchange, gather_obj, rank, world, goff, N)
    flags = wsmc.models.ssm2d_statements(ctx, wsmc.models.ssm2d_data(T), ess_perc_min=ess, scheme=scheme)
    ev = ctx.log_evidence()
    cols = {name: o.col_download(o.col_find(name)) for name in o.col_names()}
    np.savez(os.path.join(outdir, f"ex{rank}.npz"), w=o.weights_download(), flags=np.array(flags),
             anc=ctx.last_ancestors(), ev=np.array([ev]), **{k.replace("_", "U"): v for k, v in cols.items()})
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("sizes,ess,scheme", [((2048, 2048), 1.0, 0), ((3000, 1096), 0.5, 1)])
def test_exact_protocol_gloo_world2(tmp_path, sizes, ess, scheme):
    from oracle import Oracle
    import wsmc
    T, world = 8, len(sizes)
    _spawn(_exact_worker, world, (world, _free_port(), sizes, T, ess, scheme, str(tmp_path)))
    ref = Oracle(sum(sizes), seed=13)
    flags = wsmc.models.ssm2d_statements(ref, wsmc.models.ssm2d_data(T), ess_perc_min=ess, scheme=scheme)
    for r in range(world):
        p = np.load(tmp_path / f"ex{r}.npz")
        sl = slice(sum(sizes[:r]), sum(sizes[:r + 1]))
        assert list(p["flags"]) == flags
        np.testing.assert_array_equal(p["w"], ref.weights_download()[sl])
        np.testing.assert_array_equal(p["anc"], ref.last_ancestors()[sl])
        for name in ref.col_names():
            np.testing.assert_array_equal(p[name.replace("_", "U")], ref.col_download(ref.col_find(name))[..., sl],
                                          err_msg=name)
        assert p["ev"][0] == ref.log_evidence()


def _hostcomm_worker(rank, world, port, outdir):
    sys.path.insert(0, str(REPO / "weightedsampling.jl_amd"))
    from wsmc.hostcomm import HostComm
    c = HostComm(rank, world, "127.0.0.1", port, tag="t", timeout=60)
    uid = c.broadcast(b"x" * 128 if rank == 0 else None)
    c.barrier()
    m = c.max(float(rank) + 0.5)
    allv = c.allgather(rank * 10)
    c.close()
    with open(os.path.join(outdir, f"h{rank}.txt"), "w") as f:
        f.write(f"{len(uid)} {m} {allv}")


def test_hostcomm_world2(tmp_path):
    _spawn(_hostcomm_worker, 2, (2, _free_port(), str(tmp_path)))
    for r in range(2):
        assert (tmp_path / f"h{r}.txt").read_text() == "128 1.5 [0, 10]"
