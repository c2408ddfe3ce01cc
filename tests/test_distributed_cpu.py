"""Multi-process (world_size 2) CPU tests of the N > 1 path.

1. The island-resampling protocol over torch.distributed (gloo): each rank owns one
   shard (an oracle shard with its global offset), exchanges the 8-word shard record per
   Resample with all_gather, and applies the global decision locally — exactly what the
   GPU ranks do with ncclAllGather inside libwsmc. The result must equal the
   single-process run with the same shard layout, bit for bit.
2. The torch-free TCP rendezvous bench.py ranks use (wsmc.hostcomm).
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

    def __init__(self, oracle, exchange, rank):
        self.o, self.exchange, self.rank = oracle, exchange, rank

    def __getattr__(self, k):
        return getattr(self.o, k)

    def resample(self, ess_perc_min, scheme=0):
        recs = self.exchange(self.o.shard_record())
        return self.o.resample_records(ess_perc_min, scheme, np.stack(recs), self.rank)


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


@pytest.mark.parametrize("ess,scheme", [(1.0, 0), (0.5, 1)])
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
