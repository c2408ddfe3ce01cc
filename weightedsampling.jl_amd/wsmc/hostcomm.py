"""Torch-free host rendezvous for one-process-per-GPU runs on one node.

The device data path between ranks is RCCL inside libwsmc (ncclAllGather of the per-step
shard statistics). The host only needs to hand out the RCCL unique id, run barriers and
take the max of the timings. That is done here over TCP so that a rank process never
imports torch: torch bundles its own HIP/HSA runtime, and two HIP runtimes in one process
(torch's and the ROCm one libwsmc links) abort at exit.

Launch with `python -m torch.distributed.run ...` (the launcher process uses torch; the
ranks read RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT from the environment). Rank 0
listens on MASTER_PORT + 1 + k (the first free k < 16); the other ranks find it by a
handshake carrying a job tag.
"""
from __future__ import annotations

import os
import pickle
import socket
import struct
import time

_MAGIC = b"WSMCRDZV1"


def _send(sock, obj):
    data = pickle.dumps(obj)
    sock.sendall(struct.pack("<Q", len(data)) + data)


def _recv_exact(sock, n):
    buf = bytearray()
    while len(buf) < n:
        chunk = sock.recv(n - len(buf))
        if not chunk:
            raise ConnectionError("rendezvous peer closed the connection")
        buf += chunk
    return bytes(buf)


def _recv(sock):
    (n,) = struct.unpack("<Q", _recv_exact(sock, 8))
    return pickle.loads(_recv_exact(sock, n))


class HostComm:
    """allgather / barrier / broadcast / max over TCP between the ranks of one job."""

    def __init__(self, rank: int, world: int, addr: str = "127.0.0.1", port: int = 29500,
                 tag: str = "", timeout: float = 120.0):
        self.rank, self.world = int(rank), int(world)
        self.tag = (tag or os.environ.get("TORCHELASTIC_RUN_ID", "") or "wsmc").encode()
        self.peers = []
        self.sock = None
        if self.world == 1:
            return
        deadline = time.time() + timeout
        if self.rank == 0:
            srv = None
            for k in range(16):
                try:
                    s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
                    s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
                    s.bind((addr, port + 1 + k))
                    s.listen(self.world)
                    srv = s
                    break
                except OSError:
                    s.close()
            if srv is None:
                raise RuntimeError("no free rendezvous port")
            srv.settimeout(max(1.0, deadline - time.time()))
            got = {}
            while len(got) < self.world - 1:
                conn, _ = srv.accept()
                conn.settimeout(timeout)
                hello = _recv(conn)
                if not (isinstance(hello, tuple) and hello[0] == _MAGIC and hello[1] == self.tag):
                    conn.close()
                    continue
                got[int(hello[2])] = conn
                _send(conn, "ok")
            srv.close()
            self.peers = [got[r] for r in range(1, self.world)]
        else:
            while True:
                for k in range(16):
                    try:
                        s = socket.create_connection((addr, port + 1 + k), timeout=2.0)
                        s.settimeout(timeout)
                        _send(s, (_MAGIC, self.tag, self.rank))
                        if _recv(s) == "ok":
                            self.sock = s
                            break
                        s.close()
                    except (OSError, ConnectionError, EOFError, pickle.UnpicklingError):
                        continue
                if self.sock is not None:
                    break
                if time.time() > deadline:
                    raise TimeoutError("rendezvous with rank 0 timed out")
                time.sleep(0.2)

    def allgather(self, obj):
        if self.world == 1:
            return [obj]
        if self.rank == 0:
            out = [obj] + [_recv(p) for p in self.peers]
            for p in self.peers:
                _send(p, out)
            return out
        _send(self.sock, obj)
        return _recv(self.sock)

    def barrier(self) -> None:
        self.allgather(None)

    def broadcast(self, obj, src: int = 0):
        return self.allgather(obj if self.rank == src else None)[src]

    def max(self, x: float) -> float:
        return max(self.allgather(float(x)))

    def close(self) -> None:
        for p in self.peers:
            p.close()
        if self.sock is not None:
            self.sock.close()
        self.peers, self.sock = [], None


def from_env(timeout: float = 120.0) -> HostComm:
    return HostComm(int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
                    os.environ.get("MASTER_ADDR", "127.0.0.1"), int(os.environ.get("MASTER_PORT", "29500")),
                    timeout=timeout)
