"""Torch-free host rendezvous for one-process-per-GPU runs on one node.

The device data path between ranks is RCCL inside libwsmc (ncclAllGather of the per-step
shard statistics). The host only needs to hand out the RCCL unique id, run barriers and
take the max of the timings. That is done here over TCP so that a rank process never
imports torch: torch bundles its own HIP/HSA runtime, and two HIP runtimes in one process
(torch's and the ROCm one libwsmc links) abort at exit.

Launch with `python -m torch.distributed.run ...` (the launcher process uses torch; the
ranks read RANK / WORLD_SIZE / MASTER_PORT from the environment). The ranks of one job
share a node, so rank 0 listens on the loopback interface only (MASTER_PORT + 1 + k, the
first free k < 16); the other ranks find it by a fixed-size handshake carrying a magic and
a job tag, checked before anything else is read. Payloads use a plain tagged encoding
(no pickle).
"""
from __future__ import annotations

import os
import socket
import struct
import time

_MAGIC = b"WSMCRDZV2"
_HELLO = struct.Struct("<9s32sI")          # magic, job tag (padded), rank
_MAX_MSG = 1 << 30
_HANDSHAKE_S = 5.0                         # a listener that is not our rank 0 must not stall the scan


# Messages are a small tagged binary encoding of the values the ranks exchange (None,
# bool, int, float, bytes, str and lists / tuples of them); nothing received is ever
# unpickled or executed.
def _enc(obj, out: bytearray) -> None:
    if obj is None:
        out += b"N"
    elif isinstance(obj, bool):
        out += b"T" if obj else b"F"
    elif isinstance(obj, int):
        out += b"I" + struct.pack("<q", obj)
    elif isinstance(obj, float):
        out += b"D" + struct.pack("<d", obj)
    elif isinstance(obj, (bytes, bytearray)):
        out += b"B" + struct.pack("<Q", len(obj)) + bytes(obj)
    elif isinstance(obj, str):
        b = obj.encode()
        out += b"S" + struct.pack("<Q", len(b)) + b
    elif isinstance(obj, (list, tuple)):
        out += b"L" + struct.pack("<Q", len(obj))
        for x in obj:
            _enc(x, out)
    else:
        raise TypeError(f"hostcomm cannot send {type(obj).__name__}")


def _dec(buf: bytes, i: int = 0):
    t = buf[i:i + 1]
    i += 1
    if t == b"N":
        return None, i
    if t in (b"T", b"F"):
        return t == b"T", i
    if t == b"I":
        return struct.unpack_from("<q", buf, i)[0], i + 8
    if t == b"D":
        return struct.unpack_from("<d", buf, i)[0], i + 8
    if t in (b"B", b"S"):
        (n,) = struct.unpack_from("<Q", buf, i)
        i += 8
        if i + n > len(buf):
            raise ValueError("truncated message")
        v = buf[i:i + n]
        return (v if t == b"B" else v.decode()), i + n
    if t == b"L":
        (n,) = struct.unpack_from("<Q", buf, i)
        i += 8
        if n > len(buf):
            raise ValueError("bad list length")
        out = []
        for _ in range(n):
            x, i = _dec(buf, i)
            out.append(x)
        return out, i
    raise ValueError("bad message tag")


def _send(sock, obj):
    data = bytearray()
    _enc(obj, data)
    sock.sendall(struct.pack("<Q", len(data)) + bytes(data))


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
    if n > _MAX_MSG:
        raise ValueError("message too large")
    obj, i = _dec(_recv_exact(sock, n))
    if i != n:
        raise ValueError("trailing bytes in message")
    return obj


def _job_tag(tag: str) -> bytes:
    # unique per job by default: two jobs on one node do not join each other's rendezvous
    t = tag or os.environ.get("TORCHELASTIC_RUN_ID", "") or f"wsmc-{os.environ.get('MASTER_PORT', '')}"
    return t.encode()[:32]


class HostComm:
    """allgather / barrier / broadcast / max over TCP between the ranks of one job."""

    def __init__(self, rank: int, world: int, addr: str = "127.0.0.1", port: int = 29500,
                 tag: str = "", timeout: float = 120.0):
        self.rank, self.world = int(rank), int(world)
        self.tag = _job_tag(tag)
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
                # the server speaks first (a client that gave up while the connection waited in
                # the backlog sent nothing and is skipped here), then the client's hello, then
                # the acknowledgement; a rank that reconnects replaces its earlier connection
                conn.settimeout(_HANDSHAKE_S)
                try:
                    conn.sendall(_MAGIC)
                    magic, tag, r = _HELLO.unpack(_recv_exact(conn, _HELLO.size))
                except (OSError, ConnectionError, struct.error):
                    conn.close()
                    continue
                if magic != _MAGIC or tag.rstrip(b"\0") != self.tag or not 0 < r < self.world:
                    conn.close()
                    continue
                try:
                    conn.sendall(_MAGIC)
                except (OSError, ConnectionError):
                    conn.close()
                    continue
                if r in got:
                    got[r].close()
                got[r] = conn
                conn.settimeout(timeout)
            srv.close()
            self.peers = [got[r] for r in range(1, self.world)]
        else:
            while True:
                for k in range(16):
                    s = None
                    try:
                        s = socket.create_connection((addr, port + 1 + k), timeout=2.0)
                        # another process's listener on a scanned port (e.g. an RCCL bootstrap
                        # socket) does not greet: give up on it quickly and go on scanning
                        s.settimeout(_HANDSHAKE_S)
                        if _recv_exact(s, len(_MAGIC)) != _MAGIC:
                            s.close()
                            continue
                        s.sendall(_HELLO.pack(_MAGIC, self.tag, self.rank))
                        s.settimeout(max(1.0, deadline - time.time()))
                        if _recv_exact(s, len(_MAGIC)) == _MAGIC:
                            s.settimeout(timeout)
                            self.sock = s
                            break
                        s.close()
                    except (OSError, ConnectionError):
                        if s is not None:
                            s.close()
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
    """The ranks of one single-node job (torch.distributed.run): rank 0 listens on loopback.
    A job spread over several nodes cannot rendezvous here: WORLD_SIZE != LOCAL_WORLD_SIZE
    says so, and fails at once instead of waiting for the timeout. MASTER_ADDR is not
    consulted: on one node every rank reaches rank 0 through 127.0.0.1 whatever name the
    launcher exported (torch.distributed.run --standalone exports the host's FQDN)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    if world != local_world:
        raise RuntimeError(f"hostcomm serves one node: WORLD_SIZE {world} != LOCAL_WORLD_SIZE {local_world}")
    return HostComm(int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
                    "127.0.0.1", int(os.environ.get("MASTER_PORT", "29500")), timeout=timeout)
