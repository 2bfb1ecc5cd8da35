"""Connection sharding across GPUs: one process per GPU,
connections dealt round-robin (`conn_id % world == rank`), no collective on
the data path (a connection's records are serial: tlsrecordlayer.py:27-37,
python_aes.py:44, so the connection is the shard unit).

The ranks only meet for the bench's start/stop barriers, the max-over-ranks /
sum-over-ranks of its timing numbers and a gather of check digests.  That is
done by a small TCP rendezvous of our own (no PyTorch, no RCCL): rank 0 serves
`MASTER_ADDR:(MASTER_PORT + 1)` -- `torch.distributed.run` keeps its own store on
MASTER_PORT itself -- (or `TLSGPU_RDZV_PORT`), every other rank connects, and
each collective is an all-gather of byte strings through rank 0.

A rank's hello carries a shared token (`job_token()`: TLSGPU_RDZV_TOKEN, which bench.py's
own rank spawner sets to a random value; else torch.distributed.run's TORCHELASTIC_RUN_ID;
torchrun sets that to the constant "none" unless --rdzv-id / --standalone is given, and then a
single-node job's token is derived from MASTER_ADDR:MASTER_PORT and the launcher's PID, the
parent of every local rank): rank 0 drops connections that do not present it.  The token
keeps stray and foreign processes out; it is not authentication against a local process
that reads the ranks' environment.  Sockets keep a finite timeout after set-up, so a
rank that hangs ends the others with an error instead of blocking them forever."""
import errno
import os
import socket
import struct
import time

import numpy as np


def shard_indices(n, rank, world):
    """Connections owned by `rank`: round-robin, so every rank gets the same
    count +-1 and the byte load is balanced for equal-size connections."""
    return np.arange(rank, n, world, dtype=np.int64)


def device_for_rank(local_rank, device_count):
    """The GPU a rank drives: one process per GPU (`local_rank % count`), so on a
    node with fewer GPUs than ranks the ranks share devices round-robin."""
    return int(local_rank) % max(int(device_count), 1)


def _send(sock, b):
    sock.sendall(struct.pack("<Q", len(b)) + b)


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
    return _recv_exact(sock, n)


def job_token(env=None, ppid=None):
    """The rendezvous token all ranks of one job share (module docstring)."""
    env = os.environ if env is None else env
    tok = env.get("TLSGPU_RDZV_TOKEN")
    if tok:
        return tok
    run_id = env.get("TORCHELASTIC_RUN_ID") or ""
    if run_id and run_id != "none":
        return run_id
    if run_id == "none" and env.get("LOCAL_WORLD_SIZE") and env.get("LOCAL_WORLD_SIZE") == env.get("WORLD_SIZE"):
        # torch.distributed.run without --rdzv-id on one node: every rank is a child of the agent
        return "%s:%s:%d" % (env.get("MASTER_ADDR", ""), env.get("MASTER_PORT", ""),
                             os.getppid() if ppid is None else ppid)
    return run_id


class ShardGroup:
    """RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR / MASTER_PORT from the
    environment (as torch.distributed.run sets them); world size 1 needs none."""

    def __init__(self, timeout=120.0, op_timeout=900.0):
        self.rank = int(os.environ.get("RANK", "0"))
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.local = int(os.environ.get("LOCAL_RANK", str(self.rank)))
        self._peers = []   # rank 0: sockets of ranks 1..world-1 in rank order
        self._sock = None  # rank > 0: socket to rank 0
        if self.world <= 1:
            return
        addr = os.environ.get("MASTER_ADDR", "127.0.0.1")
        port = int(os.environ.get("TLSGPU_RDZV_PORT", int(os.environ.get("MASTER_PORT", "29500")) + 1))
        token = job_token().encode()[:255]
        deadline = time.monotonic() + timeout
        if self.rank == 0:
            srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            try:
                srv.bind((addr, port))
            except OSError as e:
                if e.errno == errno.EADDRINUSE:
                    raise RuntimeError("rendezvous: %s:%d is in use (MASTER_PORT + 1 by default); set TLSGPU_RDZV_PORT "
                                       "to a free port" % (addr, port)) from e
                raise
            srv.listen(self.world + 4)
            by_rank = {}
            while len(by_rank) < self.world - 1:
                left = deadline - time.monotonic()
                if left <= 0:
                    raise TimeoutError("rendezvous: %d of %d ranks joined" % (len(by_rank) + 1, self.world))
                srv.settimeout(left)
                c, _ = srv.accept()
                c.settimeout(10.0)
                try:
                    (r, n) = struct.unpack("<IB", _recv_exact(c, 5))
                    tok = _recv_exact(c, n) if n else b""
                except (OSError, ConnectionError, struct.error):
                    c.close()
                    continue
                if tok != token:  # not one of this job's ranks
                    c.close()
                    continue
                if r in by_rank or not 0 < r < self.world:
                    raise RuntimeError("rendezvous: unexpected rank %d" % r)
                c.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                c.settimeout(op_timeout)
                by_rank[r] = c
            srv.close()
            self._peers = [by_rank[r] for r in range(1, self.world)]
        else:
            while True:
                try:
                    s = socket.create_connection((addr, port), timeout=5.0)
                    break
                except OSError:
                    if time.monotonic() > deadline:
                        raise
                    time.sleep(0.05)
            s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            s.settimeout(op_timeout)
            s.sendall(struct.pack("<IB", self.rank, len(token)) + token)
            self._sock = s

    def all_gather(self, b):
        """Every rank's byte string, in rank order, on every rank."""
        b = bytes(b)
        if self.world <= 1:
            return [b]
        if self.rank == 0:
            parts = [b] + [_recv(c) for c in self._peers]
            blob = struct.pack("<I", len(parts)) + b"".join(struct.pack("<Q", len(p)) + p for p in parts)
            for c in self._peers:
                _send(c, blob)
            return parts
        _send(self._sock, b)
        blob = _recv(self._sock)
        (n,) = struct.unpack_from("<I", blob, 0)
        out, off = [], 4
        for _ in range(n):
            (L,) = struct.unpack_from("<Q", blob, off)
            out.append(blob[off + 8:off + 8 + L])
            off += 8 + L
        return out

    def barrier(self):
        self.all_gather(b"")

    def max(self, x):
        return max(struct.unpack("<d", p)[0] for p in self.all_gather(struct.pack("<d", float(x))))

    def sum(self, x):
        return float(sum(struct.unpack("<d", p)[0] for p in self.all_gather(struct.pack("<d", float(x)))))

    def gather_bytes(self, b):
        """All ranks' byte strings (rank order); for checks only."""
        return self.all_gather(b)

    def close(self):
        if self.world > 1 and (self._peers or self._sock):
            self.barrier()
        for c in self._peers:
            c.close()
        if self._sock:
            self._sock.close()
        self._peers, self._sock = [], None
