"""The replicas' control plane without PyTorch: a star of TCP sockets.

Rank 0 listens on (MASTER_ADDR, control port) and every other rank connects once; each
message is an 8-byte little-endian length plus a JSON document.  It carries only small
host-side things — the RCCL unique id, the blob header (quantization parameters, a few
hundred KB), barriers and the max over ranks of the step time.  The device data path is
RCCL (nqk_comm_*).

The control port is NQK_CTRL_PORT, else MASTER_PORT + 1: under torchrun the agent's own
TCPStore already holds MASTER_PORT.
"""
from __future__ import annotations

import base64
import json
import os
import socket
import struct
import time

_LEN = struct.Struct("<Q")


def _send(sock: socket.socket, obj) -> None:
    data = json.dumps(obj, separators=(",", ":")).encode()
    sock.sendall(_LEN.pack(len(data)) + data)


def _recv_exact(sock: socket.socket, n: int) -> bytes:
    buf = bytearray()
    while len(buf) < n:
        chunk = sock.recv(min(n - len(buf), 1 << 20))
        if not chunk:
            raise ConnectionError("control plane: peer closed the connection")
        buf += chunk
    return bytes(buf)


_MAX_MSG = 64 << 20  # the largest control message (the blob header is a few hundred KiB)


def _recv(sock: socket.socket):
    (n,) = _LEN.unpack(_recv_exact(sock, _LEN.size))
    if n > _MAX_MSG:
        raise ConnectionError(f"control plane: message of {n} bytes exceeds the {_MAX_MSG}-byte limit")
    return json.loads(_recv_exact(sock, n))


def encode_bytes(b: bytes) -> dict:
    return {"__bytes__": base64.b64encode(b).decode()}


def decode_bytes(d) -> bytes:
    return base64.b64decode(d["__bytes__"])


class ControlPlane:
    """Star-topology control plane for `world` ranks (rank 0 is the hub)."""

    def __init__(self, rank: int, world: int, addr: str | None = None, port: int | None = None,
                 timeout: float = 600.0):
        self.rank, self.world = rank, world
        self.addr = addr or os.environ.get("MASTER_ADDR", "127.0.0.1")
        if port is None:
            port = int(os.environ.get("NQK_CTRL_PORT", int(os.environ.get("MASTER_PORT", "29500")) + 1))
        self.port = port
        self.peers: dict[int, socket.socket] = {}
        self.sock = None
        if world == 1:
            return
        if rank == 0:
            srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            srv.bind((self.addr, self.port))
            srv.listen(world)
            srv.settimeout(timeout)
            try:
                while len(self.peers) < world - 1:
                    conn, _ = srv.accept()
                    conn.settimeout(timeout)
                    conn.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                    try:
                        hello = _recv(conn)
                        r = hello["rank"] if isinstance(hello, dict) else None
                    except (ValueError, KeyError, ConnectionError) as ex:
                        conn.close()
                        raise ConnectionError(f"control plane: malformed first message from a peer ({ex})") from ex
                    if not isinstance(r, int) or not (0 < r < world) or r in self.peers:
                        conn.close()
                        raise ConnectionError(f"control plane: unexpected rank {r!r}")
                    self.peers[r] = conn
            finally:
                srv.close()
        else:
            deadline = time.time() + timeout
            while True:
                try:
                    s = socket.create_connection((self.addr, self.port), timeout=10)
                    break
                except OSError:
                    if time.time() > deadline:
                        raise
                    time.sleep(0.2)
            s.settimeout(timeout)
            s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            _send(s, {"rank": rank})
            self.sock = s

    def broadcast(self, obj, src: int = 0):
        """JSON-able `obj` of rank `src` to every rank (src must be 0: the hub)."""
        if self.world == 1:
            return obj
        if src != 0:
            raise ValueError("control plane: broadcasts come from rank 0")
        if self.rank == 0:
            for r in sorted(self.peers):
                _send(self.peers[r], obj)
            return obj
        return _recv(self.sock)

    def gather(self, obj) -> list | None:
        """Every rank's `obj` to rank 0 (a list in rank order); None elsewhere."""
        if self.world == 1:
            return [obj]
        if self.rank == 0:
            out = [obj] + [None] * (self.world - 1)
            for r in sorted(self.peers):
                out[r] = _recv(self.peers[r])
            return out
        _send(self.sock, obj)
        return None

    def allreduce_max(self, x: float) -> float:
        vals = self.gather(float(x))
        return float(self.broadcast(max(vals) if self.rank == 0 else None))

    def barrier(self) -> None:
        if self.world > 1:
            self.gather(0)
            self.broadcast(0 if self.rank == 0 else None)

    def close(self) -> None:
        for s in list(self.peers.values()) + ([self.sock] if self.sock else []):
            try:
                s.close()
            except OSError:
                pass
        self.peers, self.sock = {}, None
