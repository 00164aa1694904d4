"""Minimal RESP2 codec: the subset of mason-leap-lab/redeo/resp the InfiniCache
client uses on its per-shard connections.

Client side (/root/reference/client/ecRedis.go):
  * RequestWriter.WriteMultiBulkSize / WriteBulkString / CopyBulk  (set, :233-245)
  * RequestWriter.WriteCmdString                                   (get, :275-277)
  * ResponseReader.PeekType / ReadError / ReadBulkString / StreamBulk (rec, :292-363)
Proxy side (/root/reference/proxy/types/response.go:22-33): a reply is
bulk(reqId), bulk(chunkId | "-1"), [bulk(body)] — no body for "-1"; errors are
"-<message>\\r\\n".
"""
from __future__ import annotations

import socket
from typing import List, Optional, Union

TypeError_ = "-"
TypeBulk = "$"
TypeArray = "*"
TypeInline = "+"
TypeInt = ":"


class ProtocolError(Exception):
    pass


class Writer:
    """Buffered RESP writer over a socket (RequestWriter / ResponseWriter)."""

    def __init__(self, sock: socket.socket):
        self.sock = sock
        self.buf: List[bytes] = []

    def write_multi_bulk_size(self, n: int):
        self.buf.append(b"*%d\r\n" % n)

    def write_bulk(self, b: Union[bytes, bytearray, memoryview]):
        mv = memoryview(b).cast("B")
        self.buf.append(b"$%d\r\n" % len(mv))
        self.buf.append(mv)
        self.buf.append(b"\r\n")

    def write_bulk_string(self, s: str):
        self.write_bulk(s.encode())

    def write_cmd_string(self, *args: str):
        self.write_multi_bulk_size(len(args))
        for a in args:
            self.write_bulk_string(a)

    def write_error(self, msg: str):
        self.buf.append(b"-" + msg.encode() + b"\r\n")

    def flush(self):
        if self.buf:
            self.sock.sendall(b"".join(bytes(x) if isinstance(x, memoryview) else x for x in self.buf))
            self.buf = []


class Reader:
    """Buffered RESP reader over a socket (ResponseReader / command parser)."""

    def __init__(self, sock: socket.socket):
        self.sock = sock
        self.buf = bytearray()

    def _fill(self, n: int = 1):
        while len(self.buf) < n:
            chunk = self.sock.recv(max(65536, n - len(self.buf)))
            if not chunk:
                raise EOFError("connection closed")
            self.buf += chunk

    def _line(self) -> bytes:
        while True:
            i = self.buf.find(b"\r\n")
            if i >= 0:
                line = bytes(self.buf[:i])
                del self.buf[:i + 2]
                return line
            self._fill(len(self.buf) + 1)

    def peek_type(self) -> str:
        self._fill(1)
        return chr(self.buf[0])

    def read_error(self) -> str:
        line = self._line()
        if not line.startswith(b"-"):
            raise ProtocolError("expected error, got %r" % line[:16])
        return line[1:].decode()

    def read_bulk(self) -> Optional[bytes]:
        line = self._line()
        if not line.startswith(b"$"):
            raise ProtocolError("expected bulk, got %r" % line[:16])
        n = int(line[1:])
        if n < 0:
            return None
        self._fill(n + 2)
        data = bytes(self.buf[:n])
        if self.buf[n:n + 2] != b"\r\n":
            raise ProtocolError("bulk not terminated by CRLF")
        del self.buf[:n + 2]
        return data

    def read_bulk_string(self) -> str:
        b = self.read_bulk()
        return "" if b is None else b.decode()

    def read_array_size(self) -> int:
        line = self._line()
        if not line.startswith(b"*"):
            raise ProtocolError("expected array, got %r" % line[:16])
        return int(line[1:])

    def read_command(self) -> List[bytes]:
        """One client command: a multi-bulk array of bulk strings."""
        n = self.read_array_size()
        return [self.read_bulk() for _ in range(n)]
