"""Loopback stand-in for the InfiniCache proxy (test infrastructure).

Speaks the client-facing RESP protocol of /root/reference/proxy/server/proxy.go
(HandleSet :102-165, HandleGet :167-205) with an in-memory chunk store instead
of Lambda nodes, and reproduces the one proxy behaviour the codec depends on:
the first-d rule of proxy/lambdastore/connection.go:274-306 — of the d+p GET
responses of one request only the first d carry a body, the rest are sent as
chunkId "-1" (proxy/types/response.go:22-33), so every healthy EcGet hands
Client.decode exactly p nil shards at random positions.

Fault injection: `fail_chunks` answers GETs of those chunk ids with a RESP
error (the client's `failed` + recover path, ecRedis.go:161-188); `corrupt`
flips a byte of a stored chunk (Verify-after-Reconstruct failure path).
"""
from __future__ import annotations

import os
import random
import socket
import sys
import threading

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from infinicache_amd import resp  # noqa: E402


class FakeProxy:
    def __init__(self, host="127.0.0.1", port=0, seed=20200225):
        self.sock = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        self.sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        self.sock.bind((host, port))
        self.sock.listen(256)
        self.addr = "%s:%d" % self.sock.getsockname()
        self.store = {}          # (key, chunkId) -> bytes
        self.placement = {}      # (key, chunkId) -> lambdaId
        self.late = {}           # reqId -> set of late chunk ids
        self.rng = random.Random(seed)
        self.lock = threading.Lock()
        self.fail_chunks = set()
        self.force_late = None   # fixed late set for deterministic tests
        self.sets = 0
        self.gets = 0
        self._stop = False
        self._threads = []
        t = threading.Thread(target=self._accept, daemon=True)
        t.start()
        self._threads.append(t)

    def close(self):
        self._stop = True
        try:
            self.sock.close()
        except OSError:
            pass

    def corrupt(self, key, chunk_id, pos=0):
        with self.lock:
            b = bytearray(self.store[(key, str(chunk_id))])
            b[pos] ^= 0x01
            self.store[(key, str(chunk_id))] = bytes(b)

    def _accept(self):
        while not self._stop:
            try:
                c, _ = self.sock.accept()
            except OSError:
                return
            t = threading.Thread(target=self._serve, args=(c,), daemon=True)
            t.start()

    def _serve(self, c):
        r, w = resp.Reader(c), resp.Writer(c)
        try:
            while True:
                cmd = r.read_command()
                name = cmd[0].decode().lower()
                if name == "set":
                    self._set(cmd, w)
                elif name == "get":
                    self._get(cmd, w)
                else:
                    w.write_error("ERR unknown command '%s'" % name)
                w.flush()
        except (EOFError, OSError, resp.ProtocolError):
            c.close()

    def _set(self, cmd, w):
        # set key chunkId lambdaId randBase reqId dataChunks parityChunks <body>
        key, chunk, lambda_id, _rand, req = (x.decode() for x in cmd[1:6])
        body = cmd[8]
        with self.lock:
            self.store[(key, chunk)] = body
            self.placement[(key, chunk)] = lambda_id
            self.sets += 1
        w.write_bulk_string(req)
        w.write_bulk_string(chunk)
        w.write_bulk_string(lambda_id)  # Body = lambda instance id (connection.go:332)

    def _get(self, cmd, w):
        # get key chunkId reqId dataChunks parityChunks
        key, chunk, req, d, p = (x.decode() for x in cmd[1:6])
        d, p = int(d), int(p)
        with self.lock:
            self.gets += 1
            body = self.store.get((key, chunk))
            if req not in self.late:
                self.late[req] = (set(self.force_late) if self.force_late is not None
                                  else set(self.rng.sample(range(d + p), p)))
            late = int(chunk) in self.late[req]
        if body is None:
            w.write_error("KEY %s@%s not found in lambda store, please set first." % (chunk, key))
            return
        if int(chunk) in self.fail_chunks:
            w.write_error("ERR injected failure for chunk %s" % chunk)
            return
        w.write_bulk_string(req)
        if late:
            w.write_bulk_string("-1")  # abandoned: no body follows
            return
        w.write_bulk_string(chunk)
        w.write_bulk(body)
