"""Host-side mirror of the InfiniCache client object API with the codec
underneath running on the MI355X.

Mirrors /root/reference/client/client.go and client/ecRedis.go:
  * NewClient(d, p, g)                    client.go:47-59
  * Client.Dial(addrs)                    client.go:61-128 (d+p TCP conns per proxy)
  * Client.EcSet(key, val)                ecRedis.go:58-129
  * Client.EcGet(key, size)               ecRedis.go:131-191
  * Client.encode / decode / recover      ecRedis.go:365-432
  * the per-shard RESP wire format        ecRedis.go:220-363 (infinicache_amd/resp.py)

Only the codec changes: ``EC`` is infinicache_amd.ec.NewEncoder (the gfx950
path for p > 0, DummyEncoder for p == 0).  ``decode`` keeps the reference's
Verify -> Reconstruct -> Verify flow; with ``fused_decode`` (default) the
Reconstruct+Verify pair runs as ONE device pass (RSEncoder.DecodeVerify),
returning exactly what the second Verify would.

Out of scope: the proxy, Lambda runtime, nanolog metrics and the
buraksezer/consistent ring; with several proxies ``Dial`` places keys with a
plain xxhash64 modulo (not the reference's bounded-load ring).
"""
from __future__ import annotations

import io
import random
import socket
import threading
import time
import uuid
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass, field
from typing import Dict, List, Optional

from . import resp
from .ec import DummyEncoder, NewEncoder, RSError

MaxLambdaStores = 400  # server.NumLambdaClusters (proxy/server/config.go:11)
Timeout = 120.0        # ecRedis.go:23


class ErrUnexpectedResponse(Exception):
    """Unexpected response"""


@dataclass
class DataEntry:  # client.go:23-32
    Cmd: str = ""
    ReqId: str = ""
    Begin: float = 0.0
    ReqLatency: float = 0.0
    RecLatency: float = 0.0
    Duration: float = 0.0
    AllGood: bool = False
    Corrupted: bool = False


class ecRet:  # client.go:155-189
    def __init__(self, n: int):
        self.Rets: List[object] = [None] * n
        self.Err: Optional[Exception] = None
        self._lock = threading.Lock()

    def Len(self):
        return len(self.Rets)

    def Set(self, i, v):
        self.Rets[i] = v

    def SetError(self, i, err):
        with self._lock:
            self.Rets[i] = err
            self.Err = err

    def Ret(self, i):
        r = self.Rets[i]
        return None if isinstance(r, Exception) else r

    def Error(self, i):
        r = self.Rets[i]
        return r if isinstance(r, Exception) else None


class Conn:
    def __init__(self, sock: socket.socket):
        self.conn = sock
        self.W = resp.Writer(sock)
        self.R = resp.Reader(sock)

    def Close(self):
        try:
            self.conn.close()
        except OSError:
            pass


class Client:
    def __init__(self, dataShards: int, parityShards: int, ecMaxGoroutine: int, *, device: int = -1,
                 fused_decode: bool = True):
        self.Conns: Dict[str, List[Optional[Conn]]] = {}
        self.EC = NewEncoder(dataShards, parityShards, ecMaxGoroutine, device=device)
        self.DataShards = dataShards
        self.ParityShards = parityShards
        self.Shards = dataShards + parityShards
        self.Data = DataEntry()
        self.members: List[str] = []
        self.fused_decode = fused_decode
        self._pool = ThreadPoolExecutor(max_workers=max(self.Shards, 1))

    # ------------------------------------------------------------ dialing
    def Dial(self, addrArr: List[str]) -> bool:
        self.members = list(addrArr)
        for addr in addrArr:
            try:
                self.initDial(addr)
            except OSError as err:
                print("Fail to dial %s: %s" % (addr, err))
                self.Close()
                return False
        return True

    def initDial(self, address: str):
        self.Conns[address] = [None] * self.Shards
        for i in range(self.Shards):
            self.connect(address, i)

    def connect(self, address: str, i: int):
        host, port = address.rsplit(":", 1)
        s = socket.create_connection((host, int(port)), timeout=Timeout)
        s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        self.Conns[address][i] = Conn(s)

    def disconnect(self, address: str, i: int):
        cn = self.Conns.get(address, [None] * self.Shards)[i]
        if cn is not None:
            cn.Close()
            self.Conns[address][i] = None

    def validate(self, address: str, i: int):
        if self.Conns[address][i] is None:
            self.connect(address, i)

    def Close(self):
        for addr, conns in self.Conns.items():
            for i in range(len(conns)):
                self.disconnect(addr, i)
        self._pool.shutdown(wait=False)

    def locate(self, key: str) -> str:
        if len(self.members) == 1:
            return self.members[0]
        import xxhash
        return self.members[xxhash.xxh64(key.encode()).intdigest() % len(self.members)]

    # -------------------------------------------------------------- codec
    def encode(self, obj) -> List:
        """ecRedis.go:382-402: Split -> Encode -> Verify (with ``fused_decode``
        and a GPU codec, the Encode+Verify pair is one device round trip,
        RSEncoder.EncodeVerify)."""
        shards = self.EC.Split(obj)
        if self.fused_decode and hasattr(self.EC, "EncodeVerify"):
            ok = self.EC.EncodeVerify(shards)
        else:
            self.EC.Encode(shards)
            ok = self.EC.Verify(shards)
        if not ok:
            raise RSError("Failed to verify encoding")
        return shards

    def decode(self, stats: DataEntry, data: List, size: int):
        """ecRedis.go:404-432: Verify; on failure Reconstruct then Verify
        (note the reference's inverted flag: stats.Corrupted is True on
        success, :420-426); Join into a reader."""
        try:
            stats.AllGood = self.EC.Verify(data)
        except RSError:
            stats.AllGood = False  # nil shards: (false, ErrShardSize), no math
        if not stats.AllGood:
            if self.fused_decode and hasattr(self.EC, "DecodeVerify"):
                stats.Corrupted = self.EC.DecodeVerify(data)
            else:
                self.EC.Reconstruct(data)
                try:
                    stats.Corrupted = self.EC.Verify(data)
                except RSError:
                    stats.Corrupted = False
            if not stats.Corrupted:
                raise RSError("Verification failed after reconstruction, data could be corrupted")
        out = io.BytesIO()
        self.EC.Join(out, data, size)
        out.seek(0)
        return out

    # --------------------------------------------------------- object API
    def EcSet(self, key: str, val, *args):
        dryrun = args[0] if len(args) > 0 else 0
        placements = args[1] if len(args) > 1 and len(args[1]) >= self.Shards else None
        stats = self.Data
        stats.Begin = time.time()
        stats.ReqId = str(uuid.uuid4())
        numClusters = dryrun if dryrun > 0 else MaxLambdaStores
        index = random.sample(range(numClusters), self.Shards)  # rand.Perm(n)[:Shards]
        if dryrun > 0 and placements is not None:
            placements[:self.Shards] = index
            return stats.ReqId, True
        host = self.locate(key)
        try:
            shards = self.encode(val)
        except RSError as err:
            print("EcSet failed to encode: %s" % err)
            return stats.ReqId, False
        ret = ecRet(self.Shards)
        futs = [self._pool.submit(self.set, host, key, shards[i], i, index[i], stats.ReqId, ret)
                for i in range(ret.Len())]
        for f in futs:
            f.result()
        stats.ReqLatency = time.time() - stats.Begin
        stats.Duration = stats.ReqLatency
        if ret.Err is not None:
            return stats.ReqId, False
        if placements is not None:
            for i in range(ret.Len()):
                placements[i] = int(ret.Ret(i))
        return stats.ReqId, True

    def EcGet(self, key: str, size: int, *args):
        dryrun = args[0] if len(args) > 0 else 0
        stats = self.Data
        stats.Begin = time.time()
        stats.ReqId = str(uuid.uuid4())
        if dryrun > 0:
            return stats.ReqId, None, True
        host = self.locate(key)
        ret = ecRet(self.Shards)
        futs = [self._pool.submit(self.get, host, key, i, stats.ReqId, ret) for i in range(ret.Len())]
        for f in futs:
            f.result()
        stats.RecLatency = time.time() - stats.Begin
        chunks: List[Optional[bytes]] = [None] * ret.Len()
        failed = []
        for i in range(ret.Len()):
            if ret.Error(i) is not None:
                failed.append(i)
            else:
                r = ret.Ret(i)
                chunks[i] = bytearray(r) if r is not None else None
        try:
            reader = self.decode(stats, chunks, size)
        except RSError:
            return stats.ReqId, None, False
        stats.Duration = time.time() - stats.Begin
        if failed:
            self.recover(host, key, str(uuid.uuid4()), chunks, failed)
        return stats.ReqId, reader, True

    def recover(self, addr: str, key: str, reqId: str, shards: List, failed: List[int]):
        """ecRedis.go:365-380: re-set only the errored shards."""
        ret = ecRet(self.Shards)
        futs = [self._pool.submit(self.set, addr, key, shards[i], i, 0, reqId, ret) for i in failed]
        for f in futs:
            f.result()

    # ----------------------------------------------------------- wire
    def setError(self, ret: ecRet, addr: str, i: int, err: Exception):
        if isinstance(err, (EOFError, OSError)):
            self.disconnect(addr, i)
        ret.SetError(i, err)

    def set(self, addr, key, val, i, lambdaId, reqId, ret):
        """ecRedis.go:220-259: *9 set key chunkId lambdaId MaxLambdaStores reqId d p <val>."""
        try:
            self.validate(addr, i)
            cn = self.Conns[addr][i]
            w = cn.W
            w.write_multi_bulk_size(9)
            for a in ("set", key, str(i), str(lambdaId), str(MaxLambdaStores), reqId,
                      str(self.DataShards), str(self.ParityShards)):
                w.write_bulk_string(a)
            w.write_bulk(val)
            w.flush()
        except (OSError, EOFError) as err:
            self.setError(ret, addr, i, err)
            return
        self.rec("Set", addr, i, reqId, ret)

    def get(self, addr, key, i, reqId, ret):
        """ecRedis.go:261-290: get key chunkId reqId d p."""
        try:
            self.validate(addr, i)
            cn = self.Conns[addr][i]
            cn.W.write_cmd_string("get", key, str(i), reqId, str(self.DataShards),
                                  str(self.ParityShards))
            cn.W.flush()
        except (OSError, EOFError) as err:
            self.setError(ret, addr, i, err)
            return
        self.rec("Got", addr, i, reqId, ret)

    def rec(self, prompt, addr, i, reqId, ret):
        """ecRedis.go:292-363: reqId, chunkId ("-1" = late, no body), body."""
        cn = self.Conns[addr][i]
        try:
            if cn.R.peek_type() == resp.TypeError_:
                ret.SetError(i, Exception(cn.R.read_error()))
                return
            respId = cn.R.read_bulk_string()
            if respId != reqId:
                cn.R.read_bulk_string()
                cn.R.read_bulk()
                ret.SetError(i, ErrUnexpectedResponse())
                return
            chunkId = cn.R.read_bulk_string()
            if chunkId == "-1":
                return  # abandoned late chunk: Rets[i] stays nil
            ret.Set(i, cn.R.read_bulk())
        except (OSError, EOFError, resp.ProtocolError) as err:
            self.setError(ret, addr, i, err)


def NewClient(dataShards: int, parityShards: int, ecMaxGoroutine: int, **kw) -> Client:
    return Client(dataShards, parityShards, ecMaxGoroutine, **kw)
