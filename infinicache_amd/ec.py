"""Host-side mirror of the InfiniCache client's erasure-coding interface.

Mirrors, name for name:
  * reedsolomon.Encoder (klauspost/reedsolomon v1.9.3, the interface held in
    Client.EC, /root/reference/client/client.go:38): Encode, Verify,
    Reconstruct, ReconstructData, Update, Split, Join;
  * reedsolomon.New(dataShards, parityShards, opts...) -> ``New``;
  * client.NewEncoder (/root/reference/client/ec.go:14-24) -> ``NewEncoder``;
  * client.DummyEncoder (/root/reference/client/ec.go:26-121) -> ``DummyEncoder``.

Encode/Verify/Reconstruct/ReconstructData/Update run on the MI355X through the
C ABI in include/rsgpu.h (librsgpu.so); Split/Join are host slicing, exactly
as in the Go shim design.  Go errors become exceptions of the
same names; Verify returns a bool and raises where Go returns (false, err).
There is no CPU fallback: on a machine without a gfx950 device the compute
methods raise NoDevice.

Batched device-resident entry points (``encode_dev`` & co.) take a device
pointer (int) or any object with ``data_ptr()`` (a torch tensor) laid out
[object][shard][pitch] in HBM.
"""
from __future__ import annotations

import ctypes
import os
from typing import List, Optional, Sequence

import numpy as np

from . import _lib

# ------------------------------------------------------------------ errors


class RSError(Exception):
    """Base of the codec errors; ``code`` is the RSGPU_ERR_* value."""
    code = 0

    def __init__(self, msg: Optional[str] = None):
        super().__init__(msg or self.__class__.__doc__)


class ErrInvShardNum(RSError):
    """cannot create Encoder with zero or less data/parity shards"""
    code = -1


class ErrMaxShardNum(RSError):
    """cannot create Encoder with more than 256 data+parity shards"""
    code = -2


class ErrTooFewShards(RSError):
    """too few shards given"""
    code = -3


class ErrShardNoData(RSError):
    """no shard data"""
    code = -4


class ErrShardSize(RSError):
    """shard sizes do not match"""
    code = -5


class ErrSingular(RSError):
    """matrix is singular"""
    code = -6


class ErrShortData(RSError):
    """not enough data to fill the number of requested shards"""
    code = -7


class ErrReconstructRequired(RSError):
    """reconstruction required as one or more required data shards are nil"""
    code = -8


class ErrInvalidInput(RSError):
    """invalid input"""
    code = -9


class ErrNotImplemented(RSError):
    """Not implemented"""
    code = -10


class InvalidArgument(RSError):
    """rsgpu: invalid argument"""
    code = -20


class NoDevice(RSError):
    """rsgpu: no usable gfx950 device"""
    code = -21


class HipError(RSError):
    """rsgpu: HIP runtime error"""
    code = -22


class OutOfMemory(RSError):
    """rsgpu: out of memory"""
    code = -23


_ERRORS = {c.code: c for c in (ErrInvShardNum, ErrMaxShardNum, ErrTooFewShards, ErrShardNoData,
                               ErrShardSize, ErrSingular, ErrShortData, ErrReconstructRequired,
                               ErrInvalidInput, ErrNotImplemented, InvalidArgument, NoDevice,
                               HipError, OutOfMemory)}


def _check(code: int):
    if code != 0:
        cls = _ERRORS.get(code, RSError)
        raise cls()


MATRIX_KINDS = {"vandermonde": 0, "cauchy": 1, "par1": 2}

# ---------------------------------------------------------------- helpers


def _as_u8(buf, writable: bool) -> Optional[np.ndarray]:
    """View a shard buffer as a 1-D uint8 numpy array (no copy)."""
    if buf is None:
        return None
    if isinstance(buf, np.ndarray):
        a = buf
        if not a.flags.c_contiguous and writable and a.size:
            # reshape would copy: the device would write into a temporary and
            # the caller's buffer would silently keep its old bytes
            raise InvalidArgument("output shard buffer is not contiguous")
        if a.dtype != np.uint8 or a.ndim != 1 or not a.flags.c_contiguous:
            a = a.reshape(-1).view(np.uint8)
    else:
        a = np.frombuffer(buf, dtype=np.uint8)
    if writable and not a.flags.writeable and len(a):
        raise InvalidArgument("output shard buffer is read-only")
    return a


class _ShardTable:
    """Pointer + length arrays for a list of shards (None/empty => len 0).
    Built from raw addresses in one ctypes call each (the per-object host
    path is latency-bound: this table is on it twice per Client.encode)."""

    __slots__ = ("arrs", "ptrs", "lens")

    def __init__(self, shards, writable_idx=()):
        n = len(shards)
        arrs = [_as_u8(s, i in writable_idx) for i, s in enumerate(shards)]
        addrs = [a.__array_interface__["data"][0] if a is not None and len(a) else None for a in arrs]
        self.arrs = arrs  # keeps the buffers alive for the call
        self.ptrs = ctypes.cast((ctypes.c_void_p * n)(*addrs), _lib.u8pp)
        self.lens = (ctypes.c_size_t * n)(*[len(a) if a is not None else 0 for a in arrs])


# The per-object calls marshal their shard table in C when the in-tree
# extension is built (csrc/pyshards.c: buffer protocol + a direct call of the
# rsgpu entry point, GIL released); without it, or for a buffer it cannot
# take as one contiguous byte range, _ShardTable does it through ctypes.
try:
    from . import _pyshards
except ImportError:  # pragma: no cover - the Makefile builds it beside librsgpu.so
    _pyshards = None
if os.environ.get("INFINICACHE_PY_MARSHAL") == "ctypes":  # A/B measurement
    _pyshards = None

_FN_ADDR = {}


def _fn_addr(L, name: str) -> int:
    a = _FN_ADDR.get(name)
    if a is None:
        a = _FN_ADDR[name] = ctypes.cast(getattr(L, name), ctypes.c_void_p).value
    return a


def _fast_call(L, name: str, ctx, shards, wlo: int, whi: int, missing, kind: int, arg: int = 0):
    """_pyshards.call, or None when the ctypes path must take the call."""
    if _pyshards is None or not ctx:
        return None
    return _pyshards.call(_fn_addr(L, name), ctx.value or 0, shards, wlo, whi, missing, kind, arg)


def _dptr(x) -> int:
    if x is None:
        return 0
    if hasattr(x, "data_ptr"):
        return int(x.data_ptr())
    return int(x)


def _stream_handle(stream) -> int:
    if stream is None:
        return 0
    if hasattr(stream, "cuda_stream"):
        return int(stream.cuda_stream)
    return int(stream)


def device_count() -> int:
    return _lib.load().rsgpu_device_count()


def device_ok(device: int = 0) -> bool:
    return bool(_lib.load().rsgpu_device_ok(device))

# ---------------------------------------------------------------- encoder


class RSEncoder:
    """reedsolomon.Encoder backed by the gfx950 kernels (reedsolomon.New)."""

    def __init__(self, data_shards: int, parity_shards: int, *, device: int = 0,
                 matrix: str = "vandermonde", max_goroutines: int = 0, devices=None):
        """device: one GPU, or ALL_DEVICES (-1) for every visible gfx950
        device; devices: an explicit list (one context over several GPUs,
        rsgpu_create_multi: objects never cross GPUs)."""
        L = _lib.load()
        self._L = L
        ctx = ctypes.c_void_p()
        if devices is not None:
            devs = (ctypes.c_int * len(devices))(*devices)
            _check(L.rsgpu_create_multi(data_shards, parity_shards, devs, len(devices),
                                        MATRIX_KINDS[matrix], ctypes.byref(ctx)))
        else:
            _check(L.rsgpu_create(data_shards, parity_shards, device, MATRIX_KINDS[matrix],
                                  ctypes.byref(ctx)))
        self._ctx = ctx
        self.DataShards = data_shards
        self.ParityShards = parity_shards
        self.Shards = data_shards + parity_shards
        self.device = device
        # upstream WithMaxGoroutines has no GPU meaning; kept for API parity
        self.max_goroutines = max_goroutines

    def __del__(self):
        ctx = getattr(self, "_ctx", None)
        if ctx:
            self._L.rsgpu_destroy(ctx)
            self._ctx = None

    def devices(self) -> List[int]:
        """The GPUs this encoder codes on."""
        n = self._L.rsgpu_devices(self._ctx, None, 0)
        out = (ctypes.c_int * max(n, 1))()
        self._L.rsgpu_devices(self._ctx, out, n)
        return list(out[:n])

    def worker_start(self, nslots: int = 0, idle_us: int = 0, max_shard: int = 0) -> None:
        """Per-object calls through the resident worker (rsgpu_worker_start):
        no kernel launch or stream synchronisation per call."""
        _check(self._L.rsgpu_worker_start(self._ctx, nslots, idle_us, max_shard))

    def worker_stop(self) -> None:
        _check(self._L.rsgpu_worker_stop(self._ctx))

    def worker_stats(self) -> dict:
        """{'served', 'declined', 'launches'} of the resident worker."""
        v = [ctypes.c_uint64() for _ in range(3)]
        _check(self._L.rsgpu_worker_stats(self._ctx, *[ctypes.byref(x) for x in v]))
        return dict(zip(("served", "declined", "launches"), (x.value for x in v)))

    def device_calls(self) -> List[int]:
        """Compute calls each entry of devices() has run (how work spread)."""
        n = self._L.rsgpu_device_calls(self._ctx, None, 0)
        out = (ctypes.c_uint64 * max(n, 1))()
        self._L.rsgpu_device_calls(self._ctx, out, n)
        return list(out[:n])

    def matrix(self) -> np.ndarray:
        out = np.zeros((self.Shards, self.DataShards), dtype=np.uint8)
        _check(self._L.rsgpu_matrix(self._ctx, out.ctypes.data_as(_lib.u8p)))
        return out

    # -- the 7 reedsolomon.Encoder methods -------------------------------
    def Encode(self, shards: Sequence) -> None:
        r = _fast_call(self._L, "rsgpu_encode", self._ctx, shards, self.DataShards, len(shards), None, 2)
        if r is not None:
            _check(r)
            return
        t = _ShardTable(shards, writable_idx=range(self.DataShards, len(shards)))
        _check(self._L.rsgpu_encode(self._ctx, t.ptrs, t.lens, len(shards)))

    def Verify(self, shards: Sequence) -> bool:
        r = _fast_call(self._L, "rsgpu_verify", self._ctx, shards, 0, 0, None, 1)
        if r is not None:
            _check(r[0])
            return bool(r[1])
        t = _ShardTable(shards)
        ok = ctypes.c_int(0)
        _check(self._L.rsgpu_verify(self._ctx, t.ptrs, t.lens, len(shards), ctypes.byref(ok)))
        return bool(ok.value)

    def EncodeVerify(self, shards: Sequence) -> bool:
        """Client.encode's Encode then Verify (ecRedis.go:390-395) in one
        device round trip: parity written into shards[k:], then every parity
        shard re-checked on the device image; returns Verify's boolean."""
        r = _fast_call(self._L, "rsgpu_encode_verify", self._ctx, shards, self.DataShards, len(shards), None, 1)
        if r is not None:
            _check(r[0])
            return bool(r[1])
        t = _ShardTable(shards, writable_idx=range(self.DataShards, len(shards)))
        ok = ctypes.c_int(0)
        _check(self._L.rsgpu_encode_verify(self._ctx, t.ptrs, t.lens, len(shards), ctypes.byref(ok)))
        return bool(ok.value)

    def _prepare_missing(self, shards: list, data_only: bool):
        """upstream reconstruct(): missing shards get a buffer of the shard
        size (re-using capacity is a Go notion; Python allocates)."""
        size = next((len(s) for s in shards if s is not None and len(s)), 0)
        bufs = list(shards)
        missing = []
        if size:
            for i, s in enumerate(shards):
                if s is None or len(s) == 0:
                    if data_only and i >= self.DataShards:
                        continue
                    bufs[i] = np.empty(size, dtype=np.uint8)  # every byte is written
                    missing.append(i)
        return bufs, missing

    def _reconstruct(self, shards: list, data_only: bool, fused_verify: bool):
        if not isinstance(shards, list):
            raise InvalidArgument("shards must be a list (filled in place)")
        bufs, missing = self._prepare_missing(shards, data_only)
        n = len(shards)
        # "missing": passed with length 0, the buffer is the output
        if fused_verify:
            r = _fast_call(self._L, "rsgpu_decode", self._ctx, bufs, 0, 0, missing, 1)
        else:
            r = _fast_call(self._L, "rsgpu_reconstruct", self._ctx, bufs, 0, 0, missing, 0, int(data_only))
        if r is not None:
            ok_v = 1
            if fused_verify:
                r, ok_v = r
            _check(r)
        else:
            t = _ShardTable(bufs, writable_idx=missing)
            for i in missing:
                t.lens[i] = 0
            ok = ctypes.c_int(1)
            if fused_verify:
                _check(self._L.rsgpu_decode(self._ctx, t.ptrs, t.lens, n, ctypes.byref(ok)))
            else:
                _check(self._L.rsgpu_reconstruct(self._ctx, t.ptrs, t.lens, n, int(data_only)))
            ok_v = ok.value
        for i in missing:
            shards[i] = bufs[i]
        return bool(ok_v)

    def Reconstruct(self, shards: list) -> None:
        self._reconstruct(shards, data_only=False, fused_verify=False)

    def ReconstructData(self, shards: list) -> None:
        self._reconstruct(shards, data_only=True, fused_verify=False)

    def DecodeVerify(self, shards: list) -> bool:
        """Client.decode's Reconstruct + Verify (ecRedis.go:415-420) fused in
        one device pass; returns what the Verify after Reconstruct returns."""
        return self._reconstruct(shards, data_only=False, fused_verify=True)

    def Update(self, shards: Sequence, newDatashards: Sequence) -> None:
        t = _ShardTable(shards, writable_idx=range(len(shards)))
        nt = _ShardTable(newDatashards)
        _check(self._L.rsgpu_update(self._ctx, t.ptrs, t.lens, len(shards), nt.ptrs, nt.lens,
                                    len(newDatashards)))

    def Split(self, data) -> List[np.ndarray]:
        """upstream Split: perShard = ceil(len/k); zero-pad to (k+p)*perShard;
        k+p consecutive views of ONE backing array.  (Go's cap(data) > len
        quirk does not arise: Python buffers have no spare capacity.)"""
        d = _as_u8(data, False)
        if d is None or len(d) == 0:
            raise ErrShortData()
        per = (len(d) + self.DataShards - 1) // self.DataShards
        buf = np.zeros(self.Shards * per, dtype=np.uint8)
        buf[:len(d)] = d
        return [buf[i * per:(i + 1) * per] for i in range(self.Shards)]

    def Join(self, dst, shards: Sequence, outSize: int) -> None:
        _join(self.DataShards, dst, shards, outSize)

    # -- batched device-resident API (HBM in, HBM out) --------------------
    def encode_dev(self, base, shard_len, pitch, obj_stride, nobj, stream=None):
        _check(self._L.rsgpu_encode_dev(self._ctx, _dptr(base), shard_len, pitch, obj_stride, nobj,
                                        _stream_handle(stream)))

    def verify_dev(self, base, shard_len, pitch, obj_stride, nobj, bad, stream=None):
        _check(self._L.rsgpu_verify_dev(self._ctx, _dptr(base), shard_len, pitch, obj_stride, nobj,
                                        _dptr(bad), _stream_handle(stream)))

    def reconstruct_dev(self, base, present, shard_len, pitch, obj_stride, nobj, data_only=False,
                        stream=None):
        pr = (ctypes.c_uint8 * self.Shards)(*[1 if x else 0 for x in present])
        _check(self._L.rsgpu_reconstruct_dev(self._ctx, _dptr(base), pr, shard_len, pitch,
                                             obj_stride, nobj, int(data_only),
                                             _stream_handle(stream)))

    def decode_dev(self, base, present, shard_len, pitch, obj_stride, nobj, bad, stream=None):
        pr = (ctypes.c_uint8 * self.Shards)(*[1 if x else 0 for x in present])
        _check(self._L.rsgpu_decode_dev(self._ctx, _dptr(base), pr, shard_len, pitch, obj_stride,
                                        nobj, _dptr(bad), _stream_handle(stream)))


    # -- variable-size device batches: objs = [(base, shard_len, pitch), ...]
    @staticmethod
    def _obj_table(objs):
        t = (_lib.DevObj * max(1, len(objs)))()
        for i, (b, s, p) in enumerate(objs):
            t[i].base = _dptr(b)
            t[i].shard_len = s
            t[i].pitch = p
        return t

    def encode_dev_objs(self, objs, stream=None):
        t = self._obj_table(objs)
        _check(self._L.rsgpu_encode_dev_objs(self._ctx, ctypes.addressof(t), len(objs), _stream_handle(stream)))

    def verify_dev_objs(self, objs, bad, stream=None):
        t = self._obj_table(objs)
        _check(self._L.rsgpu_verify_dev_objs(self._ctx, ctypes.addressof(t), len(objs), _dptr(bad),
                                             _stream_handle(stream)))

    def reconstruct_dev_objs(self, objs, present, data_only=False, stream=None):
        t = self._obj_table(objs)
        pr = (ctypes.c_uint8 * self.Shards)(*[1 if x else 0 for x in present])
        _check(self._L.rsgpu_reconstruct_dev_objs(self._ctx, ctypes.addressof(t), len(objs), pr, int(data_only),
                                                  _stream_handle(stream)))

    def decode_dev_objs(self, objs, present, bad, stream=None):
        t = self._obj_table(objs)
        pr = (ctypes.c_uint8 * self.Shards)(*[1 if x else 0 for x in present])
        _check(self._L.rsgpu_decode_dev_objs(self._ctx, ctypes.addressof(t), len(objs), pr, _dptr(bad),
                                             _stream_handle(stream)))

    def _present_matrix(self, present, nobj):
        pm = np.ascontiguousarray(np.asarray(present, dtype=np.uint8).reshape(nobj, self.Shards))
        return pm, pm.ctypes.data_as(_lib.u8p)

    def reconstruct_dev_multi(self, base, present, shard_len, pitch, obj_stride, nobj,
                              data_only=False, stream=None):
        """Per-object erasure patterns: present is (nobj, k+p) flags."""
        pm, pp = self._present_matrix(present, nobj)
        _check(self._L.rsgpu_reconstruct_dev_multi(self._ctx, _dptr(base), pp, shard_len, pitch,
                                                   obj_stride, nobj, int(data_only),
                                                   _stream_handle(stream)))

    def decode_dev_multi(self, base, present, shard_len, pitch, obj_stride, nobj, bad, stream=None):
        pm, pp = self._present_matrix(present, nobj)
        _check(self._L.rsgpu_decode_dev_multi(self._ctx, _dptr(base), pp, shard_len, pitch,
                                              obj_stride, nobj, _dptr(bad), _stream_handle(stream)))

    def decode_dev_masks(self, base, masks, shard_len, pitch, obj_stride, nobj, status, stream=None):
        """Per-object erasure patterns as device-resident present bitmasks
        (masks: nobj uint32 in HBM, bit i = shard i arrived); the pattern ->
        pass resolution runs on the device.  status (nobj uint32 in HBM):
        0 ok, 1 Verify-after-Reconstruct mismatch, 2 too few shards, 3 singular."""
        _check(self._L.rsgpu_decode_dev_masks(self._ctx, _dptr(base), _dptr(masks), shard_len, pitch,
                                              obj_stride, nobj, _dptr(status), _stream_handle(stream)))

    def reconstruct_dev_masks(self, base, masks, shard_len, pitch, obj_stride, nobj, data_only=False,
                              status=None, stream=None):
        _check(self._L.rsgpu_reconstruct_dev_masks(self._ctx, _dptr(base), _dptr(masks), shard_len, pitch,
                                                   obj_stride, nobj, int(data_only), _dptr(status),
                                                   _stream_handle(stream)))

    # -- batched host-memory API (pipelined H2D -> kernel -> D2H) ----------
    def copy_pieces(self, src, src_pitch, src_obj_stride, dst, dst_pitch, dst_obj_stride, shard_len, nobj,
                    rows=None, stream=None):
        """rsgpu_copy_pieces: move rows `rows` (row indices; default every
        row) of nobj objects between two device layouts (object-major or
        shard-major), exactly shard_len bytes per piece."""
        mask = (1 << self.Shards) - 1 if rows is None else sum(1 << int(i) for i in rows)
        _check(self._L.rsgpu_copy_pieces(self._ctx, _dptr(src), src_pitch, src_obj_stride, _dptr(dst), dst_pitch,
                                         dst_obj_stride, shard_len, nobj, mask, _stream_handle(stream)))

    def encode_batch(self, objs: Sequence) -> None:
        """Encode many objects, each given as its Split() result (or the
        backing array of one): parity rows are written in place.  Host
        buffers from host_alloc()/host_register() make the copies async."""
        if _pyshards is not None and self._ctx:
            r = _pyshards.encode_batch(_fn_addr(self._L, "rsgpu_encode_batch"), self._ctx.value or 0, objs,
                                       self.Shards)
            if r is not None:
                _check(r)
                return
        bases, lens, keep = [], [], []
        for o in objs:
            if isinstance(o, (list, tuple)):
                if len(o) != self.Shards:
                    raise ErrTooFewShards()
                rows = [_as_u8(s, True) for s in o]
                S = len(rows[0])
                if not all(len(r) == S and r.ctypes.data == rows[0].ctypes.data + i * S
                           for i, r in enumerate(rows)):
                    raise InvalidArgument("shards are not one contiguous Split() array")
                ptr = rows[0].ctypes.data
                keep.append(rows)
            else:
                arr = _as_u8(o, True)
                if len(arr) % self.Shards:
                    raise InvalidArgument("backing array length is not a multiple of the shard count")
                S = len(arr) // self.Shards
                ptr = arr.ctypes.data
                keep.append(arr)
            bases.append(ptr)
            lens.append(S)
        n = len(bases)
        ptrs = (_lib.u8p * n)(*[ctypes.cast(ctypes.c_void_p(b), _lib.u8p) for b in bases])
        ln = (ctypes.c_size_t * n)(*lens)
        _check(self._L.rsgpu_encode_batch(self._ctx, ptrs, ln, n))

    def decode_batch(self, objs: Sequence[list], present=None) -> List[bool]:
        """Fused Client.decode over many Gets: objs[o] is the list of k+p
        shards of object o (None/empty = did not arrive); missing shards are
        filled in place.  With ``present`` (nobj x (k+p) flags) every entry is
        a buffer and the flags say which ones arrived (no allocation).
        Returns the per-object Verify-after-Reconstruct."""
        if present is not None and _pyshards is not None and self._ctx:
            r = _pyshards.decode_batch(_fn_addr(self._L, "rsgpu_decode_batch"), self._ctx.value or 0, objs,
                                       present, self.Shards)
            if r is not None:
                _check(r[0])
                return r[1]
        nobj = len(objs)
        n = self.Shards
        ptrs = (_lib.u8p * (nobj * n))()
        pres = (ctypes.c_uint8 * (nobj * n))()
        lens = (ctypes.c_size_t * nobj)()
        keep = []
        for o, shards in enumerate(objs):
            if len(shards) != n:
                raise ErrTooFewShards()
            S = next((len(s) for s in shards if s is not None and len(s)), 0)
            if S == 0:
                raise ErrShardNoData()
            lens[o] = S
            for i, s in enumerate(shards):
                if present is not None:
                    pres[o * n + i] = 1 if present[o][i] else 0
                    if len(s) != S:
                        raise ErrShardSize()
                elif s is None or len(s) == 0:
                    s = np.zeros(S, dtype=np.uint8)
                    shards[i] = s
                else:
                    pres[o * n + i] = 1
                    if len(s) != S:
                        raise ErrShardSize()
                a = _as_u8(s, not pres[o * n + i])
                keep.append(a)
                ptrs[o * n + i] = a.ctypes.data_as(_lib.u8p)
        ok = (ctypes.c_int * max(nobj, 1))()
        _check(self._L.rsgpu_decode_batch(self._ctx, ptrs, pres, lens, nobj, ok))
        return [bool(ok[o]) for o in range(nobj)]


def shardmajor_layout(shard_len: int, nobj: int):
    """rsgpu_shardmajor_layout: (obj_stride, pitch) of a shard-major batch of
    nobj pieces of shard_len bytes on whole 128-B lines (when the gap stays
    at most shard_len / 4; else 16-B aligned pieces)."""
    L = _lib.load()
    st, pi = ctypes.c_size_t(), ctypes.c_size_t()
    _check(L.rsgpu_shardmajor_layout(shard_len, nobj, ctypes.byref(st), ctypes.byref(pi)))
    return st.value, pi.value


def host_alloc(nbytes: int) -> np.ndarray:
    """Pinned (page-locked) host buffer as a uint8 numpy array; freed with the
    array.  Use it for objects streamed through encode_batch/decode_batch."""
    L = _lib.load()
    p = ctypes.c_void_p()
    _check(L.rsgpu_host_alloc(nbytes, ctypes.byref(p)))
    buf = (ctypes.c_uint8 * nbytes).from_address(p.value)
    arr = np.frombuffer(buf, dtype=np.uint8)
    import weakref
    weakref.finalize(buf, L.rsgpu_host_free, ctypes.c_void_p(p.value))
    return arr


def host_register(arr: np.ndarray) -> None:
    """Pin an existing host buffer for async DMA (hipHostRegister)."""
    _check(_lib.load().rsgpu_host_register(arr.ctypes.data, arr.nbytes))


def host_unregister(arr: np.ndarray) -> None:
    _check(_lib.load().rsgpu_host_unregister(arr.ctypes.data))


def retired_stats() -> dict:
    """rsgpu_retired_stats: library buffers whose free is held back because a
    worker kernel is resident (count, bytes) and frees ever held back."""
    L = _lib.load()
    c, b, d = ctypes.c_size_t(), ctypes.c_size_t(), ctypes.c_uint64()
    _check(L.rsgpu_retired_stats(ctypes.byref(c), ctypes.byref(b), ctypes.byref(d)))
    return {"count": c.value, "bytes": b.value, "deferred": d.value}


def set_slab_bytes(nbytes: int) -> None:
    """rsgpu_set_slab_bytes: staged bytes per object above which host calls
    code in column slabs (< 4096: the 1 GiB default).  A test knob."""
    _check(_lib.load().rsgpu_set_slab_bytes(int(nbytes)))


def _join(k: int, dst, shards: Sequence, outSize: int) -> None:
    """upstream Join (identical logic in /root/reference/client/ec.go:83-121)."""
    if len(shards) < k:
        raise ErrTooFewShards()
    shards = shards[:k]
    size = 0
    for s in shards:
        if s is None:
            raise ErrReconstructRequired()
        size += len(s)
        if size >= outSize:
            break
    if size < outSize:
        raise ErrShortData()
    write = outSize
    for s in shards:
        if write < len(s):
            dst.write(bytes(memoryview(_as_u8(s, False))[:write]))
            return
        dst.write(bytes(_as_u8(s, False)))
        write -= len(s)


ALL_DEVICES = -1  # rsgpu.h RSGPU_ALL_DEVICES


def New(dataShards: int, parityShards: int, *, device: int = 0, matrix: str = "vandermonde",
        max_goroutines: int = 0, devices=None) -> RSEncoder:
    """reedsolomon.New: raises ErrInvShardNum / ErrMaxShardNum.  device =
    ALL_DEVICES or devices=[...] spans several GPUs (RSEncoder)."""
    return RSEncoder(dataShards, parityShards, device=device, matrix=matrix,
                     max_goroutines=max_goroutines, devices=devices)


class DummyEncoder:
    """client.DummyEncoder (/root/reference/client/ec.go:26-121): the p == 0
    codec — no parity, Verify only checks shard presence."""

    def __init__(self, DataShards: int):
        self.DataShards = DataShards

    def Encode(self, shards):
        return None

    def Verify(self, shards) -> bool:
        if len(shards) != self.DataShards:
            raise ErrTooFewShards()
        for s in shards:
            if s is None or len(s) == 0:
                raise ErrTooFewShards()
        return True

    def Reconstruct(self, shards):
        self.Verify(shards)

    def ReconstructData(self, shards):
        self.Verify(shards)

    def Update(self, shards, newDatashards):
        raise ErrNotImplemented()

    def Split(self, data):
        d = _as_u8(data, False)
        if d is None or len(d) == 0:
            raise ErrShortData()
        per = (len(d) + self.DataShards - 1) // self.DataShards
        dst: List[Optional[np.ndarray]] = [None] * self.DataShards
        i = 0
        while i < len(dst) and len(d) >= per:
            dst[i] = d[:per]
            d = d[per:]
            i += 1
        if i < len(dst):
            dst[i] = d
        return dst

    def Join(self, dst, shards, outSize):
        _join(self.DataShards, dst, shards, outSize)


def NewEncoder(dataShards: int, parityShards: int, ecMaxGoroutine: int, *, device: int = ALL_DEVICES):
    """client.NewEncoder (/root/reference/client/ec.go:14-24): p == 0 ->
    DummyEncoder; otherwise New(...), printing and swallowing the error (the
    Go factory then returns a nil Encoder, here None).  By default the
    encoder spans every visible GPU (concurrent EcSet/EcGet calls go to them
    round-robin), as the Go shim's NewEncoder does."""
    if parityShards == 0:
        return DummyEncoder(dataShards)
    try:
        return New(dataShards, parityShards, device=device, max_goroutines=ecMaxGoroutine)
    except RSError as err:
        print("newEncoder err", err)
        return None
