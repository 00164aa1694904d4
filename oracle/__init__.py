"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes loader for oracle/liboracle.so (the C restatement in rs_oracle.c) plus
the numpy restatement (rs_numpy.py).  Importable only from tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg; the product package
infinicache_amd/ never imports this module.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

# numeric error codes (same values as include/rsgpu.h)
OK = 0
ERR_INV_SHARD_NUM = -1
ERR_MAX_SHARD_NUM = -2
ERR_TOO_FEW_SHARDS = -3
ERR_SHARD_NO_DATA = -4
ERR_SHARD_SIZE = -5
ERR_SINGULAR = -6
ERR_SHORT_DATA = -7
ERR_RECONSTRUCT_REQUIRED = -8
ERR_INVALID_INPUT = -9

KINDS = {"vandermonde": 0, "cauchy": 1, "par1": 2}

_lib = None


def build() -> str:
    """Compile liboracle.so (gcc) if missing or stale."""
    src = os.path.join(HERE, "rs_oracle.c")
    if not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", HERE])
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(LIB_PATH)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        L.orc_gf_mul.restype = ctypes.c_uint8
        L.orc_gf_mul.argtypes = [ctypes.c_uint8, ctypes.c_uint8]
        L.orc_gf_div.restype = ctypes.c_uint8
        L.orc_gf_div.argtypes = [ctypes.c_uint8, ctypes.c_uint8]
        L.orc_gf_exp.restype = ctypes.c_uint8
        L.orc_gf_exp.argtypes = [ctypes.c_uint8, ctypes.c_int]
        L.orc_invert.argtypes = [ctypes.c_int, u8p, u8p]
        L.orc_build_matrix.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, u8p]
        sp = ctypes.POINTER(u8p)
        szp = ctypes.POINTER(ctypes.c_size_t)
        L.orc_apply.argtypes = [u8p, ctypes.c_int, ctypes.c_int, sp, sp, ctypes.c_size_t]
        L.orc_apply.restype = None
        L.orc_encode.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, sp, szp, ctypes.c_int]
        L.orc_verify.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, sp, szp, ctypes.c_int,
                                 ctypes.POINTER(ctypes.c_int)]
        L.orc_reconstruct.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, sp, szp,
                                      ctypes.c_int, ctypes.c_int]
        L.orc_update.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, sp, szp, ctypes.c_int,
                                 sp, szp, ctypes.c_int]
        L.orc_code_fast.argtypes = [u8p, ctypes.c_int, ctypes.c_int, sp, sp, ctypes.c_size_t,
                                    ctypes.c_int, ctypes.c_int]
        L.orc_code_fast.restype = None
        ip = ctypes.POINTER(ctypes.c_int)
        L.orc_code_batch.argtypes = [u8p, ctypes.c_int, ctypes.c_int, ip, ip, u8p, ctypes.c_size_t,
                                     ctypes.c_size_t, ctypes.c_size_t, ctypes.c_int, ctypes.c_int]
        L.orc_code_batch.restype = None
        L.orc_verify_batch.argtypes = [u8p, ctypes.c_int, ctypes.c_int, ip, ip, u8p, ctypes.c_size_t,
                                       ctypes.c_size_t, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ip]
        L.orc_verify_batch.restype = None
        _lib = L
    return _lib


def _u8p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))


def _ptrs(arrs):
    u8p = ctypes.POINTER(ctypes.c_uint8)
    return (u8p * len(arrs))(*[_u8p(a) for a in arrs])


def build_matrix(k: int, p: int, kind: str = "vandermonde"):
    out = np.zeros((k + p) * max(k, 1), dtype=np.uint8)
    e = lib().orc_build_matrix(k, p, KINDS[kind], _u8p(out))
    if e:
        return e, None
    return 0, out.reshape(k + p, k)


def invert(m: np.ndarray):
    m = np.ascontiguousarray(m, dtype=np.uint8)
    out = np.zeros_like(m)
    e = lib().orc_invert(m.shape[0], _u8p(m), _u8p(out))
    return e, (out if e == 0 else None)


def _norm(shards, size=None):
    """list of (buffer or None) -> (arrays, lens); None -> zero buffer, len 0."""
    if size is None:
        size = max((len(s) for s in shards if s is not None), default=0)
    arrs, lens = [], []
    for s in shards:
        if s is None or len(s) == 0:
            arrs.append(np.zeros(max(size, 1), dtype=np.uint8))
            lens.append(0)
        else:
            a = np.ascontiguousarray(np.frombuffer(bytes(s), dtype=np.uint8)) if not isinstance(s, np.ndarray) else np.ascontiguousarray(s, dtype=np.uint8)
            arrs.append(a.copy())
            lens.append(len(a))
    return arrs, (ctypes.c_size_t * len(lens))(*lens)


def encode(k, p, shards, kind="vandermonde"):
    """Returns (err, shards_out)."""
    arrs, lens = _norm(shards)
    e = lib().orc_encode(k, p, KINDS[kind], _ptrs(arrs), lens, len(arrs))
    return e, arrs


def verify(k, p, shards, kind="vandermonde"):
    arrs, lens = _norm(shards)
    ok = ctypes.c_int(0)
    e = lib().orc_verify(k, p, KINDS[kind], _ptrs(arrs), lens, len(arrs), ctypes.byref(ok))
    return e, bool(ok.value)


def reconstruct(k, p, shards, kind="vandermonde", data_only=False):
    arrs, lens = _norm(shards)
    e = lib().orc_reconstruct(k, p, KINDS[kind], _ptrs(arrs), lens, len(arrs), int(data_only))
    return e, arrs


def update(k, p, shards, newdata, kind="vandermonde"):
    arrs, lens = _norm(shards)
    narrs, nlens = _norm(newdata)
    e = lib().orc_update(k, p, KINDS[kind], _ptrs(arrs), lens, len(arrs), _ptrs(narrs), nlens,
                         len(narrs))
    return e, arrs


def apply(coef: np.ndarray, inputs):
    coef = np.ascontiguousarray(coef, dtype=np.uint8)
    ins = [np.ascontiguousarray(x, dtype=np.uint8) for x in inputs]
    outs = [np.zeros(len(ins[0]), dtype=np.uint8) for _ in range(coef.shape[0])]
    lib().orc_apply(_u8p(coef), coef.shape[0], coef.shape[1], _ptrs(ins), _ptrs(outs), len(ins[0]))
    return outs


def code_fast(coef: np.ndarray, inputs, nthreads=1, max_goroutines=32):
    coef = np.ascontiguousarray(coef, dtype=np.uint8)
    outs = [np.zeros(len(inputs[0]), dtype=np.uint8) for _ in range(coef.shape[0])]
    lib().orc_code_fast(_u8p(coef), coef.shape[0], coef.shape[1], _ptrs(inputs), _ptrs(outs),
                        len(inputs[0]), nthreads, max_goroutines)
    return outs


def code_batch(coef, in_rows, out_rows, base: np.ndarray, obj_stride, pitch, length, nobj,
               nthreads=1):
    """Batch CPU baseline over a [obj][shard][pitch] host buffer (in place)."""
    coef = np.ascontiguousarray(coef, dtype=np.uint8)
    ir = (ctypes.c_int * len(in_rows))(*in_rows)
    orr = (ctypes.c_int * len(out_rows))(*out_rows)
    lib().orc_code_batch(_u8p(coef), coef.shape[0], coef.shape[1], ir, orr, _u8p(base),
                         obj_stride, pitch, length, nobj, nthreads)


def verify_batch(coef, in_rows, chk_rows, base: np.ndarray, obj_stride, pitch, length, nobj,
                 nthreads=1):
    """Batch Verify over a [obj][shard][pitch] host buffer: per object, rows
    coef x in_rows recomputed and compared with the stored rows chk_rows
    (upstream Verify when coef = the parity rows over the data rows).
    Returns the per-object ok flags (uint8 array)."""
    coef = np.ascontiguousarray(coef, dtype=np.uint8)
    ir = (ctypes.c_int * len(in_rows))(*in_rows)
    cr = (ctypes.c_int * len(chk_rows))(*chk_rows)
    ok = (ctypes.c_int * max(1, nobj))()
    lib().orc_verify_batch(_u8p(coef), coef.shape[0], coef.shape[1], ir, cr, _u8p(base),
                           obj_stride, pitch, length, nobj, nthreads, ok)
    return np.array(ok[:nobj], dtype=np.uint8)
