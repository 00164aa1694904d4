"""ORACLE — TEST INFRASTRUCTURE ONLY.

Independent numpy restatement of klauspost/reedsolomon v1.9.3 (the codec the
InfiniCache client binds at /root/reference/client/ec.go:19; pinned at
/root/reference/go.mod:16).  It shares no code with oracle/rs_oracle.c: the
field tables are rebuilt here from the polynomial, and coding uses a full
256x256 multiplication table with numpy fancy indexing.  tests/ use it to
cross-check the C oracle and to generate tests/golden/ fixtures; the product
(infinicache_amd/) never imports it.

Pinning: upstream known-answer vectors in
tests/test_oracle_kat.py; the reference's own tests hold no EC vectors.
"""
from __future__ import annotations

import numpy as np

POLY = 0x11D  # upstream galois.go generating polynomial


def _tables():
    exp = np.zeros(510, dtype=np.uint8)
    log = np.zeros(256, dtype=np.int32)
    x = 1
    for i in range(255):
        exp[i] = x
        log[x] = i
        x <<= 1
        if x & 0x100:
            x ^= POLY
    exp[255:510] = exp[0:255]
    a = np.arange(256)
    la = log[a][:, None] + log[a][None, :]
    mul = exp[la % 255].astype(np.uint8)
    mul[0, :] = 0
    mul[:, 0] = 0
    return exp, log, mul


EXP, LOG, MUL = _tables()


def gf_mul(a: int, b: int) -> int:
    return int(MUL[a, b])


def gf_div(a: int, b: int) -> int:
    """upstream galDivide."""
    if a == 0:
        return 0
    if b == 0:
        raise ZeroDivisionError("galDivide by zero")
    l = int(LOG[a]) - int(LOG[b])
    if l < 0:
        l += 255
    return int(EXP[l])


def gf_exp(a: int, n: int) -> int:
    """upstream galExp: a**n with 0**0 == 1."""
    if n == 0:
        return 1
    if a == 0:
        return 0
    return int(EXP[(int(LOG[a]) * n) % 255])


class Singular(Exception):
    pass


def invert(m: np.ndarray) -> np.ndarray:
    """upstream matrix.Invert (Gauss-Jordan on [m | I])."""
    n = m.shape[0]
    w = np.concatenate([m.astype(np.uint8), np.eye(n, dtype=np.uint8)], axis=1)
    for r in range(n):
        if w[r, r] == 0:
            for rb in range(r + 1, n):
                if w[rb, r] != 0:
                    w[[r, rb]] = w[[rb, r]]
                    break
        if w[r, r] == 0:
            raise Singular("matrix is singular")
        if w[r, r] != 1:
            w[r] = MUL[gf_div(1, int(w[r, r]))][w[r]]
        for rb in range(n):
            if rb != r and w[rb, r] != 0:
                w[rb] ^= MUL[int(w[rb, r])][w[r]]
    return w[:, n:].copy()


def matmul(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    out = np.zeros((a.shape[0], b.shape[1]), dtype=np.uint8)
    for i in range(a.shape[1]):
        out ^= MUL[a[:, i][:, None], b[i][None, :]]
    return out


def build_matrix(k: int, p: int, kind: str = "vandermonde") -> np.ndarray:
    """(k+p) x k coding matrix.  vandermonde = upstream buildMatrix,
    cauchy = buildMatrixCauchy, par1 = buildMatrixPAR1."""
    n = k + p
    if kind == "cauchy":
        m = np.zeros((n, k), dtype=np.uint8)
        m[:k] = np.eye(k, dtype=np.uint8)
        for r in range(k, n):
            for c in range(k):
                m[r, c] = gf_div(1, r ^ c)
        return m
    if kind == "par1":
        m = np.zeros((n, k), dtype=np.uint8)
        m[:k] = np.eye(k, dtype=np.uint8)
        for r in range(k, n):
            for c in range(k):
                m[r, c] = gf_exp(c + 1, r - k)
        return m
    vm = np.array([[gf_exp(r, c) for c in range(k)] for r in range(n)], dtype=np.uint8)
    return matmul(vm, invert(vm[:k]))


def apply(coef: np.ndarray, inputs) -> np.ndarray:
    """rows x len output: out[r] = XOR_c coef[r, c] * inputs[c]."""
    inputs = [np.asarray(x, dtype=np.uint8) for x in inputs]
    out = np.zeros((coef.shape[0], inputs[0].shape[0]), dtype=np.uint8)
    for c, x in enumerate(inputs):
        for r in range(coef.shape[0]):
            cf = int(coef[r, c])
            if cf:
                out[r] ^= MUL[cf][x]
    return out


def encode(data_shards, p: int, kind: str = "vandermonde") -> np.ndarray:
    """Parity shards (p x S) for k data shards."""
    k = len(data_shards)
    m = build_matrix(k, p, kind)
    return apply(m[k:], data_shards)


def reconstruct(shards, k: int, p: int, kind: str = "vandermonde", data_only: bool = False):
    """upstream reconstruct(): shards is a list with None for missing ones;
    returns a new list with the missing (data, and parity unless data_only)
    shards filled.  Survivors = first k present shards in index order."""
    n = k + p
    present = [i for i in range(n) if shards[i] is not None and len(shards[i])]
    if len(present) == n:
        return list(shards)
    if len(present) < k:
        raise ValueError("too few shards")
    m = build_matrix(k, p, kind)
    valid = present[:k]
    inv = invert(m[valid])
    out = list(shards)
    subs = [np.asarray(shards[v], dtype=np.uint8) for v in valid]
    miss_data = [i for i in range(k) if i not in present]
    if miss_data:
        rec = apply(inv[miss_data], subs)
        for j, i in enumerate(miss_data):
            out[i] = rec[j]
    if not data_only:
        miss_par = [i for i in range(k, n) if i not in present]
        if miss_par:
            rec = apply(m[miss_par], [out[i] for i in range(k)])
            for j, i in enumerate(miss_par):
                out[i] = rec[j]
    return out


def split(data: bytes, k: int, p: int):
    """upstream Split with cap(data) == len(data): ceil split, zero pad to
    (k+p)*perShard, one backing array."""
    if len(data) == 0:
        raise ValueError("short data")
    per = (len(data) + k - 1) // k
    buf = np.zeros((k + p) * per, dtype=np.uint8)
    buf[: len(data)] = np.frombuffer(bytes(data), dtype=np.uint8)
    return [buf[i * per:(i + 1) * per] for i in range(k + p)]


def splitmix64_bytes(seed: int, obj: int, nbytes: int) -> np.ndarray:
    """Counter-based synthetic object bytes: word w of object o is
    splitmix64(seed ^ (o << 40) ^ w), little-endian."""
    nw = (nbytes + 7) // 8
    with np.errstate(over="ignore"):
        z = (np.uint64(seed) ^ (np.uint64(obj) << np.uint64(40))) ^ np.arange(nw, dtype=np.uint64)
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z.view(np.uint8)[:nbytes].copy()
