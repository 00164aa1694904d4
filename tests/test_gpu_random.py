"""Seeded randomized differential test: the HIP path against the CPU oracle
(oracle/rs_oracle.c, the restatement of klauspost/reedsolomon v1.9.3) over
random shapes, sizes, operations, erasure patterns and corruptions.  Every
case compares bytes (bit-exact) and booleans/errors with the oracle's
answer on the same input.  Deterministic (fixed seeds), bounded to a few
seconds on the MI355X."""
import numpy as np
import pytest

import infinicache_amd as ia
import oracle

pytestmark = pytest.mark.gpu

ERRS = {oracle.ERR_TOO_FEW_SHARDS: ia.ErrTooFewShards, oracle.ERR_SHARD_SIZE: ia.ErrShardSize,
        oracle.ERR_SHARD_NO_DATA: ia.ErrShardNoData}


def _case(rng):
    k = int(rng.integers(1, 21))
    p = int(rng.integers(1, 9))
    size = int(rng.choice([1, 2, 15, 16, 17, 63, 64, 255, 256, 1023, 4096, 4097, 12345,
                           int(rng.integers(1, 40000))]))
    kind = str(rng.choice(["vandermonde", "vandermonde", "cauchy"]))
    data = [rng.integers(0, 256, size, dtype=np.uint8) for _ in range(k)]
    e, full = oracle.encode(k, p, data + [bytes(size)] * p, kind)
    assert e == 0
    return k, p, size, kind, full


def _lose(rng, n, maxlost):
    m = int(rng.integers(1, maxlost + 1))
    return sorted(rng.choice(n, m, replace=False).tolist())


@pytest.mark.parametrize("seed", range(8))
def test_random_host_ops_vs_oracle(gpu, seed):
    rng = np.random.default_rng(1000 + seed)
    for _ in range(25):
        k, p, size, kind, full = _case(rng)
        n = k + p
        enc = ia.New(k, p, matrix=kind)
        op = str(rng.choice(["encode", "encode_verify", "verify", "reconstruct", "rdata", "decode",
                             "update"]))
        tag = (seed, op, k, p, size, kind)
        if op in ("encode", "encode_verify"):
            sh = [full[i].copy() for i in range(k)] + [np.full(size, 0xA5, np.uint8) for _ in range(p)]
            if op == "encode":
                enc.Encode(sh)
            else:
                assert enc.EncodeVerify(sh), tag
            for r in range(k, n):
                assert np.array_equal(sh[r], full[r]), tag
        elif op == "verify":
            sh = [s.copy() for s in full]
            if rng.random() < 0.5:
                sh[int(rng.integers(0, n))][int(rng.integers(0, size))] ^= int(rng.integers(1, 256))
            e, want = oracle.verify(k, p, sh, kind)
            assert e == 0
            assert enc.Verify(sh) == want, tag
        elif op in ("reconstruct", "rdata", "decode"):
            lost = _lose(rng, n, p)
            src = [s.copy() for s in full]
            if rng.random() < 0.3:  # inconsistent survivors: output must still match upstream's
                src[int(rng.integers(0, n))][int(rng.integers(0, size))] ^= 0x81
            sh = [None if i in lost else src[i].copy() for i in range(n)]
            ref = [None if i in lost else src[i].copy() for i in range(n)]
            if op == "decode":
                ok = enc.DecodeVerify(sh)
                e, want = oracle.reconstruct(k, p, ref, kind)
                assert e == 0
                e2, want_ok = oracle.verify(k, p, want, kind)
                assert e2 == 0 and ok == want_ok, tag
            else:
                (enc.ReconstructData if op == "rdata" else enc.Reconstruct)(sh)
                e, want = oracle.reconstruct(k, p, ref, kind, data_only=(op == "rdata"))
                assert e == 0
            for i in range(n):
                if op == "rdata" and i >= k and i in lost:
                    assert sh[i] is None, tag  # parity left missing, as upstream
                    continue
                assert np.array_equal(sh[i], want[i]), (tag, lost, i)
        else:  # update: a random subset of data shards replaced
            sh = [s.copy() for s in full]
            newd = [None] * k
            for c in rng.choice(k, int(rng.integers(1, k + 1)), replace=False).tolist():
                newd[c] = rng.integers(0, 256, size, dtype=np.uint8)
            e, want = oracle.update(k, p, [s.copy() for s in full], newd, kind)
            assert e == 0
            enc.Update(sh, newd)
            for i in range(n):
                assert np.array_equal(sh[i], want[i]), (tag, i)


@pytest.mark.parametrize("seed", range(4))
def test_random_error_precedence_vs_oracle(gpu, seed):
    """Argument errors: same upstream error (or success) as the oracle."""
    rng = np.random.default_rng(2000 + seed)
    for _ in range(30):
        k = int(rng.integers(1, 12))
        p = int(rng.integers(1, 6))
        n = k + p
        size = int(rng.integers(1, 64))
        cnt = n if rng.random() < 0.8 else int(rng.integers(1, n + 3))
        sh = []
        for _ in range(cnt):
            r = rng.random()
            sh.append(None if r < 0.15 else rng.integers(0, 256, size if r < 0.9 else size + 1, dtype=np.uint8))
        op = str(rng.choice(["encode", "verify", "reconstruct"]))
        e, _ = {"encode": oracle.encode, "verify": oracle.verify,
                "reconstruct": oracle.reconstruct}[op](k, p, [None if s is None else s.copy() for s in sh])
        enc = ia.New(k, p)
        call = {"encode": enc.Encode, "verify": enc.Verify, "reconstruct": enc.Reconstruct}[op]
        mine = [None if s is None else s.copy() for s in sh]
        if e == 0:
            call(mine)
        elif e in ERRS:
            with pytest.raises(ERRS[e]):
                call(mine)
        else:
            with pytest.raises(ia.RSError):
                call(mine)


@pytest.mark.parametrize("seed", range(4))
def test_random_device_batches_vs_oracle(gpu, seed):
    """Device-resident batches (the bench path): random shapes, pitches and
    object counts, uniform and mixed erasure patterns, against the oracle."""
    import torch
    rng = np.random.default_rng(3000 + seed)
    for _ in range(4):
        k = int(rng.integers(2, 17))
        p = int(rng.integers(1, 5))
        n = k + p
        S = int(rng.integers(1, 30000))
        pitch = (S + 15) // 16 * 16 + 16 * int(rng.integers(0, 40))
        nobj = int(rng.integers(1, 40))
        enc = ia.New(k, p)
        m = enc.matrix()
        host = rng.integers(0, 256, (nobj, n, pitch), dtype=np.uint8)
        buf = torch.from_numpy(host.copy()).cuda()
        st = torch.cuda.current_stream()
        enc.encode_dev(buf, S, pitch, n * pitch, nobj, st)
        torch.cuda.synchronize()
        got = buf.cpu().numpy()
        for o in range(nobj):
            want = oracle.apply(m[k:], [host[o, c, :S] for c in range(k)])
            for r in range(p):
                assert np.array_equal(got[o, k + r, :S], want[r]), (seed, k, p, S, o, r)
        # mixed patterns: each object loses its own random <= p rows
        pres = np.ones((nobj, n), dtype=np.uint8)
        for o in range(nobj):
            pres[o, rng.choice(n, int(rng.integers(1, p + 1)), replace=False)] = 0
        coded = got.copy()
        for o in range(nobj):
            for i in range(n):
                if not pres[o, i]:
                    got[o, i, :S] = rng.integers(0, 256, S, dtype=np.uint8)  # garbage in lost rows
        buf = torch.from_numpy(got).cuda()
        bad = torch.full((nobj,), 7, dtype=torch.int32, device="cuda")
        enc.decode_dev_multi(buf, pres, S, pitch, n * pitch, nobj, bad, st)
        torch.cuda.synchronize()
        out = buf.cpu().numpy()
        assert int(bad.sum()) == 0, (seed, k, p, S)
        for o in range(nobj):
            for i in range(n):
                assert np.array_equal(out[o, i, :S], coded[o, i, :S]), (seed, k, p, S, o, i)


def _call_inplace(enc, fn, bufs, lens, *extra):
    """C-ABI call with every shard pointer into the caller's buffers and
    lens[i] == 0 marking a missing shard (the cgo shim's convention)."""
    import ctypes
    from infinicache_amd import _lib
    n = len(bufs)
    ptrs = ctypes.cast((ctypes.c_void_p * n)(*[b.__array_interface__["data"][0] for b in bufs]), _lib.u8pp)
    cl = (ctypes.c_size_t * n)(*lens)
    return getattr(enc._L, fn)(enc._ctx, ptrs, cl, n, *extra)


@pytest.mark.parametrize("seed", range(6))
def test_random_pinned_split_zero_copy_vs_oracle(gpu, seed):
    """Pinned Split buffers (rsgpu_host_alloc): the passes read and write the
    rows in place over PCIe (zero-copy).  Random shapes incl. sizes that are
    not multiples of 16 (the last row's tail vector reads into the slack),
    every op, missing rows anywhere (rlo > 0), corrupted survivors."""
    import ctypes
    rng = np.random.default_rng(4000 + seed)
    for _ in range(20):
        k = int(rng.integers(1, 17))
        p = int(rng.integers(1, 5))
        n = k + p
        size = int(rng.choice([1, 3, 15, 16, 17, 100, 1023, 4097, int(rng.integers(1, 30000))]))
        data = [rng.integers(0, 256, size, dtype=np.uint8) for _ in range(k)]
        e, full = oracle.encode(k, p, data + [bytes(size)] * p)
        assert e == 0
        host = ia.host_alloc(n * size)
        rows = [host[i * size:(i + 1) * size] for i in range(n)]
        enc = ia.New(k, p)
        op = str(rng.choice(["encode", "encode_verify", "verify", "reconstruct", "decode"]))
        tag = (seed, op, k, p, size)
        for i in range(n):
            rows[i][:] = full[i] if i < k or op in ("verify", "reconstruct", "decode") else 0x5C
        if op == "encode":
            assert _call_inplace(enc, "rsgpu_encode", rows, [size] * n) == 0, tag
            for r in range(k, n):
                assert np.array_equal(rows[r], full[r]), tag
        elif op == "encode_verify":
            ok = ctypes.c_int(0)
            assert _call_inplace(enc, "rsgpu_encode_verify", rows, [size] * n, ctypes.byref(ok)) == 0, tag
            assert ok.value == 1, tag
            for r in range(k, n):
                assert np.array_equal(rows[r], full[r]), tag
        elif op == "verify":
            if rng.random() < 0.5:
                rows[int(rng.integers(0, n))][int(rng.integers(0, size))] ^= 0x11
            e, want = oracle.verify(k, p, [r.copy() for r in rows])
            ok = ctypes.c_int(7)
            assert _call_inplace(enc, "rsgpu_verify", rows, [size] * n, ctypes.byref(ok)) == 0, tag
            assert bool(ok.value) == want, tag
        else:
            lost = _lose(rng, n, p)
            if rng.random() < 0.3:
                rows[int(rng.integers(0, n))][int(rng.integers(0, size))] ^= 0x81
            ref = [None if i in lost else rows[i].copy() for i in range(n)]
            for i in lost:
                rows[i][:] = 0xEE  # garbage where the rebuilt rows go
            lens = [0 if i in lost else size for i in range(n)]
            e, want = oracle.reconstruct(k, p, ref)
            assert e == 0
            if op == "decode":
                ok = ctypes.c_int(7)
                assert _call_inplace(enc, "rsgpu_decode", rows, lens, ctypes.byref(ok)) == 0, tag
                e2, want_ok = oracle.verify(k, p, want)
                assert bool(ok.value) == want_ok, tag
            else:
                assert _call_inplace(enc, "rsgpu_reconstruct", rows, lens, 0) == 0, tag
            for i in range(n):
                assert np.array_equal(rows[i], want[i]), (tag, lost, i)
