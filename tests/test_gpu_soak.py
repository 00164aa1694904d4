"""Time-bounded randomized soak of the HIP path against the CPU oracle
(oracle/, the restatement of klauspost/reedsolomon v1.9.3).  Off by default:
set RSGPU_SOAK_SECONDS (e.g. 240) to run it on the MI355X box; the regular
`-m gpu` suite skips it.  Each iteration draws one case from a wider space
than tests/test_gpu_random.py:
  * host ops (encode, encode_verify, verify, reconstruct, rdata, decode,
    update) with up to 40 data and 10 parity shards (the generic K > 16
    kernel) and both matrix kinds;
  * device batches: encode vs the oracle's batch port, per-object Verify
    flags after random corruption, fused decode (uniform pattern), mixed
    per-object patterns, ReconstructData; shard sizes from 1 B (packed
    small-object workgroups) to 40 KB, gaps between objects;
  * pinned Split buffers (zero-copy passes) for every per-object op;
  * round 2: narrow pitches (down to byte-packed rows), device-resolved mixed
    patterns (present masks in HBM, every status value), shard-major batches
    (encode vs the oracle, per-object Verify flags, fused decode);
  * round 3: the resident worker (every per-object op, pinned and pageable,
    codes of <= 16 shards, shards up to 16 KiB) and variable-size device
    tables (rsgpu_*_dev_objs: encode, Verify flags, fused decode,
    ReconstructData over objects of different sizes and pitches); device
    masks of 17-32-shard codes (no atlas: masks read back, host-planned);
  * round 4: worker objects past max_shard in pinned Split images (column
    slices over several mailboxes, shards up to 64 KiB) and host ops coded in
    column slabs (RSGPU_SLAB_BYTES drawn small, so objects of a few KB take
    several slabs), and pageable objects of 13-20 MB whose staging copies
    run on the host copy pool;
  * round 5: the host batch pipeline over random arenas (adjacent small
    objects in one H2D), pinned and pageable, with per-object Get patterns;
  * round 6: device batches of the codes the input-triples kernel serves
    (gf_apply_tri: RS(10+4) encode, Verify and Gets with 2-3 lost shards,
    RS(10+3) and RS(12+4) Verify) on rows past 128 vectors, with corrupted
    extra (checked) shards that must flag exactly their objects.
Every result is compared bit-exact (bytes) or exactly (booleans, error
classes) with the oracle on the same input.  Prints a per-kind case count."""
import collections
import ctypes
import os
import time

import numpy as np
import pytest

import infinicache_amd as ia
import oracle

SECONDS = float(os.environ.get("RSGPU_SOAK_SECONDS", "0"))
pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(SECONDS <= 0, reason="set RSGPU_SOAK_SECONDS to run the soak")]


def _size(rng, hi=40000):
    return int(rng.choice([1, 2, 15, 16, 17, 100, 103, 255, 410, 1023, 2048, 2049, 4097,
                           int(rng.integers(1, hi))]))


def _host_case(rng, counts):
    k = int(rng.integers(1, 41))
    p = int(rng.integers(1, 11))
    n = k + p
    size = _size(rng, 20000)
    kind = str(rng.choice(["vandermonde", "cauchy"]))
    data = [rng.integers(0, 256, size, dtype=np.uint8) for _ in range(k)]
    e, full = oracle.encode(k, p, data + [bytes(size)] * p, kind)
    assert e == 0
    enc = ia.New(k, p, matrix=kind)
    op = str(rng.choice(["encode", "encode_verify", "verify", "reconstruct", "rdata", "decode", "update"]))
    tag = ("host", op, k, p, size, kind)
    counts["host_" + op] += 1
    if op in ("encode", "encode_verify"):
        sh = [full[i].copy() for i in range(k)] + [np.full(size, 0x6B, np.uint8) for _ in range(p)]
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
        assert e == 0 and enc.Verify(sh) == want, tag
    elif op == "update":
        sh = [s.copy() for s in full]
        newd = [None] * k
        for c in rng.choice(k, int(rng.integers(1, k + 1)), replace=False).tolist():
            newd[c] = rng.integers(0, 256, size, dtype=np.uint8)
        e, want = oracle.update(k, p, [s.copy() for s in full], newd, kind)
        assert e == 0
        enc.Update(sh, newd)
        for i in range(n):
            assert np.array_equal(sh[i], want[i]), (tag, i)
    else:
        lost = sorted(rng.choice(n, int(rng.integers(1, p + 1)), replace=False).tolist())
        src = [s.copy() for s in full]
        if rng.random() < 0.3:
            src[int(rng.integers(0, n))][int(rng.integers(0, size))] ^= 0x81
        sh = [None if i in lost else src[i].copy() for i in range(n)]
        ref = [None if i in lost else src[i].copy() for i in range(n)]
        e, want = oracle.reconstruct(k, p, ref, kind, data_only=(op == "rdata"))
        assert e == 0
        if op == "decode":
            ok = enc.DecodeVerify(sh)
            e2, want_ok = oracle.verify(k, p, want, kind)
            assert e2 == 0 and ok == want_ok, tag
        else:
            (enc.ReconstructData if op == "rdata" else enc.Reconstruct)(sh)
        for i in range(n):
            if op == "rdata" and i >= k and i in lost:
                assert sh[i] is None, tag
                continue
            assert np.array_equal(sh[i], want[i]), (tag, lost, i)


def _device_case(rng, counts):
    import torch
    k = int(rng.integers(1, 31))
    p = int(rng.integers(1, 9))
    n = k + p
    S = _size(rng, 40000)
    if rng.random() < 0.25:  # narrow pitch (< 16 * ceil(S / 16)): partial tail stores
        pitch = (S + 3) // 4 * 4 if rng.random() < 0.5 else S
    else:
        pitch = (S + 15) // 16 * 16 + 16 * int(rng.integers(0, 3))
    gap = 16 * int(rng.integers(0, 8))
    stride = n * pitch + gap
    nobj = int(rng.integers(1, max(2, min(400, (24 << 20) // stride))))
    kind = str(rng.choice(["vandermonde", "cauchy"]))
    enc = ia.New(k, p, matrix=kind)
    m = enc.matrix()
    host = rng.integers(0, 256, (nobj, stride), dtype=np.uint8)
    for i in range(n):  # zero pads (written rows' pads get the pads' coding)
        host[:, i * pitch + S:(i + 1) * pitch] = 0
    buf = torch.from_numpy(host.copy()).cuda()
    st = torch.cuda.current_stream()
    tag = ("dev", k, p, S, pitch, gap, nobj, kind)
    enc.encode_dev(buf, S, pitch, stride, nobj, st)
    torch.cuda.synchronize()
    got = buf.cpu().numpy()
    ref = host.copy()
    oracle.code_batch(m[k:], list(range(k)), list(range(k, n)), ref.reshape(-1), stride, pitch, S, nobj,
                      nthreads=8)
    assert np.array_equal(got, ref), tag
    counts["dev_encode"] += 1
    coded = got.copy()
    op = str(rng.choice(["verify", "decode", "multi", "rdata"]))
    counts["dev_" + op] += 1
    if op == "verify":
        hit = sorted(set(rng.integers(0, nobj, int(rng.integers(0, min(nobj, 6) + 1))).tolist()))
        for o in hit:
            r = int(rng.integers(0, n))
            got[o, r * pitch + int(rng.integers(0, S))] ^= int(rng.integers(1, 256))
        buf = torch.from_numpy(got).cuda()
        bad = torch.full((nobj,), 9, dtype=torch.int32, device="cuda")
        enc.verify_dev(buf, S, pitch, stride, nobj, bad, st)
        torch.cuda.synchronize()
        assert np.flatnonzero(bad.cpu().numpy()).tolist() == hit, tag
        return
    if op == "multi":
        pres = np.ones((nobj, n), dtype=np.uint8)
        for o in range(nobj):
            pres[o, rng.choice(n, int(rng.integers(1, p + 1)), replace=False)] = 0
    else:
        row = np.ones(n, dtype=np.uint8)
        row[rng.choice(n, int(rng.integers(1, p + 1)), replace=False)] = 0
        pres = np.tile(row, (nobj, 1))
    for o in range(nobj):
        for i in range(n):
            if not pres[o, i]:
                got[o, i * pitch:i * pitch + S] = rng.integers(0, 256, S, dtype=np.uint8)
    buf = torch.from_numpy(got.copy()).cuda()
    bad = torch.full((nobj,), 9, dtype=torch.int32, device="cuda")
    if op == "multi":
        enc.decode_dev_multi(buf, pres, S, pitch, stride, nobj, bad, st)
    elif op == "decode":
        enc.decode_dev(buf, [bool(x) for x in pres[0]], S, pitch, stride, nobj, bad, st)
    else:
        enc.reconstruct_dev(buf, [bool(x) for x in pres[0]], S, pitch, stride, nobj, data_only=True,
                            stream=st)
    torch.cuda.synchronize()
    out = buf.cpu().numpy()
    if op != "rdata":
        assert int(bad.sum()) == 0, tag
    for o in range(nobj):
        for i in range(n):
            if op == "rdata" and i >= k and not pres[o, i]:
                continue  # parity left as it was
            a = out[o, i * pitch:i * pitch + S]
            assert np.array_equal(a, coded[o, i * pitch:i * pitch + S]), (tag, op, o, i)
    # bytes outside the rebuilt rows' valid ranges are untouched (gaps, pads of other rows)
    assert np.array_equal(out[:, n * pitch:], got[:, n * pitch:]), tag


def _tri_case(rng, counts):
    import torch
    k, p = [(10, 4), (10, 4), (10, 3), (12, 4)][int(rng.integers(0, 4))]
    n = k + p
    S = int(rng.integers(2049, 60000))
    pitch = (S + 3) // 4 * 4 if rng.random() < 0.3 else (S + 15) // 16 * 16 + 16 * int(rng.integers(0, 3))
    stride = n * pitch + 16 * int(rng.integers(0, 4))
    nobj = int(rng.integers(1, 12))
    kind = str(rng.choice(["vandermonde", "cauchy"]))
    enc = ia.New(k, p, matrix=kind)
    m = enc.matrix()
    host = rng.integers(0, 256, (nobj, stride), dtype=np.uint8)
    for i in range(n):
        host[:, i * pitch + S:(i + 1) * pitch] = 0
    buf = torch.from_numpy(host.copy()).cuda()
    st = torch.cuda.current_stream()
    tag = ("tri", k, p, S, pitch, stride, nobj, kind)
    enc.encode_dev(buf, S, pitch, stride, nobj, st)
    torch.cuda.synchronize()
    coded = host.copy()
    oracle.code_batch(m[k:], list(range(k)), list(range(k, n)), coded.reshape(-1), stride, pitch, S, nobj,
                      nthreads=8)
    assert np.array_equal(buf.cpu().numpy(), coded), tag
    counts["tri_encode"] += 1
    got = coded.copy()
    if rng.random() < 0.4:  # Verify: every parity row checked
        hit = sorted(set(rng.integers(0, nobj, int(rng.integers(0, min(nobj, 4) + 1))).tolist()))
        for o in hit:
            got[o, int(rng.integers(0, n)) * pitch + int(rng.integers(0, S))] ^= int(rng.integers(1, 256))
        buf = torch.from_numpy(got).cuda()
        bad = torch.full((nobj,), 9, dtype=torch.int32, device="cuda")
        enc.verify_dev(buf, S, pitch, stride, nobj, bad, st)
        torch.cuda.synchronize()
        assert np.flatnonzero(bad.cpu().numpy()).tolist() == hit, tag
        counts["tri_verify"] += 1
        return
    # a Get: 2 or 3 shards lost (data or parity), the extra present shards checked
    lost = sorted(rng.choice(n, int(rng.integers(2, min(p, 3) + 1)), replace=False).tolist())
    present = [i not in lost for i in range(n)]
    extras = [i for i in range(n) if present[i]][k:]
    hit = []
    if extras and rng.random() < 0.6:
        hit = sorted(set(rng.integers(0, nobj, int(rng.integers(1, min(nobj, 3) + 1))).tolist()))
        for o in hit:
            e = extras[int(rng.integers(0, len(extras)))]
            got[o, e * pitch + int(rng.integers(0, S))] ^= int(rng.integers(1, 256))
    for o in range(nobj):
        for i in lost:
            got[o, i * pitch:i * pitch + S] = rng.integers(0, 256, S, dtype=np.uint8)
    buf = torch.from_numpy(got.copy()).cuda()
    bad = torch.full((nobj,), 9, dtype=torch.int32, device="cuda")
    enc.decode_dev(buf, present, S, pitch, stride, nobj, bad, st)
    torch.cuda.synchronize()
    out = buf.cpu().numpy()
    assert np.flatnonzero(bad.cpu().numpy()).tolist() == hit, (tag, lost, hit)
    for o in range(nobj):  # rebuilt from the first k present, which no corruption touched
        for i in lost:
            assert np.array_equal(out[o, i * pitch:i * pitch + S], coded[o, i * pitch:i * pitch + S]), (tag, lost, o, i)
    counts[f"tri_get_{len(lost)}lost"] += 1


def _masks_case(rng, counts):
    """Device-resolved mixed patterns: every object its own present mask
    (too few shards, an extra present parity shard corrupted, all present),
    decode / reconstruct / data-only; rebuilt rows vs the coded batch."""
    import torch
    k = int(rng.integers(1, 15))
    p = int(rng.integers(1, min(8, 16 - k) + 1))
    if rng.random() < 0.25:  # 17-32 shards: no device atlas (masks read back, host-planned)
        k = int(rng.integers(10, 29))
        p = int(rng.integers(max(1, 17 - k), min(8, 32 - k) + 1))
    n = k + p
    S = _size(rng, 30000)
    pitch = (S + 15) // 16 * 16 + 16 * int(rng.integers(0, 2))
    stride = n * pitch + 16 * int(rng.integers(0, 4))
    nobj = int(rng.integers(1, max(2, min(300, (16 << 20) // stride))))
    op = str(rng.choice(["decode", "reconstruct", "rdata"]))
    counts["masks_" + op] += 1
    enc = ia.New(k, p)
    host = rng.integers(0, 256, (nobj, stride), dtype=np.uint8)
    for i in range(n):
        host[:, i * pitch + S:(i + 1) * pitch] = 0
    buf = torch.from_numpy(host).cuda()
    st = torch.cuda.current_stream()
    enc.encode_dev(buf, S, pitch, stride, nobj, st)
    torch.cuda.synchronize()
    coded = buf.cpu().numpy()
    got = coded.copy()
    pres = np.ones((nobj, n), dtype=np.uint8)
    want_status = np.zeros(nobj, np.int64)
    for o in range(nobj):
        nl = int(rng.integers(0, p + 2))  # p + 1: too few shards
        pres[o, rng.choice(n, min(nl, n), replace=False)] = 0
        if pres[o].sum() < k:
            want_status[o] = 2
            continue
        for i in np.flatnonzero(pres[o] == 0):
            got[o, i * pitch:i * pitch + S] = rng.integers(0, 256, S, dtype=np.uint8)
        last = int(np.nonzero(pres[o])[0][-1])
        if op == "decode" and pres[o].sum() > k and last >= k and rng.random() < 0.3:
            got[o, last * pitch + int(rng.integers(0, S))] ^= 0x24  # an extra (checked) shard
            want_status[o] = 1
    masks = (pres.astype(np.int64) << np.arange(n)).sum(axis=1).astype(np.int32)
    buf = torch.from_numpy(got.copy()).cuda()
    status = torch.full((nobj,), 9, dtype=torch.int32, device="cuda")
    dm = torch.from_numpy(masks).cuda()
    if op == "decode":
        enc.decode_dev_masks(buf, dm, S, pitch, stride, nobj, status, st)
    else:
        enc.reconstruct_dev_masks(buf, dm, S, pitch, stride, nobj, data_only=op == "rdata", status=status,
                                  stream=st)
    torch.cuda.synchronize()
    out = buf.cpu().numpy()
    tag = ("masks", op, k, p, S, pitch, nobj)
    assert np.array_equal(status.cpu().numpy(), want_status), tag
    for o in range(nobj):
        if want_status[o] == 2:
            assert np.array_equal(out[o], got[o]), tag
            continue
        for i in range(n):
            a = out[o, i * pitch:i * pitch + S]
            if pres[o, i] or (op == "rdata" and i >= k):
                assert np.array_equal(a, got[o, i * pitch:i * pitch + S]), (tag, o, i)
            else:
                assert np.array_equal(a, coded[o, i * pitch:i * pitch + S]), (tag, o, i)


def _shard_major_case(rng, counts):
    """[shard][object] batches: encode vs the oracle (the batch is one long
    object per row), Verify flags per object, fused decode."""
    import torch
    k = int(rng.integers(1, 21))
    p = int(rng.integers(1, 7))
    n = k + p
    S = _size(rng, 5000)
    ostride = S if rng.random() < 0.5 else (S + 15) // 16 * 16
    nobj = int(rng.integers(2, max(3, min(3000, (8 << 20) // (n * ostride)))))
    pitch = nobj * ostride + 16 * int(rng.integers(0, 3))
    counts["shardmajor"] += 1
    enc = ia.New(k, p)
    m = enc.matrix()
    host = np.zeros((n, pitch), np.uint8)
    for i in range(k):
        host[i, :nobj * ostride].reshape(nobj, ostride)[:, :S] = rng.integers(0, 256, (nobj, S), dtype=np.uint8)
    buf = torch.from_numpy(host.copy()).cuda()
    st = torch.cuda.current_stream()
    enc.encode_dev(buf, S, pitch, ostride, nobj, st)
    torch.cuda.synchronize()
    got = buf.cpu().numpy()
    piece = lambda a, i: a[i, :nobj * ostride].reshape(nobj, ostride)[:, :S]
    want = oracle.apply(m[k:], [piece(host, i).reshape(-1) for i in range(k)])
    tag = ("shardmajor", k, p, S, ostride, nobj)
    for r in range(p):
        assert np.array_equal(piece(got, k + r).reshape(-1), want[r]), tag
    hit = sorted(set(rng.integers(0, nobj, int(rng.integers(0, 5))).tolist()))
    bad_in = got.copy()
    for o in hit:
        piece(bad_in, int(rng.integers(0, n)))[o, int(rng.integers(0, S))] ^= 0x42
    bad = torch.full((nobj,), 9, dtype=torch.int32, device="cuda")
    enc.verify_dev(torch.from_numpy(bad_in).cuda(), S, pitch, ostride, nobj, bad, st)
    torch.cuda.synchronize()
    assert np.flatnonzero(bad.cpu().numpy()).tolist() == hit, tag
    lost = sorted(rng.choice(n, int(rng.integers(1, p + 1)), replace=False).tolist())
    erased = got.copy()
    for i in lost:
        piece(erased, i)[:] = 0xA5
    buf = torch.from_numpy(erased).cuda()
    bad.fill_(9)
    enc.decode_dev(buf, [i not in lost for i in range(n)], S, pitch, ostride, nobj, bad, st)
    torch.cuda.synchronize()
    out = buf.cpu().numpy()
    assert not bad.any(), tag
    for i in range(n):
        assert np.array_equal(piece(out, i), piece(got, i)), (tag, lost, i)


def _call(enc, fn, bufs, lens, *extra):
    n = len(bufs)
    from infinicache_amd import _lib
    ptrs = ctypes.cast((ctypes.c_void_p * n)(*[b.__array_interface__["data"][0] for b in bufs]), _lib.u8pp)
    return getattr(enc._L, fn)(enc._ctx, ptrs, (ctypes.c_size_t * n)(*lens), n, *extra)


def _pinned_case(rng, counts):
    k = int(rng.integers(1, 17))
    p = int(rng.integers(1, 5))
    n = k + p
    size = _size(rng, 60000)
    data = [rng.integers(0, 256, size, dtype=np.uint8) for _ in range(k)]
    e, full = oracle.encode(k, p, data + [bytes(size)] * p)
    assert e == 0
    host = ia.host_alloc(n * size)
    rows = [host[i * size:(i + 1) * size] for i in range(n)]
    enc = ia.New(k, p)
    op = str(rng.choice(["encode", "encode_verify", "verify", "reconstruct", "decode"]))
    counts["pinned_" + op] += 1
    tag = ("pinned", op, k, p, size)
    for i in range(n):
        rows[i][:] = full[i] if i < k or op in ("verify", "reconstruct", "decode") else 0x5C
    if op in ("encode", "encode_verify"):
        if op == "encode":
            assert _call(enc, "rsgpu_encode", rows, [size] * n) == 0, tag
        else:
            ok = ctypes.c_int(0)
            assert _call(enc, "rsgpu_encode_verify", rows, [size] * n, ctypes.byref(ok)) == 0, tag
            assert ok.value == 1, tag
        for r in range(k, n):
            assert np.array_equal(rows[r], full[r]), tag
    elif op == "verify":
        if rng.random() < 0.5:
            rows[int(rng.integers(0, n))][int(rng.integers(0, size))] ^= 0x11
        e, want = oracle.verify(k, p, [r.copy() for r in rows])
        ok = ctypes.c_int(7)
        assert _call(enc, "rsgpu_verify", rows, [size] * n, ctypes.byref(ok)) == 0, tag
        assert bool(ok.value) == want, tag
    else:
        lost = sorted(rng.choice(n, int(rng.integers(1, p + 1)), replace=False).tolist())
        if rng.random() < 0.3:
            rows[int(rng.integers(0, n))][int(rng.integers(0, size))] ^= 0x81
        ref = [None if i in lost else rows[i].copy() for i in range(n)]
        for i in lost:
            rows[i][:] = 0xEE
        lens = [0 if i in lost else size for i in range(n)]
        e, want = oracle.reconstruct(k, p, ref)
        assert e == 0
        if op == "decode":
            ok = ctypes.c_int(7)
            assert _call(enc, "rsgpu_decode", rows, lens, ctypes.byref(ok)) == 0, tag
            e2, want_ok = oracle.verify(k, p, want)
            assert e2 == 0 and bool(ok.value) == want_ok, tag
        else:
            assert _call(enc, "rsgpu_reconstruct", rows, lens, 0) == 0, tag
        for i in range(n):
            assert np.array_equal(rows[i], want[i]), (tag, lost, i)


_WORKERS = {}


def _worker_enc(k, p, kind):
    """one worker-enabled encoder per code (a start builds atlases and launches)"""
    key = (k, p, kind)
    if key not in _WORKERS:
        if len(_WORKERS) >= 6:
            _WORKERS.pop(next(iter(_WORKERS))).worker_stop()
        enc = ia.New(k, p, matrix=kind)
        enc.worker_start(nslots=4)
        _WORKERS[key] = enc
    return _WORKERS[key]


def _worker_case(rng, counts):
    k = int(rng.integers(1, 14))
    p = int(rng.integers(1, min(5, 16 - k) + 1))
    n = k + p
    size = _size(rng, 16384 if rng.random() < 0.7 else 65536)
    kind = str(rng.choice(["vandermonde", "cauchy"]))
    enc = _worker_enc(k, p, kind)
    data = [rng.integers(0, 256, size, dtype=np.uint8) for _ in range(k)]
    e, full = oracle.encode(k, p, data + [bytes(size)] * p, kind)
    assert e == 0
    pinned = rng.random() < 0.5
    if pinned:
        host = ia.host_alloc(n * size)
        rows = [host[i * size:(i + 1) * size] for i in range(n)]
    else:
        rows = [np.empty(size, np.uint8) for _ in range(n)]
    op = str(rng.choice(["encode", "encode_verify", "verify", "reconstruct", "rdata", "decode"]))
    counts["worker_" + op] += 1
    tag = ("worker", op, k, p, size, kind, pinned)
    for i in range(n):
        rows[i][:] = full[i] if i < k or op not in ("encode", "encode_verify") else 0x5C
    if op in ("encode", "encode_verify"):
        if op == "encode":
            enc.Encode(rows)
        else:
            assert enc.EncodeVerify(rows), tag
        for r in range(k, n):
            assert np.array_equal(rows[r], full[r]), tag
    elif op == "verify":
        if rng.random() < 0.5:
            rows[int(rng.integers(0, n))][int(rng.integers(0, size))] ^= 0x11
        e, want = oracle.verify(k, p, [r.copy() for r in rows], kind)
        assert e == 0 and enc.Verify(rows) == want, tag
    else:
        lost = sorted(rng.choice(n, int(rng.integers(1, p + 1)), replace=False).tolist())
        if rng.random() < 0.3:
            rows[int(rng.integers(0, n))][int(rng.integers(0, size))] ^= 0x81
        ref = [None if i in lost else rows[i].copy() for i in range(n)]
        e, want = oracle.reconstruct(k, p, [None if r is None else r.copy() for r in ref], kind,
                                     data_only=(op == "rdata"))
        assert e == 0
        lens = [0 if i in lost else size for i in range(n)]
        for i in lost:
            rows[i][:] = 0xEE
        if op == "decode":
            ok = ctypes.c_int(7)
            assert _call(enc, "rsgpu_decode", rows, lens, ctypes.byref(ok)) == 0, tag
            e2, want_ok = oracle.verify(k, p, want, kind)
            assert e2 == 0 and bool(ok.value) == want_ok, tag
        else:
            assert _call(enc, "rsgpu_reconstruct", rows, lens, int(op == "rdata")) == 0, tag
        for i in range(n):
            if op == "rdata" and i >= k and i in lost:
                assert (rows[i] == 0xEE).all(), tag  # missing parity left alone
                continue
            assert np.array_equal(rows[i], want[i]), (tag, lost, i)


def _objs_case(rng, counts):
    """variable-size device tables: objects of different sizes and pitches,
    one launch per pass"""
    import torch
    k = int(rng.integers(1, 21))
    p = int(rng.integers(1, 7))
    n = k + p
    kind = str(rng.choice(["vandermonde", "cauchy"]))
    enc = ia.New(k, p, matrix=kind)
    m = enc.matrix()
    nobj = int(rng.integers(1, 40))
    layout, off = [], 0
    for _ in range(nobj):
        S = _size(rng, 60000)
        pitch = (S + 15) // 16 * 16 + 16 * int(rng.integers(0, 3))
        layout.append((off, S, pitch))
        off += n * pitch + 16 * int(rng.integers(0, 4))
    host = rng.integers(0, 256, off + 64, dtype=np.uint8)
    buf = torch.from_numpy(host.copy()).cuda()
    objs = [(buf.data_ptr() + o, S, pitch) for o, S, pitch in layout]
    st = torch.cuda.current_stream()
    tag = ("objs", k, p, nobj, kind)
    enc.encode_dev_objs(objs, st)
    torch.cuda.synchronize()
    got = buf.cpu().numpy()
    rows = lambda a, o, S, pitch: [a[o + i * pitch: o + i * pitch + S] for i in range(n)]
    for o, S, pitch in layout:
        r = rows(got, o, S, pitch)
        want = oracle.apply(m[k:], [h.copy() for h in rows(host, o, S, pitch)[:k]])
        for j in range(p):
            assert np.array_equal(r[k + j], want[j]), (tag, S)
    counts["objs_encode"] += 1
    coded = got.copy()
    op = str(rng.choice(["verify", "decode", "rdata"]))
    counts["objs_" + op] += 1
    bad = torch.full((nobj,), 9, dtype=torch.int32, device="cuda")
    if op == "verify":
        hit = sorted(set(rng.integers(0, nobj, int(rng.integers(0, min(nobj, 5) + 1))).tolist()))
        for i in hit:
            o, S, pitch = layout[i]
            got[o + int(rng.integers(0, n)) * pitch + int(rng.integers(0, S))] ^= 0x33
        buf = torch.from_numpy(got).cuda()
        objs = [(buf.data_ptr() + o, S, pitch) for o, S, pitch in layout]
        enc.verify_dev_objs(objs, bad, st)
        torch.cuda.synchronize()
        assert np.flatnonzero(bad.cpu().numpy()).tolist() == hit, tag
        return
    lost = sorted(rng.choice(n, int(rng.integers(1, p + 1)), replace=False).tolist())
    for o, S, pitch in layout:
        for i in lost:
            got[o + i * pitch: o + i * pitch + S] = 0xA5
    buf = torch.from_numpy(got.copy()).cuda()
    objs = [(buf.data_ptr() + o, S, pitch) for o, S, pitch in layout]
    present = [i not in lost for i in range(n)]
    if op == "decode":
        enc.decode_dev_objs(objs, present, bad, st)
    else:
        enc.reconstruct_dev_objs(objs, present, data_only=True, stream=st)
    torch.cuda.synchronize()
    out = buf.cpu().numpy()
    if op == "decode":
        assert not bad.any(), tag
    for o, S, pitch in layout:
        for i in range(n):
            a = out[o + i * pitch: o + i * pitch + S]
            if op == "rdata" and i >= k and i in lost:
                assert (a == 0xA5).all(), tag
            else:
                assert np.array_equal(a, coded[o + i * pitch: o + i * pitch + S]), (tag, op, lost, i)


def _large_pageable_case(rng, counts):
    """a pageable object past the host copy pool's threshold (12 MiB of rows):
    the staging copies run on the pool (hostcopy.cpp)"""
    k, p = 10, int(rng.integers(1, 5))
    n = k + p
    size = int(rng.integers(1_300_000, 2_000_000))
    data = [rng.integers(0, 256, size, dtype=np.uint8) for _ in range(k)]
    e, full = oracle.encode(k, p, data + [bytes(size)] * p)
    assert e == 0
    enc = ia.New(k, p)
    sh = [np.frombuffer(bytes(full[i]), np.uint8).copy() if i < k else np.zeros(size, np.uint8) for i in range(n)]
    assert enc.EncodeVerify(sh)
    for i in range(k, n):
        assert np.array_equal(sh[i], np.frombuffer(bytes(full[i]), np.uint8)), ("large", i)
    lost = sorted(rng.choice(n, p, replace=False).tolist())
    got = [None if i in lost else sh[i] for i in range(n)]
    assert enc.DecodeVerify(got)
    for i in lost:
        assert np.array_equal(got[i], np.frombuffer(bytes(full[i]), np.uint8)), ("large", lost, i)
    counts["large_pageable"] += 1


def _slab_case(rng, counts):
    """a host op with a small slab size: the object is coded in column slabs"""
    ia.set_slab_bytes(int(rng.integers(4096, 1 << 16)))
    try:
        _host_case(rng, counts)
        counts["slabs"] += 1
    finally:
        ia.set_slab_bytes(0)


def _batch_case(rng, counts):
    """round 5: the host batch pipeline (rsgpu_encode_batch / _decode_batch):
    1-14 objects of 1 B - 700 KB (now and then one past the 4 MiB group
    limit), Split images back to back in one arena with random gaps (runs of
    adjacent small objects move as one H2D), pinned or pageable; encode vs
    the oracle, then a Get per object with its own present pattern (exactly
    k bodies, or extra bodies with a corrupted one: coded alone, flagged)."""
    k = int(rng.integers(1, 17))
    p = int(rng.integers(1, 5))
    n = k + p
    kind = str(rng.choice(["vandermonde", "cauchy"]))
    enc = ia.New(k, p, matrix=kind)
    nobj = int(rng.integers(1, 15))
    sizes = [_size(rng, 700000) for _ in range(nobj)]
    if rng.random() < 0.1:
        sizes[int(rng.integers(0, nobj))] = int(rng.integers(4 << 20, 6 << 20))
    Ss = [(nb + k - 1) // k for nb in sizes]
    gaps = [int(rng.choice([0, 0, 0, 16, 4096])) for _ in range(nobj)]
    total = sum(n * S + g for S, g in zip(Ss, gaps))
    pinned = rng.random() < 0.5
    arena = ia.host_alloc(total) if pinned else np.empty(total, np.uint8)
    objs, fulls, off = [], [], 0
    for S, g in zip(Ss, gaps):
        data = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)]
        e, full = oracle.encode(k, p, data + [bytes(S)] * p, kind)
        assert e == 0
        img = arena[off:off + n * S]
        for i in range(k):
            img[i * S:(i + 1) * S] = full[i]
        img[k * S:] = 0x3C
        objs.append([img[i * S:(i + 1) * S] for i in range(n)])
        fulls.append(full)
        off += n * S + g
    tag = ("batch", k, p, kind, nobj, sizes, gaps, pinned)
    enc.encode_batch(objs)
    for o in range(nobj):
        for i in range(k, n):
            assert np.array_equal(objs[o][i], fulls[o][i]), (tag, o, i)
    present, want_ok = [], []
    for o in range(nobj):
        nlost = int(rng.integers(0, p + 1))
        lost = set(rng.choice(n, nlost, replace=False).tolist())
        pr = [i not in lost for i in range(n)]
        for i in lost:
            objs[o][i][:] = 0xA5
        ok = True
        extra = [i for i in range(n) if pr[i]][k:]
        if extra and rng.random() < 0.3:  # a corrupted body beyond the survivors
            j = extra[int(rng.integers(0, len(extra)))]
            objs[o][j][int(rng.integers(0, Ss[o]))] ^= 0x5A
            ok = j < k  # upstream Verify compares parity rows only
        present.append(pr)
        want_ok.append(ok)
    counts["batch_" + ("pinned" if pinned else "pageable")] += 1
    got = enc.decode_batch(objs, present=present)
    for o in range(nobj):
        if not want_ok[o] or got[o] != want_ok[o]:
            # the oracle decides (a corrupted data extra still verifies)
            ref = [objs[o][i].copy() if present[o][i] else None for i in range(n)]
            e, rec = oracle.reconstruct(k, p, ref, kind)
            assert e == 0
            e, v = oracle.verify(k, p, rec, kind)
            assert e == 0 and got[o] == v, (tag, o)
        for i in range(n):
            if not present[o][i]:
                assert np.array_equal(objs[o][i], fulls[o][i]), (tag, o, i)


def test_gpu_soak_vs_oracle(gpu):
    seed = int(os.environ.get("RSGPU_SOAK_SEED", "20261016"))
    rng = np.random.default_rng(seed)
    counts = collections.Counter()
    t0 = last = time.time()
    while time.time() - t0 < SECONDS:
        r = rng.random()
        if r < 0.22:
            _host_case(rng, counts)
        elif r < 0.36:
            _device_case(rng, counts)
        elif r < 0.42:
            _tri_case(rng, counts)
        elif r < 0.54:
            _masks_case(rng, counts)
        elif r < 0.66:
            _shard_major_case(rng, counts)
        elif r < 0.76:
            _pinned_case(rng, counts)
        elif r < 0.88:
            _worker_case(rng, counts)
        elif r < 0.94:
            _objs_case(rng, counts)
        elif r < 0.96:
            _slab_case(rng, counts)
        elif r < 0.99:
            _batch_case(rng, counts)
        else:
            _large_pageable_case(rng, counts)
        if time.time() - last > 30:  # progress line (a silent GPU run reads as hung)
            last = time.time()
            print(f"soak {last - t0:.0f}s: {sum(counts.values())} cases", flush=True)
    for enc in _WORKERS.values():
        enc.worker_stop()
    _WORKERS.clear()
    print(f"soak seed {seed}, {time.time() - t0:.0f} s, {sum(counts.values())} cases:", flush=True)
    for key in sorted(counts):
        print(f"  {key:22s} {counts[key]}", flush=True)
