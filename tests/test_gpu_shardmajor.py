"""Shard-major batches ([shard][object]: shard i of object o at
base + i*pitch + o*obj_stride) against the CPU oracle, bit-exact.

InfiniCache sends shard i of an object to Lambda node i (client/ecRedis.go
EcSet, one RESP set per shard, :58-129); a batch laid out shard-major keeps
each node's shards of many objects contiguous.  Coding is byte-position-wise,
so such a batch is coded as ONE object whose shard is the whole row
(gf_kernels.hip launch_plan): small objects stream at the large-object rate.
Covered: pieces back to back (obj_stride = S) and 16-B aligned (gaps are pad
bytes), per-object Verify flags and decode clears attributed by byte
position, corrupted pad gaps not flagged, a tight pitch (the last object goes
through the scratch path), K > 16, and the device-resolved mixed patterns."""
import numpy as np
import pytest

import infinicache_amd as ia
import oracle

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def _batch(k, p, S, nobj, stride, pitch, seed):
    n = k + p
    g = torch.Generator(device="cuda").manual_seed(seed)
    flat = torch.zeros(n * pitch, dtype=torch.uint8, device="cuda")
    rows = flat.view(n, pitch)
    for i in range(n):  # only the pieces hold data; gaps and row tails zero
        piece = torch.randint(0, 256, (nobj, S), dtype=torch.uint8, device="cuda", generator=g)
        rows[i, :nobj * stride].view(nobj, stride)[:, :S] = piece if stride > S else piece
    return flat, rows


def _pieces(rows, i, nobj, S, stride):
    return rows[i, :nobj * stride].view(nobj, stride)[:, :S]


def _expect_parity(enc, rows, k, p, nobj, S, stride):
    h = rows.cpu().numpy()
    m = enc.matrix()
    data = [h[i, :nobj * stride].reshape(nobj, stride)[:, :S].reshape(-1) for i in range(k)]
    return oracle.apply(m[k:], data)  # the batch IS one object: one long row per shard


@pytest.mark.parametrize("k,p,S,nobj,aligned", [(10, 2, 103, 5000, False), (10, 2, 103, 5000, True),
                                                (10, 4, 1, 3000, False), (10, 2, 17, 777, True),
                                                (10, 2, 4096, 300, False), (6, 3, 1000, 50, True),
                                                (20, 4, 103, 600, False)])
def test_shard_major_encode_verify_decode(gpu, k, p, S, nobj, aligned):
    n = k + p
    stride = (S + 15) // 16 * 16 if aligned else S
    pitch = (nobj * stride + 255) // 256 * 256
    flat, rows = _batch(k, p, S, nobj, stride, pitch, seed=S * 31 + nobj)
    enc = ia.New(k, p)
    s = torch.cuda.current_stream()
    before = rows.clone()
    enc.encode_dev(flat, S, pitch, stride, nobj, s)
    torch.cuda.synchronize()
    want = _expect_parity(enc, before, k, p, nobj, S, stride)
    for r in range(p):
        got = _pieces(rows, k + r, nobj, S, stride).cpu().numpy().reshape(-1)
        assert np.array_equal(got, want[r]), r
    # data rows untouched
    assert torch.equal(rows[:k], before[:k])
    # Verify: per-object flags; garbage in the pad gaps is not a mismatch
    hit = sorted({0, nobj - 1, nobj // 3})
    for o in hit:
        _pieces(rows, (o * 5) % n, nobj, S, stride)[o, (o * 7) % S] ^= 0x5A
    if aligned and stride > S:
        rows[:, :nobj * stride].view(n, nobj, stride)[:, 1::2, S:] = 0xEE  # pads
    bad = torch.full((nobj,), 9, dtype=torch.int32, device="cuda")
    enc.verify_dev(flat, S, pitch, stride, nobj, bad, s)
    torch.cuda.synchronize()
    if k <= 16:  # K <= 16: one launch over the whole row, flags by byte position
        assert np.flatnonzero(bad.cpu().numpy()).tolist() == hit
    else:  # K > 16 with flags: per-object launches, same flags
        assert np.flatnonzero(bad.cpu().numpy()).tolist() == hit
    for o in hit:
        _pieces(rows, (o * 5) % n, nobj, S, stride)[o, (o * 7) % S] ^= 0x5A
    golden = [_pieces(rows, i, nobj, S, stride).clone() for i in range(n)]
    # fused decode (healthy Get: data 0 and k//2 lost) clears every flag
    lost = (0, k // 2)
    for i in lost:
        _pieces(rows, i, nobj, S, stride).fill_(0xC3)
    bad.fill_(7)
    enc.decode_dev(flat, [i not in lost for i in range(n)], S, pitch, stride, nobj, bad, s)
    torch.cuda.synchronize()
    assert not bad.any()
    for i in range(n):
        assert torch.equal(_pieces(rows, i, nobj, S, stride), golden[i]), i


@pytest.mark.parametrize("k,p,S,stride,nobj", [(10, 2, 103, 128, 3000), (10, 2, 100, 128, 2000), (10, 4, 410, 512, 700),
                                               (20, 4, 103, 128, 500)])
def test_shard_major_wide_gaps(gpu, k, p, S, stride, nobj):
    """Pieces at a stride past roundup16(S): gaps up to S/4 are coded along
    as pad bytes (one-object conversion: 103 -> 128, 410 -> 512), wider ones
    (100 -> 128) object by object; parity, per-object Verify flags (garbage in
    the gaps is not a mismatch) and fused decode against the oracle."""
    n = k + p
    pitch = (nobj * stride + 255) // 256 * 256
    flat, rows = _batch(k, p, S, nobj, stride, pitch, seed=S + stride + nobj)
    enc = ia.New(k, p)
    s = torch.cuda.current_stream()
    before = rows.clone()
    enc.encode_dev(flat, S, pitch, stride, nobj, s)
    torch.cuda.synchronize()
    want = _expect_parity(enc, before, k, p, nobj, S, stride)
    for r in range(p):
        assert np.array_equal(_pieces(rows, k + r, nobj, S, stride).cpu().numpy().reshape(-1), want[r]), r
    assert torch.equal(rows[:k], before[:k])
    rows[:, :nobj * stride].view(n, nobj, stride)[:, ::3, S:] = 0x5D  # garbage in the gaps
    hit = sorted({1, nobj // 2, nobj - 1})
    for o in hit:
        _pieces(rows, (o * 3) % n, nobj, S, stride)[o, (o * 11) % S] ^= 0x81
    bad = torch.full((nobj,), 9, dtype=torch.int32, device="cuda")
    enc.verify_dev(flat, S, pitch, stride, nobj, bad, s)
    torch.cuda.synchronize()
    assert np.flatnonzero(bad.cpu().numpy()).tolist() == hit
    for o in hit:
        _pieces(rows, (o * 3) % n, nobj, S, stride)[o, (o * 11) % S] ^= 0x81
    golden = [_pieces(rows, i, nobj, S, stride).clone() for i in range(n)]
    lost = (2, k)
    for i in lost:
        _pieces(rows, i, nobj, S, stride).fill_(0x3C)
    bad.fill_(7)
    enc.decode_dev(flat, [i not in lost for i in range(n)], S, pitch, stride, nobj, bad, s)
    torch.cuda.synchronize()
    assert not bad.any()
    for i in range(n):
        assert torch.equal(_pieces(rows, i, nobj, S, stride), golden[i]), i


@pytest.mark.parametrize("k,p,S,nobj", [(10, 2, 103, 1001), (16, 2, 1, 988), (10, 2, 5, 777), (4, 4, 17, 301)])
def test_shard_major_tight_pitch_last_object(gpu, k, p, S, nobj):
    """pitch = (nobj-1)*stride + S exactly: the last object's piece ends the
    row, its last 16-B vector would read past the batch; it is coded through
    the scratch copy (and the conversion to one object is not taken).  Pieces
    narrower than a vector (S = 1, 5): a piece's last vector may only be
    written up to the piece's end (obj_stride), never into the next object's
    piece or, at a row's end, into the next row (found by the soak)."""
    n = k + p
    stride = S
    pitch = (nobj - 1) * stride + S
    flat = torch.randint(0, 256, (n * pitch,), dtype=torch.uint8, device="cuda")
    rows = flat.view(n, pitch)
    enc = ia.New(k, p)
    s = torch.cuda.current_stream()
    before = rows.clone()
    enc.encode_dev(flat, S, pitch, stride, nobj, s)
    torch.cuda.synchronize()
    want = _expect_parity(enc, before, k, p, nobj, S, stride)
    for r in range(p):
        assert np.array_equal(rows[k + r].cpu().numpy(), want[r]), r


def test_shard_major_mixed_patterns_masks(gpu):
    """Device-resolved mixed patterns on a shard-major batch (16-B aligned
    pieces, as the masks calls require)."""
    k, p, S, nobj = 10, 2, 103, 4000
    n = k + p
    stride = 112
    pitch = nobj * stride
    flat, rows = _batch(k, p, S, nobj, stride, pitch, seed=5)
    enc = ia.New(k, p)
    s = torch.cuda.current_stream()
    enc.encode_dev(flat, S, pitch, stride, nobj, s)
    golden = rows.clone()
    rng = np.random.default_rng(3)
    present = np.ones((nobj, n), dtype=np.uint8)
    np.put_along_axis(present, np.argsort(rng.random((nobj, n)), axis=1)[:, :p], 0, axis=1)
    view = rows.view(n, nobj, stride)
    pm = torch.from_numpy(present.T.copy()).to("cuda").bool()
    view[..., :S][~pm] = 0x77
    masks = (present.astype(np.int64) << np.arange(n)).sum(axis=1).astype(np.int32)
    status = torch.full((nobj,), 9, dtype=torch.int32, device="cuda")
    enc.decode_dev_masks(flat, torch.from_numpy(masks).to("cuda"), S, pitch, stride, nobj, status, s)
    torch.cuda.synchronize()
    assert not status.any()
    assert torch.equal(view[..., :S], golden.view(n, nobj, stride)[..., :S])


@pytest.mark.parametrize("k,p,S,nobj,op", [(10, 2, 103, 900, "decode"), (10, 4, 100, 700, "reconstruct"),
                                           (10, 4, 60, 700, "data"), (6, 6, 30, 500, "decode"),
                                           (12, 4, 200, 300, "reconstruct"), (3, 1, 16, 2000, "decode"),
                                           (4, 2, 1, 3000, "decode")])
def test_shard_major_masks_vs_oracle(gpu, k, p, S, nobj, op):
    """Short rows of a shard-major batch through the lanes kernel (objects
    side by side in every shard row, each lane its own pattern): random per-object
    patterns with 0..p+1 lost (too few shards included), corrupted survivors
    and corrupted extra shards, each object against the oracle's
    Reconstruct / ReconstructData / fused decode."""
    n = k + p
    stride = (S + 15) // 16 * 16
    pitch = nobj * stride
    flat, rows = _batch(k, p, S, nobj, stride, pitch, seed=k * 100 + S)
    enc = ia.New(k, p)
    s = torch.cuda.current_stream()
    enc.encode_dev(flat, S, pitch, stride, nobj, s)
    torch.cuda.synchronize()
    rng = np.random.default_rng(S + nobj)
    present = np.ones((nobj, n), dtype=np.uint8)
    for o in range(nobj):
        nl = int(rng.integers(0, p + 2 if o % 9 == 4 else p + 1))
        present[o, rng.choice(n, nl, replace=False)] = 0
    view = rows.view(n, nobj, stride)
    pm = torch.from_numpy(present.T.copy()).to("cuda").bool()
    view[..., :S][~pm] = 0x77
    # corrupt one present byte of every 5th object (a survivor or an extra)
    for o in range(0, nobj, 5):
        i = int(rng.choice(np.flatnonzero(present[o])))
        view[i, o, int(rng.integers(0, S))] ^= 0x21
    h = view[..., :S].cpu().numpy()
    masks = (present.astype(np.int64) << np.arange(n)).sum(axis=1).astype(np.int32)
    status = torch.full((nobj,), 9, dtype=torch.int32, device="cuda")
    dm = torch.from_numpy(masks).to("cuda")
    if op == "decode":
        enc.decode_dev_masks(flat, dm, S, pitch, stride, nobj, status, s)
    else:
        enc.reconstruct_dev_masks(flat, dm, S, pitch, stride, nobj, data_only=op == "data", status=status, stream=s)
    torch.cuda.synchronize()
    got = view[..., :S].cpu().numpy()
    st = status.cpu().numpy()
    for o in range(nobj):
        shards = [h[i, o].copy() if present[o, i] else None for i in range(n)]
        if present[o].sum() < k:
            assert st[o] == 2, o
            assert np.array_equal(got[:, o], h[:, o]), o
            continue
        e, want = oracle.reconstruct(k, p, shards, data_only=op == "data")
        assert e == 0
        for i in range(n):
            if op == "data" and i >= k and not present[o, i]:  # ReconstructData leaves missing parity alone
                assert np.array_equal(got[i, o], h[i, o]), (o, i)
            else:
                assert np.array_equal(got[i, o], want[i]), (o, i)
        if op == "decode":  # Verify over the rebuilt object: any corrupted present shard shows
            e, okv = oracle.verify(k, p, [got[i, o] for i in range(n)])
            assert st[o] == (0 if okv else 1), (o, present[o])
        else:
            assert st[o] == 0, o


def _obj_major_golden(k, p, S, nobj, seed):
    """nobj objects' n rows (data random, parity from the oracle), (nobj, n, S)."""
    rng = np.random.default_rng(seed)
    data = rng.integers(0, 256, (nobj, k, S), dtype=np.uint8)
    m = ia.New(k, p).matrix()
    # coding is byte-position-wise: every object's row c back to back is one long row
    par = oracle.apply(m[k:], [np.ascontiguousarray(data[:, c, :]).reshape(-1) for c in range(k)])
    full = np.empty((nobj, k + p, S), np.uint8)
    full[:, :k] = data
    for r in range(p):
        full[:, k + r] = np.frombuffer(bytes(par[r]), np.uint8).reshape(nobj, S)
    return full


@pytest.mark.parametrize("k,p,S,nobj,src_align", [(10, 2, 103, 3000, 1), (10, 2, 103, 2000, 16), (10, 4, 410, 500, 16),
                                                  (6, 3, 1000, 64, 1), (10, 2, 17, 700, 1), (10, 2, 4099, 40, 256),
                                                  (12, 4, 128, 300, 128)])
def test_shardmajor_helper_get_batch_vs_oracle(gpu, k, p, S, nobj, src_align):
    """a Get batch arrives object-major (each object's
    bodies back to back, any pitch), rsgpu_copy_pieces moves it into the
    library's whole-line shard-major layout (rsgpu_shardmajor_layout), the
    per-object patterns are decoded there (*_dev_masks) and the rows come
    back object-major: bit-exact against the oracle, pad bytes of the
    destination untouched (every piece copy writes exactly shard_len bytes)."""
    n = k + p
    stride, pitch = ia.shardmajor_layout(S, nobj)
    assert stride % 16 == 0 and pitch % 256 == 0 and pitch >= nobj * stride >= nobj * S
    whole = (-S % 128) * 4 <= S
    assert (stride % 128 == 0) == whole or stride == (S + 15) // 16 * 16
    full = _obj_major_golden(k, p, S, nobj, seed=S * 7 + nobj)
    sp = (S + src_align - 1) // src_align * src_align
    src = torch.zeros((nobj, n, sp), dtype=torch.uint8, device="cuda")
    src[:, :, :S] = torch.from_numpy(full).to("cuda")
    sm = torch.full((n, pitch), 0x77, dtype=torch.uint8, device="cuda")
    enc = ia.New(k, p)
    s = torch.cuda.current_stream()
    enc.copy_pieces(src, sp, n * sp, sm, pitch, stride, S, nobj, stream=s)
    torch.cuda.synchronize()
    pieces = sm[:, :nobj * stride].view(n, nobj, stride)
    assert torch.equal(pieces[:, :, :S].permute(1, 0, 2).cpu(), torch.from_numpy(full))
    if stride > S:  # gaps untouched by the copy
        assert bool((pieces[:, :, S:] == 0x77).all())
    # per-object erasures (0..p lost, first-d rule on the survivors), lost pieces garbage
    rng = np.random.default_rng(nobj + S)
    present = np.ones((nobj, n), np.uint8)
    for o in range(nobj):
        present[o, rng.choice(n, int(rng.integers(0, p + 1)), replace=False)] = 0
    lost = torch.from_numpy(present == 0).to("cuda")  # (nobj, n)
    pv = pieces.permute(1, 0, 2)  # (nobj, n, stride) view
    pv[..., :S][lost] = 0xA5
    masks = (present.astype(np.int64) * (1 << np.arange(n, dtype=np.int64))).sum(axis=1).astype(np.uint32)
    dmask = torch.from_numpy(masks.view(np.int32)).to("cuda")
    status = torch.full((nobj,), 9, dtype=torch.int32, device="cuda")
    enc.decode_dev_masks(sm, dmask, S, pitch, stride, nobj, status, s)
    out = torch.zeros((nobj, n, sp), dtype=torch.uint8, device="cuda")
    if sp > S:
        out[:, :, S:] = 0x3C
    enc.copy_pieces(sm, pitch, stride, out, sp, n * sp, S, nobj, stream=s)
    torch.cuda.synchronize()
    assert int(status.abs().sum().item()) == 0, np.flatnonzero(status.cpu().numpy())[:5]
    assert np.array_equal(out[:, :, :S].cpu().numpy(), full)
    if sp > S:
        assert bool((out[:, :, S:] == 0x3C).all())


@pytest.mark.parametrize("S,nobj,rows", [(1, 1, (0,)), (103, 777, (1, 5, 11)), (4099, 33, (0, 11)),
                                         (17, 4000, tuple(range(12))), (1000, 3, (2, 3))])
def test_copy_pieces_exact_rows_both_ways(gpu, S, nobj, rows):
    """Only the listed rows' shard_len bytes move, at odd strides both ways
    (object-major byte-packed <-> shard-major at an unaligned stride)."""
    k, p = 10, 2
    n = k + p
    enc = ia.New(k, p)
    g = torch.Generator(device="cuda").manual_seed(S + nobj)
    src = torch.randint(0, 256, (nobj, n, S), dtype=torch.uint8, device="cuda", generator=g)  # byte-packed
    ds = S + 3  # unaligned stride
    dp = nobj * ds + 5
    dst = torch.full((n, dp), 0x11, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()
    enc.copy_pieces(src, S, n * S, dst, dp, ds, S, nobj, rows=rows, stream=s)
    back = torch.full((nobj, n, S + 1), 0x22, dtype=torch.uint8, device="cuda")
    enc.copy_pieces(dst, dp, ds, back, S + 1, n * (S + 1), S, nobj, rows=rows, stream=s)
    torch.cuda.synchronize()
    want = torch.full((n, dp), 0x11, dtype=torch.uint8)
    h = src.cpu()
    for i in rows:
        want[i, :nobj * ds].view(nobj, ds)[:, :S] = h[:, i]
    assert torch.equal(dst.cpu(), want)
    wb = torch.full((nobj, n, S + 1), 0x22, dtype=torch.uint8)
    for i in rows:
        wb[:, i, :S] = h[:, i]
    assert torch.equal(back.cpu(), wb)
