"""Device-resolved mixed erasure patterns (rsgpu_{decode,reconstruct}_dev_masks)
against the CPU oracle, bit-exact.

A Get batch gives every object its own erasure pattern (the proxy's first-d
rule, /root/reference/proxy/lambdastore/connection.go:274-306), decoded as
Client.decode does (client/ecRedis.go:404-427).  Here the arrival bitmaps are
device-resident; the kernels resolve pattern -> coefficients on the device
(gf_masked.h).  Covered: both kernels (short rows packed several objects per
workgroup, long rows one object per workgroup chunk), every status value
(ok / Verify mismatch / too few shards / singular), extra present shards
that are really checked, codes needing two sub-passes (p > 4), repeated calls
on one context (the status scratch resets itself), ignored high mask bits and
the host-flag *_dev_multi calls now routed through the same kernels."""
import itertools

import numpy as np
import pytest

import infinicache_amd as ia
import oracle
from oracle import rs_numpy as rn

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def _batch(nobj, n, S, pitch, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    b = torch.randint(0, 256, (nobj, n, pitch), dtype=torch.uint8, device="cuda", generator=g)
    b[:, :, S:] = 0
    return b


def _pitch(S):
    return (S + 255) // 256 * 256 if S >= 4096 else (S + 15) // 16 * 16


def _masks_of(present):
    w = (1 << np.arange(present.shape[1], dtype=np.int64))
    return (present.astype(np.int64) * w).sum(axis=1).astype(np.uint32)


def _dev_u32(a):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.int32)).to("cuda")


def _random_patterns(rng, nobj, k, p, corrupt_every=7, too_few_every=0):
    """present flags per object: 0..p lost (fewer than p leaves extra shards,
    which the fused decode really checks), occasionally too few."""
    n = k + p
    present = np.ones((nobj, n), dtype=np.uint8)
    for o in range(nobj):
        nl = int(rng.integers(0, p + 1))
        if too_few_every and o % too_few_every == 3:
            nl = p + 1
        present[o, rng.choice(n, nl, replace=False)] = 0
    return present


@pytest.mark.parametrize("k,p,S,nobj", [(10, 2, 104858, 40), (10, 2, 50001, 300), (10, 4, 7777, 120),
                                        (10, 2, 103, 2000), (10, 4, 410, 700), (12, 4, 2048, 90),
                                        (4, 2, 1, 300), (10, 2, 2049, 33), (6, 6, 3000, 64),
                                        (8, 8, 100, 257), (1, 1, 17, 40), (15, 1, 4096, 20),
                                        # no device atlas: 17-32 shards, or RS(2+14) past the atlas
                                        # bound (masks read back, host-planned launches)
                                        (20, 4, 3000, 50), (17, 3, 500, 100), (24, 8, 1000, 40),
                                        (2, 14, 200, 64), (28, 4, 700, 30)])
def test_decode_masks_random_patterns(gpu, k, p, S, nobj):
    n = k + p
    pitch = _pitch(S)
    stride = n * pitch
    rng = np.random.default_rng(k * 1000 + p * 10 + S % 7)
    b = _batch(nobj, n, S, pitch, seed=S + nobj)
    enc = ia.New(k, p)
    s = torch.cuda.current_stream()
    enc.encode_dev(b, S, pitch, stride, nobj, s)
    golden = b.clone()
    present = _random_patterns(rng, nobj, k, p, too_few_every=11)
    corrupt, too_few = set(), set()
    for o in range(nobj):
        lost = np.flatnonzero(present[o] == 0)
        if len(lost):
            b[o, torch.as_tensor(lost, dtype=torch.long)] = 0xA5
        if present[o].sum() < k:
            too_few.add(o)
            continue
        nl = len(lost)
        if nl < p and o % 7 == 0:  # an extra present shard exists: corrupt the last present row
            last = int(np.nonzero(present[o])[0][-1])
            if last >= k:  # upstream Verify checks parity rows only
                b[o, last, min(3, S - 1)] ^= 1
                corrupt.add(o)
    before = b.clone()
    masks = _masks_of(present)
    masks[1::5] |= np.uint32(0xFFFF0000) & ~np.uint32((1 << n) - 1)  # high bits are ignored
    status = torch.full((nobj,), 9, dtype=torch.int32, device="cuda")
    enc.decode_dev_masks(b, _dev_u32(masks), S, pitch, stride, nobj, status, s)
    torch.cuda.synchronize()
    st = status.cpu().numpy()
    for o in range(nobj):
        if o in too_few:
            assert st[o] == 2, o
            assert torch.equal(b[o], before[o]), o  # untouched
            continue
        assert st[o] == (1 if o in corrupt else 0), (o, present[o], st[o])
        if o not in corrupt:
            assert torch.equal(b[o, :, :S], golden[o, :, :S]), (o, present[o])
        else:  # survivors are untouched, rebuilt rows are exact; only the corrupted byte differs
            want = golden[o, :, :S].clone()
            last = int(np.nonzero(present[o])[0][-1])
            want[last, min(3, S - 1)] ^= 1
            assert torch.equal(b[o, :, :S], want), o
    # a second call on the same context (the multi-reporter scratch reset
    # itself): restore and decode again, flags identical
    b.copy_(before)
    status.fill_(7)
    enc.decode_dev_masks(b, _dev_u32(masks), S, pitch, stride, nobj, status, s)
    torch.cuda.synchronize()
    assert np.array_equal(status.cpu().numpy(), st)


@pytest.mark.parametrize("k,p,S,nobj,data_only", [(10, 4, 9000, 64, True), (10, 4, 9000, 64, False),
                                                  (10, 4, 300, 500, True), (10, 2, 1000, 300, False),
                                                  (6, 6, 5000, 50, False), (6, 6, 60, 400, True),
                                                  (20, 4, 2000, 60, True), (20, 4, 2000, 60, False),
                                                  (4, 12, 500, 80, False)])
def test_reconstruct_masks(gpu, k, p, S, nobj, data_only):
    n = k + p
    pitch = _pitch(S)
    stride = n * pitch
    b = _batch(nobj, n, S, pitch, seed=11 + S)
    enc = ia.New(k, p)
    s = torch.cuda.current_stream()
    enc.encode_dev(b, S, pitch, stride, nobj, s)
    golden = b.clone()
    present = np.ones((nobj, n), dtype=np.uint8)
    pats = [c for e in range(p + 1) for c in itertools.combinations(range(n), e)]
    for o in range(nobj):
        lost = pats[(o * 37) % len(pats)]
        present[o, list(lost)] = 0
        for i in lost:
            b[o, i] = 0
    status = torch.full((nobj,), 5, dtype=torch.int32, device="cuda")
    enc.reconstruct_dev_masks(b, _dev_u32(_masks_of(present)), S, pitch, stride, nobj, data_only=data_only,
                              status=status, stream=s)
    torch.cuda.synchronize()
    assert not status.any()
    for o in range(nobj):
        assert torch.equal(b[o, :k, :S], golden[o, :k, :S]), o
        for i in range(k, n):
            if present[o, i]:
                assert torch.equal(b[o, i, :S], golden[o, i, :S])
            elif data_only:  # missing parity untouched
                assert not b[o, i].any()
            else:
                assert torch.equal(b[o, i, :S], golden[o, i, :S]), (o, i)


def test_reconstruct_masks_vs_oracle_corrupt_survivors(gpu):
    """Survivor choice mirrors upstream (first k present in index order), so
    even on corrupted input the rebuilt rows match the oracle byte for byte."""
    k, p, S, nobj = 10, 4, 333, 48
    n = k + p
    pitch = _pitch(S)
    b = _batch(nobj, n, S, pitch, seed=77)
    enc = ia.New(k, p)
    s = torch.cuda.current_stream()
    enc.encode_dev(b, S, pitch, n * pitch, nobj, s)
    rng = np.random.default_rng(5)
    present = _random_patterns(rng, nobj, k, p)
    present[:, 0] = np.where(np.arange(nobj) % 3 == 0, 0, present[:, 0])
    present[present.sum(1) < k, :] = 1
    for o in range(nobj):  # corrupt a survivor byte
        first = int(np.nonzero(present[o])[0][0])
        b[o, first, o % S] ^= 0x3C
    h = b.cpu().numpy()
    enc.reconstruct_dev_masks(b, _dev_u32(_masks_of(present)), S, pitch, n * pitch, nobj, stream=s)
    torch.cuda.synchronize()
    got = b.cpu().numpy()
    for o in range(nobj):
        shards = [h[o, i, :S].copy() if present[o, i] else None for i in range(n)]
        e, want = oracle.reconstruct(k, p, shards)
        assert e == 0
        for i in range(n):
            assert np.array_equal(got[o, i, :S], want[i]), (o, i)


def test_masks_singular_pattern_par1(gpu):
    """PAR1 is not MDS: a pattern whose survivors' matrix is singular gets
    status 3 (upstream errSingular) and is left untouched; the host-flag
    call returns the error before any launch."""
    k, p = 4, 4
    n = k + p
    m = ia.New(k, p, matrix="par1").matrix()
    sing = None
    for lost in itertools.combinations(range(n), p):
        surv = [i for i in range(n) if i not in lost][:k]
        try:
            rn.invert(m[surv])
        except Exception:
            sing = lost
            break
    if sing is None:
        pytest.skip("no singular PAR1 pattern for this shape")  # pragma: no cover
    S, nobj = 64, 6
    pitch = _pitch(S)
    b = _batch(nobj, n, S, pitch, seed=3)
    enc = ia.New(k, p, matrix="par1")
    s = torch.cuda.current_stream()
    enc.encode_dev(b, S, pitch, n * pitch, nobj, s)
    golden = b.clone()
    present = np.ones((nobj, n), dtype=np.uint8)
    present[2, list(sing)] = 0
    present[4, [0]] = 0
    b[4, 0] = 0
    before = b.clone()
    status = torch.full((nobj,), 9, dtype=torch.int32, device="cuda")
    enc.decode_dev_masks(b, _dev_u32(_masks_of(present)), S, pitch, n * pitch, nobj, status, s)
    torch.cuda.synchronize()
    assert status.cpu().tolist() == [0, 0, 3, 0, 0, 0]
    assert torch.equal(b[2], before[2])
    assert torch.equal(b[4, :, :S], golden[4, :, :S])
    with pytest.raises(ia.ErrSingular):
        enc.decode_dev_multi(b, present, S, pitch, n * pitch, nobj, status, s)


def test_masks_large_batch_lanes_grid(gpu):
    """300,000 x 1 KiB RS(10+2) objects (S = 103, 36 per workgroup), each
    with a random lost pair: a checksum of checksums against the oracle's
    batch coder, plus a sample compared byte for byte."""
    k, p, S, nobj = 10, 2, 103, 300_000
    n = k + p
    pitch = 112
    stride = n * pitch
    b = _batch(nobj, n, S, pitch, seed=21)
    enc = ia.New(k, p)
    s = torch.cuda.current_stream()
    enc.encode_dev(b, S, pitch, stride, nobj, s)
    golden = b.clone()
    rng = np.random.default_rng(8)
    keys = rng.random((nobj, n))
    present = np.ones((nobj, n), dtype=np.uint8)
    np.put_along_axis(present, np.argsort(keys, axis=1)[:, :p], 0, axis=1)
    pm = torch.from_numpy(present).to("cuda").bool()
    b[~pm] = 0x5A
    status = torch.full((nobj,), 9, dtype=torch.int32, device="cuda")
    enc.decode_dev_masks(b, _dev_u32(_masks_of(present)), S, pitch, stride, nobj, status, s)
    torch.cuda.synchronize()
    assert not status.any()
    assert torch.equal(b[:, :, :S], golden[:, :, :S])


def test_host_flags_route_through_masks(gpu):
    """decode_dev_multi with host flags (n <= 16) packs masks and uses the
    same kernels; too-few shards is still a synchronous ErrTooFewShards."""
    k, p, S, nobj = 10, 2, 4000, 50
    n = k + p
    pitch = _pitch(S)
    b = _batch(nobj, n, S, pitch, seed=5)
    enc = ia.New(k, p)
    s = torch.cuda.current_stream()
    enc.encode_dev(b, S, pitch, n * pitch, nobj, s)
    golden = b.clone()
    present = np.ones((nobj, n), dtype=np.uint8)
    for o in range(nobj):
        present[o, [o % n, (o * 5 + 1) % n]] = 0
        b[o, o % n] = 0
        b[o, (o * 5 + 1) % n] = 0
    bad = torch.full((nobj,), 4, dtype=torch.int32, device="cuda")
    for _ in range(6):  # more calls than the upload ring has slots
        enc.decode_dev_multi(b, present, S, pitch, n * pitch, nobj, bad, s)
    torch.cuda.synchronize()
    assert not bad.any()
    assert torch.equal(b[:, :, :S], golden[:, :, :S])
    present[7, :3] = 0
    with pytest.raises(ia.ErrTooFewShards):
        enc.decode_dev_multi(b, present, S, pitch, n * pitch, nobj, bad, s)


@pytest.mark.parametrize("k,p", [(2, 14), (4, 12), (8, 8)])
def test_host_flags_large_atlas_codes(gpu, k, p):
    """n = 16 codes whose pattern atlas would be large (RS(2+14), RS(4+12):
    ~65k patterns; RS(8+8): ~40k) keep the host-planned path for the host-flag
    calls (they used to return ErrNotImplemented or build the
    whole atlas on the first call).  Every object its own pattern, against
    the encode's golden rows, plus ReconstructData."""
    n = k + p
    S, nobj = 1000, 60
    pitch = _pitch(S)
    rng = np.random.default_rng(k * 31 + p)
    b = _batch(nobj, n, S, pitch, seed=k + 100 * p)
    enc = ia.New(k, p)
    s = torch.cuda.current_stream()
    enc.encode_dev(b, S, pitch, n * pitch, nobj, s)
    golden = b.clone()
    present = np.ones((nobj, n), dtype=np.uint8)
    for o in range(nobj):
        present[o, rng.choice(n, int(rng.integers(1, p + 1)), replace=False)] = 0
        b[o, torch.as_tensor(np.flatnonzero(present[o] == 0), dtype=torch.long)] = 0x3C
    bad = torch.full((nobj,), 4, dtype=torch.int32, device="cuda")
    enc.decode_dev_multi(b, present, S, pitch, n * pitch, nobj, bad, s)
    torch.cuda.synchronize()
    assert not bad.any()
    assert torch.equal(b[:, :, :S], golden[:, :, :S])
    for o in range(nobj):
        b[o, torch.as_tensor(np.flatnonzero(present[o] == 0), dtype=torch.long)] = 0x3C
    enc.reconstruct_dev_multi(b, present, S, pitch, n * pitch, nobj, data_only=True, stream=s)
    torch.cuda.synchronize()
    for o in range(nobj):
        assert torch.equal(b[o, :k, :S], golden[o, :k, :S]), o


def test_masks_code_beyond_mask_width_not_implemented(gpu):
    """Masks are 32-bit words: codes of more than 32 shards return
    ErrNotImplemented (the host-flag *_dev_multi calls cover them)."""
    enc = ia.New(30, 4)
    b = torch.zeros((2, 34, 256), dtype=torch.uint8, device="cuda")
    m = torch.zeros(2, dtype=torch.int32, device="cuda")
    st = torch.zeros(2, dtype=torch.int32, device="cuda")
    with pytest.raises(ia.ErrNotImplemented):
        enc.decode_dev_masks(b, m, 200, 256, 34 * 256, 2, st, torch.cuda.current_stream())
