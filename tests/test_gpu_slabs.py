"""Objects of any size through the host API: column slabs (rsgpu.cpp run_host).

Upstream's reedsolomon.Encoder codes shards of any length.  A pass addresses
its staged image with 32-bit offsets, so the per-object host calls code an
object whose staged image passes the slab size (1 GiB; rsgpu_set_slab_bytes / RSGPU_SLAB_BYTES
overrides it) as consecutive column slabs of every row, and the batch
pipelines hand such objects to that path.  Every operation is a byte-column
map, so the result must equal the unslabbed oracle's bit for bit; check
flags are OR-ed over the slabs.

Small objects with the slab size set to 64 KiB (rsgpu_set_slab_bytes) exercise every operation with
several slabs (incl. a ragged last one) against the oracle; one RS(10+2)
object of 12 x 360 MiB (a 4.2 GB Split image, past what one pass addresses)
runs at the default slab size, checked on column windows around every slab
boundary (the coding is column-wise, so windows are exact checks)."""
import os

import numpy as np
import pytest

import infinicache_amd as ia
import oracle
from oracle import rs_numpy as rn

pytestmark = pytest.mark.gpu
SEED = 0x51AB


@pytest.fixture
def small_slabs():
    # the library reads the slab size once; tests set it through the C ABI
    ia.set_slab_bytes(64 << 10)
    try:
        yield 64 << 10
    finally:
        ia.set_slab_bytes(0)


def _full(k, p, size, idx):
    d = rn.splitmix64_bytes(SEED, idx, k * size).reshape(k, size)
    e, sh = oracle.encode(k, p, [d[i] for i in range(k)] + [bytes(size)] * p)
    assert e == 0
    return sh


@pytest.mark.parametrize("k,p,size", [(10, 2, 10000), (10, 4, 20001), (4, 2, 40000)])
def test_every_host_op_in_slabs(gpu, small_slabs, k, p, size):
    n = k + p
    assert n * size + 16 > small_slabs  # several slabs per object
    full = _full(k, p, size, idx=size)
    enc = ia.New(k, p)
    # Encode / Verify / EncodeVerify
    sh = [full[i].copy() for i in range(k)] + [np.zeros(size, np.uint8) for _ in range(p)]
    enc.Encode(sh)
    assert all(np.array_equal(sh[i], full[i]) for i in range(n))
    assert enc.Verify(sh)
    for pos in (0, 4096, size - 1):  # a mismatch in the first, second and last slab
        bad = [s.copy() for s in sh]
        bad[n - 1][pos] ^= 0x11
        assert not enc.Verify(bad), pos
    sh2 = [full[i].copy() for i in range(k)] + [np.full(size, 7, np.uint8) for _ in range(p)]
    assert enc.EncodeVerify(sh2)
    assert all(np.array_equal(sh2[i], full[i]) for i in range(n))
    # Reconstruct / ReconstructData / DecodeVerify
    lost = (0, k - 1) if p == 2 else (1, 5, k, n - 1)
    got = [None if i in lost else full[i].copy() for i in range(n)]
    enc.Reconstruct(got)
    assert all(np.array_equal(got[i], full[i]) for i in range(n))
    got = [None if i in lost else full[i].copy() for i in range(n)]
    enc.ReconstructData(got)
    assert all(np.array_equal(got[i], full[i]) for i in range(k))
    got = [None if i == 2 else full[i].copy() for i in range(n)]
    assert enc.DecodeVerify(got) and np.array_equal(got[2], full[2])
    got = [None if i == 2 else full[i].copy() for i in range(n)]
    got[n - 1][size - 3] ^= 1  # an extra shard wrong in the last slab only
    assert not enc.DecodeVerify(got)
    # Update
    rng = np.random.default_rng(size)
    new = [None] * k
    for c in (0, k - 1):
        new[c] = rng.integers(0, 256, size, dtype=np.uint8)
    e, want = oracle.update(k, p, full, new)
    assert e == 0
    up = [s.copy() for s in full]
    enc.Update(up, new)
    assert all(np.array_equal(up[i], want[i]) for i in range(n))


def test_pinned_split_image_in_slabs(gpu, small_slabs):
    k, p, size = 10, 2, 9000
    n = k + p
    full = _full(k, p, size, idx=3)
    enc = ia.New(k, p)
    buf = ia.host_alloc(n * size)
    sh = [buf[i * size:(i + 1) * size] for i in range(n)]
    for i in range(n):
        sh[i][:] = full[i] if i < k else 0
    enc.Encode(sh)
    assert all(np.array_equal(sh[i], full[i]) for i in range(n))
    got = [None if i in (3, 11) else sh[i] for i in range(n)]
    enc.Reconstruct(got)
    assert all(np.array_equal(got[i], full[i]) for i in range(n))


def test_batches_hand_big_objects_to_slabs(gpu, small_slabs):
    """encode_batch / decode_batch: objects past the slab size take the
    per-object path, the others the pipeline, in one call."""
    k, p = 10, 2
    n = k + p
    sizes = [100, 9000, 300, 20000, 5]
    fulls = [_full(k, p, s, idx=50 + j) for j, s in enumerate(sizes)]
    enc = ia.New(k, p)
    objs = [np.concatenate([f[i] if i < k else np.zeros(len(f[0]), np.uint8) for i in range(n)]) for f in fulls]
    enc.encode_batch(objs)
    for o, f in zip(objs, fulls):
        assert np.array_equal(o, np.concatenate(f))
    gets, pres = [], []
    for j, f in enumerate(fulls):
        lost = {j % n} if j == 3 else {j % n, (j + 4) % n}  # object 3: 11 present, one extra check
        gets.append([np.zeros(len(f[0]), np.uint8) if i in lost else f[i].copy() for i in range(n)])
        pres.append([i not in lost for i in range(n)])
    gets[3][11][17] ^= 1  # object 3 (slabbed): an extra shard is wrong -> its flag fails
    ok = enc.decode_batch(gets, pres)
    assert ok == [True, True, True, False, True]
    for j, (g, f) in enumerate(zip(gets, fulls)):
        for i in range(k):
            assert np.array_equal(g[i], f[i]), (j, i)


def test_object_past_4gib_image(gpu):
    """One RS(10+2) object whose Split image is 12 x 360 MiB (4.2 GB): past
    the 4 GiB one pass addresses, coded at the default slab size (1 GiB
    staged per slab, 4 slabs).  Checked on column windows around every slab
    boundary and both ends, against the oracle on the same columns."""
    if os.environ.get("RSGPU_SLAB_BYTES"):
        pytest.skip("needs the default slab size")
    k, p = 10, 2
    n = k + p
    S = 360 << 20
    img = ia.host_alloc(n * S)
    rows = [img[i * S:(i + 1) * S] for i in range(n)]
    rng = np.random.default_rng(11)
    blk = rng.integers(0, 256, 1 << 20, dtype=np.uint8)
    for i in range(k):  # data rows: one random MiB rolled per (row, MiB)
        r = rows[i].reshape(-1, 1 << 20)
        for j in range(r.shape[0]):
            r[j] = np.roll(blk, 7919 * i + 104729 * j)
    for i in range(k, n):
        rows[i][:] = 0
    enc = ia.New(k, p)
    assert enc.EncodeVerify(rows)
    L = ((1 << 30) - 16) // n // 4096 * 4096  # run_host's slab length at the default size
    wins = sorted({0, S - 8192} | {b - 4096 for b in range(L, S, L)})
    for w0 in wins:
        cols = slice(w0, w0 + 8192)
        e, want = oracle.encode(k, p, [rows[i][cols].copy() for i in range(k)] + [bytes(8192)] * p)
        assert e == 0
        for i in range(k, n):
            assert np.array_equal(rows[i][cols], want[i]), (w0, i)
    # Get with data rows 0 and 5 lost: rebuilt in place, checked on the windows
    keep = {i: [rows[i][w0:w0 + 8192].copy() for w0 in wins] for i in (0, 5)}
    rows[0][:] = 0
    rows[5][:] = 0xEE
    ok = enc.decode_batch([rows], [[i not in (0, 5) for i in range(n)]])
    assert ok == [True]
    for i in (0, 5):
        for w0, want in zip(wins, keep[i]):
            assert np.array_equal(rows[i][w0:w0 + 8192], want), (i, w0)


def test_device_objects_past_4gib_rows(gpu):
    """Device-resident objects whose rows span more than 4 GiB (the 32-bit
    offsets one pass addresses): rsgpu_{encode,verify,reconstruct,decode}_dev
    code them in column slabs through a scratch image (launch_huge).  Two
    RS(10+2) objects of 12 x 360 MiB rows (9 GB of HBM); parity, flags and
    rebuilt rows checked against the oracle on column windows around every
    slab boundary."""
    torch = pytest.importorskip("torch")
    k, p = 10, 2
    n = k + p
    S = 360 << 20
    pitch = S + 256
    nobj = 2
    stride = n * pitch
    buf = torch.empty(nobj * stride, dtype=torch.uint8, device="cuda")
    g = torch.Generator(device="cuda").manual_seed(77)
    v = buf.view(nobj, n, pitch)
    v[:, :k, :S] = torch.randint(0, 256, (nobj, k, S), dtype=torch.uint8, device="cuda", generator=g)
    enc = ia.New(k, p)
    enc.encode_dev(buf, S, pitch, stride, nobj)
    torch.cuda.synchronize()
    slab = ((1 << 30) // n) // 4096 * 4096  # launch_huge's slab at 12 rows
    wins = sorted({0, S - 8192} | {b - 4096 for b in range(slab, S, slab)})
    host = {}
    for o in range(nobj):
        for w0 in wins:
            rows = v[o, :, w0:w0 + 8192].cpu().numpy()
            e, want = oracle.encode(k, p, [rows[i].copy() for i in range(k)] + [bytes(8192)] * p)
            assert e == 0
            for i in range(k, n):
                assert np.array_equal(rows[i], want[i]), (o, w0, i)
            host[o, w0] = rows
    bad = torch.full((nobj,), 7, dtype=torch.int32, device="cuda")
    enc.verify_dev(buf, S, pitch, stride, nobj, bad)
    torch.cuda.synchronize()
    assert bad.tolist() == [0, 0]
    v[1, n - 1, wins[-2]] ^= 1  # object 1: one parity byte wrong, in a far slab
    enc.verify_dev(buf, S, pitch, stride, nobj, bad)
    torch.cuda.synchronize()
    assert bad.tolist() == [0, 1]
    v[1, n - 1, wins[-2]] ^= 1
    # a Get with data rows 0 and 5 lost: rebuilt in place (fused decode)
    v[:, 0, :S] = 0
    v[:, 5, :S] = 0xEE
    present = [i not in (0, 5) for i in range(n)]
    bad.fill_(7)
    enc.decode_dev(buf, present, S, pitch, stride, nobj, bad)
    torch.cuda.synchronize()
    assert bad.tolist() == [0, 0]
    for o in range(nobj):
        for w0 in wins:
            got = v[o, :, w0:w0 + 8192].cpu().numpy()
            assert np.array_equal(got[0], host[o, w0][0]) and np.array_equal(got[5], host[o, w0][5]), (o, w0)
    del buf
    torch.cuda.empty_cache()
