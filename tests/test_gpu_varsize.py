"""Variable-size device batches (rsgpu_*_dev_objs): objects of 1 B to
100 MiB, each with its own pitch, coded in ONE launch per pass, against the
oracle (bit-exact).  Config 5's objects range from 4 KiB to 100 MiB
(client/ecRedis.go:96 Set buffer of any length); before this call a batch of
mixed sizes took one launch per object."""
import numpy as np
import pytest

import infinicache_amd as ia
import oracle
from oracle import rs_numpy as rn

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

K, P = 10, 2
N = K + P


def _layout(nbytes_list, rng, align=16):
    """object-major objects back to back in one device buffer, each with its
    own pitch >= roundup16(S) and a random gap after it"""
    objs, off = [], 0
    for nb in nbytes_list:
        S = (nb + K - 1) // K
        pitch = (S + 15) // 16 * 16 + int(rng.integers(0, 4)) * align
        objs.append((off, S, pitch))
        off += N * pitch + int(rng.integers(0, 3)) * 64
    return objs, off + 256


def _fill(total, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    return torch.randint(0, 256, (total,), dtype=torch.uint8, device="cuda", generator=g)


def _rows(h, off, S, pitch):
    return [h[off + i * pitch: off + i * pitch + S] for i in range(N)]


SIZES = [1, 15, 16, 17, 160, 1024, 4096, 4097, 65536, 77777, 1 << 20, (4 << 20) + 3, 100 << 20]


def test_encode_decode_objs_1B_to_100MiB_one_launch(gpu):
    rng = np.random.default_rng(5)
    enc = ia.New(K, P)
    m = enc.matrix()
    layout, total = _layout(SIZES, rng)
    buf = _fill(total, 11)
    base = buf.data_ptr()
    objs = [(base + off, S, pitch) for off, S, pitch in layout]
    s = torch.cuda.current_stream()
    enc.encode_dev_objs(objs, s)
    torch.cuda.synchronize()
    h = buf.cpu().numpy()
    for off, S, pitch in layout:
        rows = _rows(h, off, S, pitch)
        want = oracle.code_fast(m[K:], rows[:K], nthreads=16)
        for r in range(P):
            assert np.array_equal(rows[K + r], want[r]), (S, r)
    golden = buf.clone()
    # a Get that lost data shards 0 and 5: one fused-decode launch for all sizes
    lost = (0, 5)
    for off, S, pitch in layout:
        for i in lost:
            buf[off + i * pitch: off + i * pitch + S] = 0xC3
    bad = torch.full((len(objs),), 5, dtype=torch.int32, device="cuda")
    enc.decode_dev_objs(objs, [i not in lost for i in range(N)], bad, s)
    torch.cuda.synchronize()
    assert not bad.any()
    h2 = buf.cpu().numpy()
    hg = golden.cpu().numpy()
    for off, S, pitch in layout:
        for i in range(N):
            assert np.array_equal(h2[off + i * pitch: off + i * pitch + S], hg[off + i * pitch: off + i * pitch + S]), (S, i)


def test_objs_checks_verify_and_data_only(gpu):
    """Extra present parity shards are checked per object (the flag lands at
    the object's own index), Verify flags per object, ReconstructData leaves
    missing parity alone."""
    rng = np.random.default_rng(9)
    enc = ia.New(K, P)
    sizes = [33, 5000, 104858, 9, 1 << 16, 250001, 7]
    layout, total = _layout(sizes, rng)
    buf = _fill(total, 12)
    objs = [(buf.data_ptr() + off, S, pitch) for off, S, pitch in layout]
    s = torch.cuda.current_stream()
    enc.encode_dev_objs(objs, s)
    golden = buf.clone()
    bad = torch.full((len(objs),), 5, dtype=torch.int32, device="cuda")
    enc.verify_dev_objs(objs, bad, s)
    torch.cuda.synchronize()
    assert not bad.any()
    corrupt = {1, 5}
    for o in corrupt:  # the last parity row's last byte
        off, S, pitch = layout[o]
        buf[off + 11 * pitch + S - 1] ^= 0x40
    enc.verify_dev_objs(objs, bad, s)
    torch.cuda.synchronize()
    assert [int(x) for x in bad.cpu()] == [1 if o in corrupt else 0 for o in range(len(objs))]
    # lose data shard 3 only: 11 present, shard 11 is an extra the decode checks
    for off, S, pitch in layout:
        buf[off + 3 * pitch: off + 3 * pitch + S] = 0
    enc.decode_dev_objs(objs, [i != 3 for i in range(N)], bad, s)
    torch.cuda.synchronize()
    assert [int(x) for x in bad.cpu()] == [1 if o in corrupt else 0 for o in range(len(objs))]
    h, hg = buf.cpu().numpy(), golden.cpu().numpy()
    for off, S, pitch in layout:  # the rebuilt row is right whatever the extra shard says
        assert np.array_equal(h[off + 3 * pitch: off + 3 * pitch + S], hg[off + 3 * pitch: off + 3 * pitch + S])
    # ReconstructData: data 0 and parity 10 missing -> only row 0 written
    buf.copy_(golden)
    for off, S, pitch in layout:
        buf[off: off + S] = 0
        buf[off + 10 * pitch: off + 10 * pitch + S] = 0x11
    enc.reconstruct_dev_objs(objs, [i not in (0, 10) for i in range(N)], data_only=True, stream=s)
    torch.cuda.synchronize()
    h = buf.cpu().numpy()
    for off, S, pitch in layout:
        assert np.array_equal(h[off: off + S], hg[off: off + S])
        assert (h[off + 10 * pitch: off + 10 * pitch + S] == 0x11).all()


@pytest.mark.parametrize("k,p", [(4, 6), (20, 4), (16, 16)])
def test_objs_other_codes(gpu, k, p):
    """p > 4 rows (two sub-passes) and K > 16 (the generic kernel, object by
    object) behind the same call."""
    n = k + p
    rng = np.random.default_rng(k + p)
    enc = ia.New(k, p)
    m = enc.matrix()
    objs, off = [], 0
    for nb in [100, 70000, 3, 1 << 18]:
        S = (nb + k - 1) // k
        pitch = (S + 15) // 16 * 16
        objs.append((off, S, pitch))
        off += n * pitch
    buf = _fill(off + 64, k * 100 + p)
    t = [(buf.data_ptr() + o, S, pitch) for o, S, pitch in objs]
    s = torch.cuda.current_stream()
    enc.encode_dev_objs(t, s)
    torch.cuda.synchronize()
    h = buf.cpu().numpy()
    for o, S, pitch in objs:
        rows = [h[o + i * pitch: o + i * pitch + S] for i in range(n)]
        want = oracle.apply(m[k:], rows[:k])
        for r in range(p):
            assert np.array_equal(rows[k + r], want[r])
    golden = buf.clone()
    lost = sorted(rng.choice(n, p, replace=False).tolist())
    for o, S, pitch in objs:
        for i in lost:
            buf[o + i * pitch: o + i * pitch + S] = 0x77
    bad = torch.full((len(objs),), 5, dtype=torch.int32, device="cuda")
    enc.decode_dev_objs(t, [i not in lost for i in range(n)], bad, s)
    torch.cuda.synchronize()
    assert not bad.any()
    h, hg = buf.cpu().numpy(), golden.cpu().numpy()
    for o, S, pitch in objs:
        for i in range(n):
            assert np.array_equal(h[o + i * pitch: o + i * pitch + S], hg[o + i * pitch: o + i * pitch + S])
