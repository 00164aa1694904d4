"""The input-triples kernel (gf_kernels.hip gf_apply_tri) on every shape it
serves, through the C ABI's device-batch calls, against the oracle: rows of
more than 128 16-B vectors (the kernel's range), ragged tails, a row pitch
that is not a multiple of 16 (packed last-vector stores, and the batch's last
object through launch_plan's scratch copy), and check flags per object.

Shapes (K inputs, R rows, KI identity inputs):
  * (10, 4, 0)  RS(10+4) Encode;
  * (14, 4, 4)  RS(10+4) Verify, (13, 3, 3) RS(10+3) Verify, (16, 4, 4)
    RS(12+4) Verify;
  * (12, 4, 2)  RS(10+4) Get with 2 data shards lost (Client.decode,
    client/ecRedis.go:404-427: 2 rows rebuilt, 2 extra shards checked);
  * (11, 4, 1)  RS(10+4) Get with 3 data shards lost (1 extra shard)."""
import numpy as np
import pytest

import infinicache_amd as ia
import oracle

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def _batch(k, p, nobj, S, pitch, seed):
    n = k + p
    g = torch.Generator(device="cuda").manual_seed(seed)
    b = torch.randint(0, 256, (nobj, n, pitch), dtype=torch.uint8, device="cuda", generator=g)
    b[:, :, S:] = 0
    return b


def _oracle_parity(m, k, p, h, S):
    n = k + p
    want = h.copy()
    for o in range(h.shape[0]):
        par = oracle.apply(m[k:], [h[o, c, :S] for c in range(k)])
        for r in range(p):
            want[o, k + r, :S] = par[r]
    return want


@pytest.mark.parametrize("S,pitch", [(70001, 70144), (4099, 4100), (419431, 419584)])
def test_tri_encode_verify_rs10_4(gpu, S, pitch):
    k, p, nobj = 10, 4, 3
    n = k + p
    enc = ia.New(k, p)
    st = torch.cuda.current_stream()
    b = _batch(k, p, nobj, S, pitch, seed=S)
    enc.encode_dev(b, S, pitch, n * pitch, nobj, st)
    torch.cuda.synchronize()
    h = b.cpu().numpy()
    want = _oracle_parity(enc.matrix(), k, p, h, S)
    assert np.array_equal(h[:, :, :S], want[:, :, :S])
    if pitch > S:  # bytes between rows untouched
        assert not h[:, :, S:].any()
    bad = torch.full((nobj,), 9, dtype=torch.int32, device="cuda")
    enc.verify_dev(b, S, pitch, n * pitch, nobj, bad, st)
    torch.cuda.synchronize()
    assert bad.tolist() == [0] * nobj
    b[0, 3, S - 1] ^= 0x01        # data row, last byte
    b[2, 13, 0] ^= 0x80           # parity row, first byte
    enc.verify_dev(b, S, pitch, n * pitch, nobj, bad, st)
    torch.cuda.synchronize()
    assert bad.tolist() == [1, 0, 1]


@pytest.mark.parametrize("k,p", [(10, 3), (12, 4)])
def test_tri_verify_other_codes(gpu, k, p):
    S, nobj = 9000, 4
    n = k + p
    pitch = 9008
    enc = ia.New(k, p)
    st = torch.cuda.current_stream()
    b = _batch(k, p, nobj, S, pitch, seed=k * 7 + p)
    enc.encode_dev(b, S, pitch, n * pitch, nobj, st)
    torch.cuda.synchronize()
    h = b.cpu().numpy()
    assert np.array_equal(h[:, :, :S], _oracle_parity(enc.matrix(), k, p, h, S)[:, :, :S])
    bad = torch.full((nobj,), 9, dtype=torch.int32, device="cuda")
    enc.verify_dev(b, S, pitch, n * pitch, nobj, bad, st)
    torch.cuda.synchronize()
    assert bad.tolist() == [0] * nobj
    b[1, n - 1, S // 2] ^= 0x44
    b[3, 0, 17] ^= 0x02
    enc.verify_dev(b, S, pitch, n * pitch, nobj, bad, st)
    torch.cuda.synchronize()
    assert bad.tolist() == [0, 1, 0, 1]


@pytest.mark.parametrize("lost", [(0, 5), (1, 8), (2, 3, 9)])
@pytest.mark.parametrize("S,pitch", [(104858, 105216), (5003, 5004)])
def test_tri_get_with_extra_checks(gpu, lost, S, pitch):
    """12 (or 11) of 14 shards present: the rebuilt rows equal the oracle's
    Reconstruct from the first 10 present, every clean object's flag is 0, and
    one corrupted byte of an extra (checked) parity shard flags exactly its
    object, however the rebuilt rows come out."""
    k, p, nobj = 10, 4, 5
    n = k + p
    enc = ia.New(k, p)
    st = torch.cuda.current_stream()
    b = _batch(k, p, nobj, S, pitch, seed=S + len(lost))
    enc.encode_dev(b, S, pitch, n * pitch, nobj, st)
    torch.cuda.synchronize()
    golden = b.clone()
    present = [i not in lost for i in range(n)]
    surv = [i for i in range(n) if present[i]][:k]
    extra = [i for i in range(n) if present[i]][k:]
    assert len(extra) == n - len(lost) - k
    b[3, extra[-1], S - 1] ^= 0x5A
    for i in lost:
        b[:, i] = 0xC3
    bad = torch.full((nobj,), 7, dtype=torch.int32, device="cuda")
    enc.decode_dev(b, present, S, pitch, n * pitch, nobj, bad, st)
    torch.cuda.synchronize()
    assert bad.tolist() == [0, 0, 0, 1, 0]
    h = b.cpu().numpy()
    g = golden.cpu().numpy()
    # rows rebuilt from the first k present shards: equal to the data before
    assert np.array_equal(h[:, list(lost), :S], g[:, list(lost), :S])
    # and to the oracle's restatement of upstream Reconstruct on the same rows
    m = enc.matrix()
    e, inv = oracle.invert(m[surv])
    assert e == 0
    for o in (0, 4):
        want = oracle.apply(inv[list(lost)], [g[o, c, :S] for c in surv])
        for j, i in enumerate(lost):
            assert np.array_equal(h[o, i, :S], want[j])
