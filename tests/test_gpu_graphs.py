"""HIP graph capture of the device-resident calls: after a first (planning)
call, rsgpu_encode_dev / rsgpu_decode_dev / rsgpu_decode_dev_masks issue only
stream-ordered work (kernel launches, async memsets), so a serving loop can
capture a batch's Set + Get into one graph and replay it.  Replays are
compared bit-exact with the oracle on fresh data written into the same
buffers between replays."""
import numpy as np
import pytest

import infinicache_amd as ia
import oracle

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def _check(buf, k, p, S, nobj, lost):
    host = buf[:, :, :S].cpu().numpy()
    for o in range(0, nobj, max(1, nobj // 5)):
        e, want = oracle.encode(k, p, [host[o, i].copy() for i in range(k)] + [bytes(S)] * p)
        assert e == 0
        for i in range(k, k + p):
            assert np.array_equal(host[o, i], want[i]), (o, i)
    return host


def test_capture_encode_decode_step(gpu):
    k, p, S, nobj = 10, 2, 70001, 64
    n = k + p
    pitch = (S + 255) // 256 * 256
    buf = torch.zeros((nobj, n, pitch), dtype=torch.uint8, device="cuda")
    bad = torch.zeros(nobj, dtype=torch.int32, device="cuda")
    enc = ia.New(k, p)
    present = [i not in (0, 5) for i in range(n)]
    st = torch.cuda.Stream()
    g = torch.Generator(device="cuda").manual_seed(5)
    with torch.cuda.stream(st):
        buf[:, :k, :S] = torch.randint(0, 256, (nobj, k, S), dtype=torch.uint8, device="cuda", generator=g)
        # first calls plan and upload (outside the capture)
        enc.encode_dev(buf, S, pitch, n * pitch, nobj, st)
        enc.decode_dev(buf, present, S, pitch, n * pitch, nobj, bad, st)
    st.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=st):
        enc.encode_dev(buf, S, pitch, n * pitch, nobj, st)
        enc.decode_dev(buf, present, S, pitch, n * pitch, nobj, bad, st)
    for rep in range(3):
        with torch.cuda.stream(st):
            buf[:, :k, :S] = torch.randint(0, 256, (nobj, k, S), dtype=torch.uint8, device="cuda", generator=g)
            keep = buf[:, [0, 5], :S].clone()
            buf[:, k:, :] = 0x5A  # stale parity: the replay must recompute it
        st.synchronize()
        graph.replay()
        torch.cuda.synchronize()
        assert int(bad.sum()) == 0, rep
        assert torch.equal(buf[:, [0, 5], :S], keep), rep  # rebuilt rows == the data
        _check(buf, k, p, S, nobj, (0, 5))


def test_capture_mixed_pattern_decode(gpu):
    """decode_dev_masks (patterns resolved on the device from masks in HBM)
    inside a graph: new erasure patterns between replays need no host work."""
    k, p, S, nobj = 10, 2, 4099, 300
    n = k + p
    pitch = (S + 15) // 16 * 16
    buf = torch.zeros((nobj, n, pitch), dtype=torch.uint8, device="cuda")
    masks = torch.zeros(nobj, dtype=torch.int32, device="cuda")
    status = torch.zeros(nobj, dtype=torch.int32, device="cuda")
    enc = ia.New(k, p)
    st = torch.cuda.Stream()
    g = torch.Generator(device="cuda").manual_seed(9)
    rng = np.random.default_rng(9)

    def new_masks():
        m = np.full(nobj, (1 << n) - 1, dtype=np.int64)
        for o in range(nobj):
            for i in rng.choice(n, p, replace=False):
                m[o] &= ~(1 << int(i))
        return torch.from_numpy(m.astype(np.int32)).cuda()

    with torch.cuda.stream(st):
        buf[:, :k, :S] = torch.randint(0, 256, (nobj, k, S), dtype=torch.uint8, device="cuda", generator=g)
        enc.encode_dev(buf, S, pitch, n * pitch, nobj, st)
        masks.copy_(new_masks())
        enc.decode_dev_masks(buf, masks, S, pitch, n * pitch, nobj, status, st)  # builds the atlas
    st.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=st):
        enc.decode_dev_masks(buf, masks, S, pitch, n * pitch, nobj, status, st)
    for rep in range(3):
        full = buf.clone()
        m = new_masks()
        masks.copy_(m)
        mh = m.cpu().numpy()
        for o in range(nobj):  # garbage into each object's missing rows
            for i in range(n):
                if not (mh[o] >> i) & 1:
                    buf[o, i, :S] = 0xC3
        torch.cuda.synchronize()
        graph.replay()
        torch.cuda.synchronize()
        assert int(status.abs().sum()) == 0, rep
        assert torch.equal(buf[:, :, :S], full[:, :, :S]), rep
