"""Multi-device contexts, the host pipeline at config-5 sizes, and the
host-memory edge cases, through the C ABI against the oracle (bit-exact).

* A context over every visible GPU (RSGPU_ALL_DEVICES / rsgpu_create_multi,
  what the Go shim's NewEncoder builds, client/ec.go:14-24): per-object
  calls round-robin, batch calls split objects o -> device o mod N,
  device-resident calls follow the memory.  The test box has one GPU, so
  these run the forwarding path with N = 1; the driver's 8-GPU node runs the
  same code with N = 8.
* BASELINE config 5's host pipeline at its real sizes: a log-uniform trace
  with 4 KiB objects and a 64+ MiB object (client/ecRedis.go:96 Set buffer,
  :161-173 gathered Get buffers), pinned and pageable.
* Pinned user memory (rsgpu_host_register, no slack past the buffer) with a
  shard size that is not a multiple of 16."""
import os

import numpy as np
import pytest

import infinicache_amd as ia
import oracle
from oracle import rs_numpy as rn

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
SEED = 0x1F1C


def _full(k, p, size, idx):
    d = rn.splitmix64_bytes(SEED, idx, k * size).reshape(k, size)
    e, sh = oracle.encode(k, p, [d[i] for i in range(k)] + [bytes(size)] * p)
    assert e == 0
    return sh


def test_all_devices_context(gpu):
    enc = ia.New(10, 2, device=ia.ALL_DEVICES)
    assert enc.devices() == [d for d in range(ia.device_count()) if ia.device_ok(d)]
    # per-object calls round-robin over the devices: Client.encode / decode
    for i, size in enumerate([1, 103, 4096, 104858, 77777]):
        full = _full(10, 2, size, 900 + i)
        sh = [full[j].copy() if j < 10 else np.zeros(size, np.uint8) for j in range(12)]
        assert enc.EncodeVerify(sh)
        for j in range(12):
            assert np.array_equal(sh[j], full[j]), (size, j)
        got = [None if j in (i % 12, (i + 5) % 12) else sh[j] for j in range(12)]
        assert enc.DecodeVerify(got)
        for j in range(12):
            assert np.array_equal(got[j], full[j]), (size, j)


def test_multi_device_batches(gpu):
    devs = [d for d in range(ia.device_count()) if ia.device_ok(d)]
    enc = ia.New(10, 4, devices=devs)
    sizes = [5, 4096, 1 << 20, 333, 70001, 4 << 20, 17]
    objs, fulls = [], []
    for i, nb in enumerate(sizes):
        data = rn.splitmix64_bytes(SEED, 950 + i, nb)
        sh = enc.Split(data)
        S = len(sh[0])
        buf = ia.host_alloc(14 * S) if i % 2 else np.zeros(14 * S, np.uint8)
        buf[:] = np.concatenate(sh)
        objs.append([buf[j * S:(j + 1) * S] for j in range(14)])
        e, want = oracle.encode(10, 4, [s.copy() for s in sh[:10]] + [bytes(S)] * 4)
        fulls.append(want)
    enc.encode_batch(objs)
    for sh, want in zip(objs, fulls):
        for j in range(14):
            assert np.array_equal(sh[j], want[j])
    lost = [(0, 5), (1, 2, 3), (), (13,), (0, 10, 11, 12), (6, 7), (9,)]
    present = [[j not in lost[o] for j in range(14)] for o in range(len(sizes))]
    for o in range(len(sizes)):
        for j in lost[o]:
            objs[o][j][:] = 0xEE
    ok = enc.decode_batch(objs, present=present)
    assert ok == [True] * len(sizes)
    for sh, want in zip(objs, fulls):
        for j in range(14):
            assert np.array_equal(sh[j], want[j])


def test_multi_device_dev_calls_follow_the_memory(gpu):
    enc = ia.New(10, 2, device=ia.ALL_DEVICES)
    k, p, S, nobj = 10, 2, 5000, 6
    pitch = 5120
    g = torch.Generator(device="cuda:0").manual_seed(4)
    b = torch.randint(0, 256, (nobj, k + p, pitch), dtype=torch.uint8, device="cuda:0", generator=g)
    b[:, :, S:] = 0
    enc.encode_dev(b, S, pitch, (k + p) * pitch, nobj, torch.cuda.current_stream())
    torch.cuda.synchronize()
    h = b.cpu().numpy()
    m = enc.matrix()
    for o in range(nobj):
        want = oracle.apply(m[k:], [h[o, c, :S] for c in range(k)])
        for r in range(p):
            assert np.array_equal(h[o, k + r, :S], want[r])
    hostbuf = np.zeros((k + p) * pitch, np.uint8)  # not device memory: no device owns it
    with pytest.raises(ia.InvalidArgument):
        enc.encode_dev(hostbuf.ctypes.data, S, pitch, (k + p) * pitch, 1)


@pytest.mark.parametrize("entries", [2, 3])
def test_repeated_device_entries_every_forwarding_path(gpu, entries):
    """N > 1 on the one-GPU test box: a context over device 0 listed N times
    has N independent entries, so every multi-device forwarding path runs
    with N > 1 (client/client.go:47-59, ecRedis.go:102-109 fan-out):
    per-object round robin, the batch split o -> entry o mod N on N - 1 extra
    host threads with the merged ok[], and device-resident calls routed by
    the memory's owner (entries of one device in turn).  Every result
    against the oracle; device_calls() shows each path reached each entry."""
    k, p = 10, 2
    n = k + p
    enc = ia.New(k, p, devices=[0] * entries)
    assert enc.devices() == [0] * entries
    m = enc.matrix()

    def spread(before):
        now = enc.device_calls()
        return [a - b for a, b in zip(now, before)]

    # per-object host calls: round robin over the entries
    c0 = enc.device_calls()
    for i, size in enumerate([1, 103, 4096, 104858, 77777, 5000]):
        full = _full(k, p, size, 1200 + i)
        sh = [full[j].copy() if j < k else np.zeros(size, np.uint8) for j in range(n)]
        assert enc.EncodeVerify(sh)
        for j in range(n):
            assert np.array_equal(sh[j], full[j]), (size, j)
        got = [None if j in (i % n, (i + 7) % n) else sh[j] for j in range(n)]
        assert enc.DecodeVerify(got)
        for j in range(n):
            assert np.array_equal(got[j], full[j]), (size, j)
    d = spread(c0)
    assert all(x >= 12 // entries for x in d), d

    # host batches: object o -> entry o mod N, one host thread per extra
    # entry; object 4's parity is corrupted before decode, so its ok[] entry
    # must come back False at index 4 whatever entry coded it
    c0 = enc.device_calls()
    sizes = [5, 4096, 1 << 20, 333, 70001, 17, 9999]
    objs, fulls = [], []
    for i, nb in enumerate(sizes):
        data = rn.splitmix64_bytes(SEED, 1300 + i, nb)
        sh = enc.Split(data)
        S = len(sh[0])
        buf = ia.host_alloc(n * S) if i % 2 else np.zeros(n * S, np.uint8)
        buf[:] = np.concatenate(sh)
        objs.append([buf[j * S:(j + 1) * S] for j in range(n)])
        e, want = oracle.encode(k, p, [s.copy() for s in sh[:k]] + [bytes(S)] * p)
        fulls.append(want)
    enc.encode_batch(objs)
    for sh, want in zip(objs, fulls):
        for j in range(n):
            assert np.array_equal(sh[j], want[j])
    assert all(x >= 1 for x in spread(c0))
    lost = [(0, 5), (1,), (2, 3), (), (4,), (10, 11), (6,)]
    for o in range(len(sizes)):
        for j in lost[o]:
            objs[o][j][:] = 0xEE
    objs[4][11][0] ^= 1  # extra present parity shard of object 4 disagrees
    present = [[j not in lost[o] for j in range(n)] for o in range(len(sizes))]
    ok = enc.decode_batch(objs, present=present)
    assert ok == [o != 4 for o in range(len(sizes))], ok
    for o, (sh, want) in enumerate(zip(objs, fulls)):
        for j in range(n):
            if not (o == 4 and j == 11):
                assert np.array_equal(sh[j], want[j]), (o, j)

    # device-resident calls: each on its own buffer, routed to the entries
    # of device 0 in turn (sub_for), through the plain, host-flag and
    # device-mask forms
    c0 = enc.device_calls()
    S, pitch, nobj = 3000, 3072, 5
    s = torch.cuda.current_stream()
    for t in range(2 * entries):
        g = torch.Generator(device="cuda:0").manual_seed(40 + t)
        b = torch.randint(0, 256, (nobj, n, pitch), dtype=torch.uint8, device="cuda:0", generator=g)
        b[:, :, S:] = 0
        enc.encode_dev(b, S, pitch, n * pitch, nobj, s)
        torch.cuda.synchronize()
        golden = b.clone()
        h = golden.cpu().numpy()
        for o in range(nobj):
            want = oracle.apply(m[k:], [h[o, c, :S] for c in range(k)])
            for r in range(p):
                assert np.array_equal(h[o, k + r, :S], want[r])
        pres = np.ones((nobj, n), np.uint8)
        for o in range(nobj):
            pres[o, [(o + t) % n, (o + t + 3) % n]] = 0
        for o in range(nobj):
            b[o, np.flatnonzero(pres[o] == 0)] = 0x5A
        st = torch.full((nobj,), 9, dtype=torch.int32, device="cuda:0")
        if t % 2:
            masks = torch.from_numpy((pres.astype(np.int64) << np.arange(n)).sum(1).astype(np.int32)).cuda()
            enc.decode_dev_masks(b, masks, S, pitch, n * pitch, nobj, st, s)
        else:
            enc.decode_dev_multi(b, pres, S, pitch, n * pitch, nobj, st, s)
        torch.cuda.synchronize()
        assert not st.any()
        assert torch.equal(b[:, :, :S], golden[:, :, :S]), t
    d = spread(c0)
    assert all(x >= 2 for x in d), d


def test_repeated_entries_concurrent_callers(gpu):
    """Several host threads on one 3-entry context: per-object calls spread
    over the entries' own slot pools and streams concurrently."""
    import threading
    k, p = 10, 2
    n = k + p
    enc = ia.New(k, p, devices=[0, 0, 0])
    errors = []

    def caller(tid):
        try:
            for i in range(6):
                size = 1000 + 97 * tid + i
                full = _full(k, p, size, 1400 + tid * 10 + i)
                sh = [full[j].copy() if j < k else np.zeros(size, np.uint8) for j in range(n)]
                assert enc.EncodeVerify(sh)
                got = [None if j in (tid % n, (i + 4) % n) else sh[j] for j in range(n)]
                assert enc.DecodeVerify(got)
                for j in range(n):
                    assert np.array_equal(got[j], full[j])
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    th = [threading.Thread(target=caller, args=(t,)) for t in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
    assert not errors, errors
    assert all(x > 0 for x in enc.device_calls())


@pytest.mark.parametrize("pinned", [False, True])
def test_trace_pipeline_config5_sizes(gpu, pinned):
    """encode_batch + decode_batch over a small log-uniform trace: 4 KiB
    objects beside one 64+ MiB object (S > 6.7 MB), against the oracle."""
    k, p = 10, 2
    n = k + p
    enc = ia.New(k, p)
    rng = np.random.Generator(np.random.PCG64(20200225))
    sizes = [4096, 4096 + 7] + [int(x) for x in np.exp(rng.uniform(np.log(4096), np.log(1 << 20), 4))]
    sizes += [(64 << 20) + 12345]
    objs, wants = [], []
    for i, nb in enumerate(sizes):
        S = (nb + k - 1) // k
        buf = ia.host_alloc(n * S) if pinned else np.empty(n * S, np.uint8)
        buf[:nb] = rn.splitmix64_bytes(SEED, 1000 + i, nb)
        buf[nb:] = 0
        sh = [buf[j * S:(j + 1) * S] for j in range(n)]
        want = oracle.code_fast(enc.matrix()[k:], [sh[j] for j in range(k)], nthreads=16)
        objs.append(sh)
        wants.append(want)
    enc.encode_batch(objs)
    for sh, want in zip(objs, wants):
        for r in range(p):
            assert np.array_equal(sh[k + r], want[r])
    golden = [[sh[j].copy() for j in range(n)] for sh in objs]
    lost = (0, 5)
    for sh in objs:
        for j in lost:
            sh[j][:] = 0
    ok = enc.decode_batch(objs, present=[[j not in lost for j in range(n)]] * len(objs))
    assert all(ok)
    for sh, gd in zip(objs, golden):
        for j in range(n):
            assert np.array_equal(sh[j], gd[j])


@pytest.mark.parametrize("S", [1003, 4097, 104858])
def test_registered_user_buffer_unaligned_shards(gpu, S):
    """A numpy Split buffer pinned with rsgpu_host_register (no slack: the
    last row's 16-B vector would run past the end, so the pass must not read
    it in place) and unregistered afterwards."""
    k, p = 10, 2
    n = k + p
    enc = ia.New(k, p)
    full = _full(k, p, S, 1100 + S % 97)
    buf = np.empty(n * S, np.uint8)
    ia.host_register(buf)
    try:
        for j in range(n):
            buf[j * S:(j + 1) * S] = full[j] if j < k else 0
        sh = [buf[j * S:(j + 1) * S] for j in range(n)]
        enc.Encode(sh)
        for j in range(n):
            assert np.array_equal(sh[j], full[j])
        assert enc.Verify(sh)
        sh[k][:] = 0
        assert enc.EncodeVerify(sh)
        assert np.array_equal(sh[k], full[k])
        got = [None if j in (0, n - 1) else sh[j] for j in range(n)]
        enc.Reconstruct(got)
        for j in range(n):
            assert np.array_equal(got[j], full[j])
    finally:
        ia.host_unregister(buf)


def test_pass_image_cache_keyed_by_shard_len(gpu):
    """A wide code (n > 16: host-planned mixed-pattern path) decoded twice on
    one encoder, same pitch, two shard lengths: the cached pass images must
    not carry the first call's span into the second."""
    k, p = 20, 4
    n = k + p
    enc = ia.New(k, p)
    pitch = 8192
    s = torch.cuda.current_stream()
    for S, seed in ((1000, 1), (8000, 2)):
        nobj = 5
        g = torch.Generator(device="cuda").manual_seed(seed)
        b = torch.randint(0, 256, (nobj, n, pitch), dtype=torch.uint8, device="cuda", generator=g)
        b[:, :, S:] = 0
        enc.encode_dev(b, S, pitch, n * pitch, nobj, s)
        golden = b.clone()
        present = np.ones((nobj, n), np.uint8)
        for o in range(nobj):
            present[o, [o, o + 7]] = 0
            b[o, o] = 0
            b[o, o + 7] = 0
        bad = torch.full((nobj,), 3, dtype=torch.int32, device="cuda")
        enc.decode_dev_multi(b, present, S, pitch, n * pitch, nobj, bad, s)
        torch.cuda.synchronize()
        assert not bad.any()
        assert torch.equal(b[:, :, :S], golden[:, :, :S]), S


_GROUP_CHILD = r'''
import sys
import numpy as np
sys.path.insert(0, sys.argv[1])
import infinicache_amd as ia
import oracle
from oracle import rs_numpy as rn
k, p = 10, 2
n = k + p
enc = ia.New(k, p)
m = enc.matrix()
rng = np.random.default_rng(7)
# Split images back to back in one pinned arena: small ones (grouped), two
# past kGroupObjMax (4 MiB images), and one gap that breaks the adjacency
sizes = [4096, 4099, 70000, 1 << 20, 5 << 20, 333, 65536, 100, 4 << 20, 12345, 777777, 3000]
Ss = [(nb + k - 1) // k for nb in sizes]
offs = [0]
for i, S in enumerate(Ss):
    offs.append(offs[-1] + n * S + (4096 if i == 6 else 0))
arena = ia.host_alloc(offs[-1])
objs, datas = [], []
for i, (nb, S) in enumerate(zip(sizes, Ss)):
    img = arena[offs[i]:offs[i] + n * S]
    img[:] = 0
    img[:nb] = rn.splitmix64_bytes(0x5EED, 4000 + i, nb)
    objs.append([img[j * S:(j + 1) * S] for j in range(n)])
enc.encode_batch(objs)
for sh in objs:
    want = oracle.code_fast(m[k:], [sh[j] for j in range(k)], nthreads=8)
    for r in range(p):
        assert np.array_equal(sh[k + r], want[r]), "encode"
golden = [[s.copy() for s in sh] for sh in objs]
# Gets: exactly k bodies (grouped), 11 bodies (a check row: coded alone),
# one of them with a corrupted extra shard (flag), and all 12 (Verify)
present, expect_ok = [], []
for i, sh in enumerate(objs):
    pr = [True] * n
    if i % 4 == 3:
        lost = [int(x) for x in rng.choice(n, 1, replace=False)]
    elif i == 10:
        lost = []
    else:
        lost = [int(x) for x in rng.choice(n, 2, replace=False)]
    for j in lost:
        pr[j] = False
        sh[j][:] = 0xA5
    ok = True
    if i == 7:  # corrupt a present parity shard beyond the survivors
        extra = [j for j in range(n) if pr[j]][k:]
        if extra:
            sh[extra[0]][0] ^= 1
            ok = False
    present.append(pr)
    expect_ok.append(ok)
got = enc.decode_batch(objs, present=present)
assert got == expect_ok, (got, expect_ok)
for i, (sh, gd) in enumerate(zip(objs, golden)):
    for j in range(n):
        if not present[i][j]:
            assert np.array_equal(sh[j], gd[j]), ("decode", i, j)
print("group ok", len(objs))
'''


@pytest.mark.parametrize("group", ["0", str(8 << 20), str(64 << 10)])
def test_batches_group_adjacent_small_objects(gpu, group):
    """RSGPU_PIPE_GROUP (read once, so a child process per setting): batches
    of Split images back to back in one pinned arena move their small
    objects as one H2D per group; every result equals the oracle's, Gets
    with check rows (extra bodies, a corrupted one flagged) are coded alone,
    a gap or an image past 4 MiB ends a group.  Off ("0") is the same batch
    through the per-object copies."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, RSGPU_PIPE_GROUP=group)
    r = subprocess.run([sys.executable, "-c", _GROUP_CHILD, root], capture_output=True, text=True, timeout=240,
                       env=env, cwd=root)
    assert r.returncode == 0, r.stderr[-3000:] + r.stdout
    assert "group ok 12" in r.stdout
