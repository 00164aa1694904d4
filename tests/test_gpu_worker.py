"""The resident per-object worker (rsgpu_worker_start) against the oracle,
bit-exact: Client.encode (ecRedis.go:382-402) and Client.decode (:404-432) on
single objects, the reference's own call granularity (one object per EcSet /
EcGet; the example object is 1 KiB, client/example/main.go:15,26).

Covered: every per-object operation (Encode, fused Encode+Verify, Verify,
Reconstruct, ReconstructData, fused decode with real extra-shard checks),
pinned Split images read and written in place and pageable buffers staged
through the mailbox images, one pinned buffer rewritten between calls (the
worker must never see stale bytes), shard sizes 1 B - 16 KiB around the
16-B vector tails, several codes (two sub-passes for p > 4, n = 16), idle
exit + relaunch, stop / restart, concurrent callers (declined calls take
the stream path), objects above max_shard, and a multi-entry context."""
import ctypes
import threading
import time

import numpy as np
import pytest

import infinicache_amd as ia
import oracle
from oracle import rs_numpy as rn

pytestmark = pytest.mark.gpu
SEED = 0x3C3C


def _full(k, p, size, idx):
    d = rn.splitmix64_bytes(SEED, idx, k * size).reshape(k, size)
    e, sh = oracle.encode(k, p, [d[i] for i in range(k)] + [bytes(size)] * p)
    assert e == 0
    return [np.frombuffer(bytes(s), np.uint8) for s in sh]


def _image(n, S, pinned):
    buf = ia.host_alloc(n * S) if pinned else np.zeros(n * S, np.uint8)
    return buf, [buf[i * S:(i + 1) * S] for i in range(n)]


@pytest.mark.parametrize("pinned", [True, False])
def test_worker_every_op_vs_oracle(gpu, pinned):
    k, p = 10, 2
    n = k + p
    enc = ia.New(k, p)
    enc.worker_start(max_shard=16384)
    for idx, S in enumerate([1, 15, 16, 17, 103, 410, 1000, 4096, 4099, 16384]):
        full = _full(k, p, S, idx)
        buf, sh = _image(n, S, pinned)
        for j in range(k):
            sh[j][:] = full[j]
        assert enc.EncodeVerify(sh)
        for j in range(n):
            assert np.array_equal(sh[j], full[j]), (S, j)
        sh[k][:] = 0
        enc.Encode(sh)
        assert np.array_equal(sh[k], full[k])
        assert enc.Verify(sh)
        sh[n - 1][S - 1] ^= 0x80
        assert not enc.Verify(sh)
        sh[n - 1][S - 1] ^= 0x80
        # a Get that received exactly k bodies: data 0 and 5 missing (the
        # mirror allocates their buffers, as upstream reconstruct does)
        got = [None if j in (0, 5) else sh[j] for j in range(n)]
        assert enc.DecodeVerify(got)
        assert np.array_equal(got[0], full[0]) and np.array_equal(got[5], full[5])
        # one lost data row: the extra parity shard is really checked
        bad = [None if j == 3 else sh[j] for j in range(n)]
        assert enc.DecodeVerify(bad)
        assert np.array_equal(bad[3], full[3])
        sh[11][0] ^= 1
        bad = [None if j == 3 else sh[j] for j in range(n)]
        assert not enc.DecodeVerify(bad)
        assert np.array_equal(bad[3], full[3])  # rebuilt from the first k present, as upstream
        sh[11][0] ^= 1
        # Reconstruct / ReconstructData
        got = [None if j in (1, 10) else sh[j] for j in range(n)]
        enc.Reconstruct(got)
        assert np.array_equal(got[1], full[1]) and np.array_equal(got[10], full[10])
        got = [None if j in (2, 11) else sh[j] for j in range(n)]
        enc.ReconstructData(got)
        assert np.array_equal(got[2], full[2]) and got[11] is None  # parity left missing
    st = enc.worker_stats()
    assert st["served"] >= 80 and st["launches"] >= 1, st


def test_worker_in_place_pinned_image_missing_rows(gpu):
    """The Go shim's route (i): one pinned Split image, the missing rows
    passed as their own (zero-length marked) slices of it, rebuilt in place."""
    k, p = 10, 2
    n = k + p
    enc = ia.New(k, p)
    enc.worker_start(max_shard=8192)
    L = ia._lib.load()
    import ctypes
    for idx, S in enumerate([103, 2048, 5003]):
        full = _full(k, p, S, 50 + idx)
        buf, sh = _image(n, S, True)
        for j in range(n):
            sh[j][:] = full[j]
            if j in (0, 5):
                sh[j][:] = 0xEE
        ok = ctypes.c_int(-1)
        present = sum(1 << j for j in range(n) if j not in (0, 5))
        assert L.rsgpu_decode_image(enc._ctx, buf.ctypes.data, S, n, present, ctypes.byref(ok)) == 0
        assert ok.value == 1
        for j in range(n):
            assert np.array_equal(sh[j], full[j]), (S, j)
    assert enc.worker_stats()["served"] >= 3


def test_worker_buffer_rewritten_between_calls(gpu):
    """One pinned image re-filled with new bytes 300 times: every request must
    read what the host wrote last (no stale GPU cache lines)."""
    k, p, S = 10, 2, 103
    n = k + p
    enc = ia.New(k, p)
    enc.worker_start(nslots=2)
    m = enc.matrix()
    buf, sh = _image(n, S, True)
    rng = np.random.default_rng(1)
    for it in range(300):
        data = rng.integers(0, 256, (k, S), dtype=np.uint8)
        for j in range(k):
            sh[j][:] = data[j]
        assert enc.EncodeVerify(sh)
        want = oracle.apply(m[k:], [data[j] for j in range(k)])
        for r in range(p):
            assert np.array_equal(sh[k + r], want[r]), it
    assert enc.worker_stats()["served"] >= 300


@pytest.mark.parametrize("k,p", [(1, 1), (4, 2), (10, 4), (6, 6), (12, 4), (13, 3)])
def test_worker_codes(gpu, k, p):
    n = k + p
    enc = ia.New(k, p)
    enc.worker_start()
    rng = np.random.default_rng(n * 7 + p)
    for it, S in enumerate([7, 333, 3000]):
        full = _full(k, p, S, 100 + it)
        sh = [full[j].copy() if j < k else np.zeros(S, np.uint8) for j in range(n)]
        assert enc.EncodeVerify(sh)
        for j in range(n):
            assert np.array_equal(sh[j], full[j])
        lost = sorted(rng.choice(n, int(rng.integers(1, p + 1)), replace=False).tolist())
        got = [None if j in lost else sh[j].copy() for j in range(n)]
        assert enc.DecodeVerify(got)
        for j in range(n):
            assert np.array_equal(got[j], full[j]), (k, p, S, lost, j)
    assert enc.worker_stats()["served"] >= 6


def test_worker_idle_exit_relaunch_and_stop(gpu):
    k, p = 10, 2
    n = k + p
    enc = ia.New(k, p)
    enc.worker_start(nslots=4, idle_us=2000)  # leaves after 2 ms without requests
    full = _full(k, p, 1000, 7)
    for rnd in range(4):
        sh = [full[j].copy() if j < k else np.zeros(1000, np.uint8) for j in range(n)]
        assert enc.EncodeVerify(sh)
        assert np.array_equal(sh[k], full[k])
        time.sleep(0.03)
    st = enc.worker_stats()
    assert st["launches"] >= 4, st  # one relaunch per idle period
    enc.worker_stop()
    served = enc.worker_stats()["served"]
    sh = [full[j].copy() if j < k else np.zeros(1000, np.uint8) for j in range(n)]
    assert enc.EncodeVerify(sh)  # stream path again
    assert np.array_equal(sh[k + 1], full[k + 1])
    enc.worker_start(nslots=3)
    assert enc.EncodeVerify(sh)
    assert enc.worker_stats()["served"] >= 1


def test_worker_large_shards_take_stream_path(gpu):
    """Past the column slices' limit (64 KiB shards) every object takes the
    stream path, pinned or pageable; pageable objects past max_shard but
    within it go to several mailboxes through their images (staged slices)."""
    k, p = 10, 2
    n = k + p
    enc = ia.New(k, p)
    enc.worker_start(max_shard=4096)
    full = _full(k, p, 70000, 9)
    sh = [full[j].copy() if j < k else np.zeros(70000, np.uint8) for j in range(n)]
    assert enc.EncodeVerify(sh)
    assert np.array_equal(sh[k], full[k])
    assert enc.worker_stats()["served"] == 0
    full = _full(k, p, 9000, 10)
    sh = [full[j].copy() if j < k else np.zeros(9000, np.uint8) for j in range(n)]
    assert enc.EncodeVerify(sh)
    assert all(np.array_equal(sh[j], full[j]) for j in range(n))
    assert enc.worker_stats()["served"] == 1


def test_worker_concurrent_callers(gpu):
    """8 threads on 3 mailboxes: calls that find every mailbox busy take the
    stream path; every result is exact either way."""
    k, p = 10, 2
    n = k + p
    enc = ia.New(k, p)
    enc.worker_start(nslots=3)
    errors = []

    def caller(tid):
        try:
            for i in range(25):
                S = 64 + 37 * tid + i
                full = _full(k, p, S, 1000 + tid * 100 + i)
                buf, sh = _image(n, S, tid % 2 == 0)
                for j in range(k):
                    sh[j][:] = full[j]
                assert enc.EncodeVerify(sh)
                got = [None if j in (tid % n, (i + 3) % n) else sh[j] for j in range(n)]
                assert enc.DecodeVerify(got)
                for j in range(n):
                    assert np.array_equal(got[j], full[j])
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    th = [threading.Thread(target=caller, args=(t,)) for t in range(8)]
    for t in th:
        t.start()
    for t in th:
        t.join(180)
    assert not errors, errors[:3]
    st = enc.worker_stats()
    assert st["served"] + st["declined"] == 8 * 25 * 2, st
    assert st["served"] > 0


def test_worker_multi_entry_context(gpu):
    k, p = 10, 2
    n = k + p
    enc = ia.New(k, p, devices=[0, 0])
    enc.worker_start(nslots=2)
    # worker start / stop are not compute calls: the counts
    # below come from the coding calls alone
    base = enc.device_calls()
    assert base == [0, 0], base
    for i, S in enumerate([5, 800, 4096]):
        full = _full(k, p, S, 300 + i)
        sh = [full[j].copy() if j < k else np.zeros(S, np.uint8) for j in range(n)]
        assert enc.EncodeVerify(sh)
        got = [None if j in (i, i + 6) else sh[j] for j in range(n)]
        assert enc.DecodeVerify(got)
        for j in range(n):
            assert np.array_equal(got[j], full[j])
    assert enc.worker_stats()["served"] >= 6
    assert all(c > b for c, b in zip(enc.device_calls(), base)), (enc.device_calls(), base)


def test_worker_deadline_takes_request_back(gpu, monkeypatch):
    """post_and_wait's deadline (RSGPU_WORKER_TIMEOUT_US, read when the worker
    starts): with a 1 us deadline, a call that had to relaunch the idle
    kernel finds no start mark on its slot in time, takes its request back
    and goes down the stream path (declined); a call whose workgroup is
    running waits for it.  Every result is exact either way, and every call
    is either served or declined."""
    k, p = 10, 2
    n = k + p
    monkeypatch.setenv("RSGPU_WORKER_TIMEOUT_US", "1")
    enc = ia.New(k, p)
    enc.worker_start(nslots=2, idle_us=1000)  # leaves after 1 ms without requests
    calls = 0
    for i in range(40):
        S = 103 + 7 * i
        full = _full(k, p, S, 400 + i)
        sh = [full[j].copy() if j < k else np.zeros(S, np.uint8) for j in range(n)]
        assert enc.EncodeVerify(sh)
        for j in range(n):
            assert np.array_equal(sh[j], full[j]), (i, j)
        got = [None if j in (i % n, (i + 4) % n) else sh[j] for j in range(n)]
        assert enc.DecodeVerify(got)
        for j in range(n):
            assert np.array_equal(got[j], full[j]), (i, j)
        calls += 2
        if i % 2:
            time.sleep(0.005)  # the kernel idles out: the next call relaunches it
    st = enc.worker_stats()
    assert st["served"] + st["declined"] == calls, st
    assert st["declined"] > 0 and st["launches"] >= 2, st
    enc.worker_stop()


@pytest.mark.parametrize("nslots,max_shard", [(16, 4096), (8, 16384)])
def test_worker_staged_column_slices_pageable(gpu, nslots, max_shard):
    """Pageable objects past max_shard (the Go Split array an EcSet passes):
    staged column slices, every operation through the mirror (missing rows
    are fresh buffers), against the oracle."""
    k, p = 10, 2
    n = k + p
    enc = ia.New(k, p)
    enc.worker_start(nslots=nslots, max_shard=max_shard)
    served = declined = 0
    for idx, S in enumerate([max_shard + 1, 9000, 16384, 26215]):
        full = _full(k, p, S, 800 + idx)
        sh = [full[j].copy() if j < k else np.full(S, 0x33, np.uint8) for j in range(n)]
        assert enc.EncodeVerify(sh), S
        assert all(np.array_equal(sh[j], full[j]) for j in range(n)), S
        sh[k + 1][:] = 0
        enc.Encode(sh)
        assert np.array_equal(sh[k + 1], full[k + 1]), S
        assert enc.Verify(sh), S
        sh[k][S - 1] ^= 4
        assert not enc.Verify(sh), S
        sh[k][S - 1] ^= 4
        got = [None if j in (0, 5) else sh[j] for j in range(n)]
        assert enc.DecodeVerify(got), S
        assert np.array_equal(got[0], full[0]) and np.array_equal(got[5], full[5]), S
        bad = [None if j == 7 else sh[j] for j in range(n)]
        bad[11] = bad[11].copy()
        bad[11][0] ^= 1
        assert not enc.DecodeVerify(bad), S
        assert np.array_equal(bad[7], full[7]), S
        got = [None if j in (2, 11) else sh[j] for j in range(n)]
        enc.ReconstructData(got)
        assert np.array_equal(got[2], full[2]) and got[11] is None, S
        got = [None if j in (3, 10) else sh[j] for j in range(n)]
        enc.Reconstruct(got)
        assert np.array_equal(got[3], full[3]) and np.array_equal(got[10], full[10]), S
        st = enc.worker_stats()
        if S <= 16384:  # staged slices (up to 16 KiB shards): every call above served
            assert st["served"] - served == 8 and st["declined"] == declined, (S, st)
        else:  # past it: the stream path
            assert st["served"] == served, (S, st)
        served, declined = st["served"], st["declined"]


@pytest.mark.parametrize("nslots", [16, 4])
def test_worker_column_slices_of_large_pinned_objects(gpu, nslots):
    """Objects past max_shard in one pinned Split image go to several
    mailboxes as column slices at the image's pitch (worker_run_split):
    every operation against the oracle, slices ending mid-vector (the last
    one) and on 16-B boundaries, mismatches in the first and last slice."""
    k, p = 10, 2
    n = k + p
    enc = ia.New(k, p)
    enc.worker_start(nslots=nslots, max_shard=1024)
    served0 = enc.worker_stats()["served"]
    assert enc.worker_stats() == {"served": 0, "declined": 0, "launches": 0}
    for idx, S in enumerate([1025, 4099, 6554, 33333, 65536]):
        full = _full(k, p, S, 600 + idx)
        buf, sh = _image(n, S, True)
        for j in range(k):
            sh[j][:] = full[j]
        assert enc.EncodeVerify(sh)
        for j in range(n):
            assert np.array_equal(sh[j], full[j]), (S, j)
        assert enc.worker_stats()["served"] == served0 + 1, (S, enc.worker_stats())
        sh[k][:] = 0
        enc.Encode(sh)
        assert np.array_equal(sh[k], full[k]), S
        assert enc.Verify(sh)
        for pos in (0, S - 1):
            sh[n - 1][pos] ^= 0x80
            assert not enc.Verify(sh), (S, pos)
            sh[n - 1][pos] ^= 0x80
        # Gets on the image itself (the Go shim's route: missing rows are rows
        # of the pinned image, rebuilt in place; *_image calls)
        L = ia._lib.load()
        ok = ctypes.c_int(-1)

        def call(fn, present, *extra):
            return fn(enc._ctx, buf.ctypes.data, S, n, ctypes.c_uint64(present), *extra)

        def lost(*rows):
            for j in rows:
                sh[j][:] = 0xEE
            return sum(1 << j for j in range(n) if j not in rows)

        assert call(L.rsgpu_decode_image, lost(0, 5), ctypes.byref(ok)) == 0 and ok.value == 1, S
        assert np.array_equal(sh[0], full[0]) and np.array_equal(sh[5], full[5]), S
        sh[11][S - 1] ^= 1  # the extra shard wrong in the last slice only
        assert call(L.rsgpu_decode_image, lost(3), ctypes.byref(ok)) == 0 and ok.value == 0, S
        assert np.array_equal(sh[3], full[3]), S  # rebuilt from the first k present, as upstream
        sh[11][S - 1] ^= 1
        assert call(L.rsgpu_reconstruct_image, lost(1, 10), 0) == 0, S
        assert np.array_equal(sh[1], full[1]) and np.array_equal(sh[10], full[10]), S
        assert call(L.rsgpu_reconstruct_image, lost(2, 11), 1) == 0, S  # ReconstructData
        assert np.array_equal(sh[2], full[2]) and np.all(sh[11] == 0xEE), S  # parity left as it was
        sh[11][:] = full[11]
        st = enc.worker_stats()
        assert st["served"] - served0 == 9 and st["declined"] == 0, (S, st)  # every call above
        served0 = st["served"]
    # past the slices' limit (64 KiB shards): the stream path, results exact
    S = 104858
    full = _full(k, p, S, 699)
    buf, sh = _image(n, S, True)
    for j in range(k):
        sh[j][:] = full[j]
    assert enc.EncodeVerify(sh)
    assert all(np.array_equal(sh[j], full[j]) for j in range(n))
    st = enc.worker_stats()
    assert st["served"] == served0 and st["declined"] == 1, st


def test_worker_column_slices_beside_small_callers(gpu):
    """Large pinned objects (column slices over several mailboxes) and 1 KiB
    callers on one worker: slices and small requests share the mailboxes,
    calls that find too few free take the stream path; every result exact."""
    k, p = 10, 2
    n = k + p
    enc = ia.New(k, p)
    enc.worker_start(nslots=8)
    errors = []

    def caller(tid):
        try:
            for i in range(20):
                S = 50000 + 4099 * tid + 17 * i if tid < 2 else 103 + tid + i
                full = _full(k, p, S, 2000 + tid * 100 + i)
                buf, sh = _image(n, S, True)
                for j in range(k):
                    sh[j][:] = full[j]
                assert enc.EncodeVerify(sh)
                got = [None if j in (tid % n, (i + 3) % n) else sh[j] for j in range(n)]
                assert enc.DecodeVerify(got)
                for j in range(n):
                    assert np.array_equal(got[j], full[j]), (tid, i, j)
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    th = [threading.Thread(target=caller, args=(t,)) for t in range(6)]
    for t in th:
        t.start()
    for t in th:
        t.join(180)
    assert not errors, errors[:3]
    st = enc.worker_stats()
    assert st["served"] + st["declined"] == 6 * 20 * 2, st
    assert st["served"] > 0


def test_worker_slices_on_multi_entry_context(gpu):
    """Column slices through a multi-entry context (per-object calls go to
    the entries round-robin, each entry its own worker): pinned images and
    pageable buffers past max_shard, every result exact, every entry used."""
    k, p = 10, 2
    n = k + p
    enc = ia.New(k, p, devices=[0, 0])
    enc.worker_start(nslots=8, max_shard=2048)
    for i, (S, pinned) in enumerate([(20000, True), (9000, False), (50001, True), (16000, False)] * 2):
        full = _full(k, p, S, 900 + i)
        buf, sh = _image(n, S, pinned)
        for j in range(k):
            sh[j][:] = full[j]
        assert enc.EncodeVerify(sh), (S, pinned)
        assert all(np.array_equal(sh[j], full[j]) for j in range(n)), (S, pinned)
        got = [None if j in (i % n, (i + 7) % n) else sh[j] for j in range(n)]
        assert enc.DecodeVerify(got), (S, pinned)
        assert all(np.array_equal(got[j], full[j]) for j in range(n)), (S, pinned)
    st = enc.worker_stats()
    assert st["served"] >= 8, st
    assert all(c > 0 for c in enc.device_calls()), enc.device_calls()
