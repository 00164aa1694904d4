"""The resident worker beside the rest of the library (VERDICT r03 next #2,
ADVICE r03 high/medium): concurrent EcSet / EcGet callers on one Client.EC
(client/ecRedis.go:58-191) mix 1 KiB objects, which the worker serves, with
multi-MiB objects, which take the stream path and grow its staging.

While the worker's kernel is resident, a runtime call that synchronises the
device (hipFree / hipHostFree, a null-stream hipMemcpy) waits for it to
leave, which never happens while other callers keep it busy.  These tests
keep it busy from 4 threads and require every other path to finish within a
stated wall-clock bound, bit-exact against the oracle:
  * per-object stream-path calls of growing size (64 KiB -> 4 MiB -> 16 MiB
    objects: the context's staging slot grows at every step),
  * a wide-code (RS(20+4): no device atlas) *_dev_masks call, whose masks
    come back to the host and whose generic plans are uploaded on first use,
  * worker_stop / worker_start while callers are in flight (ADVICE r03
    medium: late callers are declined to the stream path, never served by a
    launch whose mailboxes are being freed)."""
import threading
import time

import numpy as np
import pytest

import infinicache_amd as ia
import oracle
from oracle import rs_numpy as rn

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

K, P = 10, 2
N = K + P
BUSY_CAP_S = 20.0   # the busy callers stop by themselves after this: the test ends even if a call stalls
STREAM_BOUND_S = 8.0  # every stream-path / device call of the other thread must finish within this


def _full(k, p, size, idx):
    d = rn.splitmix64_bytes(0x5EED, idx, k * size).reshape(k, size)
    e, sh = oracle.encode(k, p, [d[i] for i in range(k)] + [bytes(size)] * p)
    assert e == 0
    return [np.frombuffer(bytes(s), np.uint8) for s in sh]


class _Busy:
    """4 threads, each coding its own 1 KiB object (S = 103) through the
    worker in a loop: fused encode+verify, then a decode with two lost rows."""

    def __init__(self, enc, nthreads=4):
        self.enc = enc
        self.stop = threading.Event()
        self.errors = []
        self.calls = [0] * nthreads
        self.th = [threading.Thread(target=self._run, args=(t,), daemon=True) for t in range(nthreads)]

    def _run(self, tid):
        S = 103
        full = _full(K, P, S, 7000 + tid)
        buf = ia.host_alloc(N * S)
        sh = [buf[i * S:(i + 1) * S] for i in range(N)]
        t_end = time.monotonic() + BUSY_CAP_S
        i = 0
        try:
            while not self.stop.is_set() and time.monotonic() < t_end:
                for j in range(K):
                    sh[j][:] = full[j]
                for j in range(K, N):
                    sh[j][:] = 0
                assert self.enc.EncodeVerify(sh)
                for j in range(K, N):
                    assert np.array_equal(sh[j], full[j]), (tid, i, j)
                lost = (tid % N, (i + 5) % N)
                got = [None if j in lost else sh[j] for j in range(N)]
                assert self.enc.DecodeVerify(got)
                for j in lost:
                    assert np.array_equal(got[j], full[j]), (tid, i, j)
                self.calls[tid] += 2
                i += 1
        except Exception as e:  # noqa: BLE001
            self.errors.append(f"thread {tid} call {i}: {e!r}")

    def __enter__(self):
        for t in self.th:
            t.start()
        # the kernel is resident once the callers are being served
        t0 = time.monotonic()
        while sum(self.calls) < 40 and time.monotonic() - t0 < 30 and not self.errors:
            time.sleep(0.005)
        return self

    def __exit__(self, *a):
        self.stop.set()
        for t in self.th:
            t.join(BUSY_CAP_S + 30)


def _timed(fn, log, what):
    t0 = time.monotonic()
    r = fn()
    log.append((what, time.monotonic() - t0))
    return r


def test_worker_busy_beside_stream_path_growth_and_wide_masks(gpu):
    enc = ia.New(K, P)
    enc.worker_start(nslots=8)  # defaults: 50 ms idle exit, max_shard 4 KiB
    # the wide-code batch is built before the worker runs; it is coded while it runs
    kw, pw, Sw, nobj = 20, 4, 3000, 50
    nw = kw + pw
    pitch = (Sw + 15) // 16 * 16
    side = torch.cuda.Stream()  # non-blocking: never ordered behind the worker's stream
    wide = ia.New(kw, pw)
    with torch.cuda.stream(side):
        g = torch.Generator(device="cuda").manual_seed(11)
        b = torch.randint(0, 256, (nobj, nw, pitch), dtype=torch.uint8, device="cuda", generator=g)
        b[:, :, Sw:] = 0
        wide.encode_dev(b, Sw, pitch, nw * pitch, nobj, side)
        golden = b.clone()
    side.synchronize()
    rng = np.random.default_rng(5)
    present = np.ones((nobj, nw), np.uint8)
    for o in range(nobj):
        present[o, rng.choice(nw, int(rng.integers(1, pw + 1)), replace=False)] = 0
    masks = (present.astype(np.int64) * (1 << np.arange(nw, dtype=np.int64))).sum(axis=1).astype(np.uint32)

    log = []
    with _Busy(enc) as busy:
        assert not busy.errors, busy.errors[:2]
        t_start = time.monotonic()
        for idx, size in enumerate([64 << 10, 4 << 20, 16 << 20]):
            obj = rn.splitmix64_bytes(0xB16, idx, size)
            sh = enc.Split(obj)  # pageable shards: staged through the context's slot, which grows
            _timed(lambda: enc.Encode(sh), log, f"Encode {size >> 10} KiB")
            S = len(sh[0])
            e, want = oracle.encode(K, P, [bytes(s) for s in sh[:K]] + [bytes(S)] * P)
            assert e == 0
            for r in range(P):
                assert np.array_equal(sh[K + r], want[K + r]), (size, r)
            got = [None if j in (1, 10) else sh[j] for j in range(N)]
            assert _timed(lambda: enc.DecodeVerify(got), log, f"DecodeVerify {size >> 10} KiB")
            for j in (1, 10):
                assert np.array_equal(got[j], want[j]), (size, j)
        with torch.cuda.stream(side):
            for o in range(nobj):
                lost = np.flatnonzero(present[o] == 0)
                b[o, torch.as_tensor(lost, dtype=torch.long)] = 0xA5
            dmask = torch.from_numpy(masks.view(np.int32)).to("cuda", non_blocking=False)
            status = torch.full((nobj,), 9, dtype=torch.int32, device="cuda")

        def wide_call():
            wide.decode_dev_masks(b, dmask, Sw, pitch, nw * pitch, nobj, status, side)
            side.synchronize()

        _timed(wide_call, log, "RS(20+4) decode_dev_masks")
        t_all = time.monotonic() - t_start
        calls_during = sum(busy.calls)
    assert not busy.errors, busy.errors[:2]
    print("stream-path / device calls while the worker was busy:",
          ", ".join(f"{w} {t * 1e3:.1f} ms" for w, t in log), f"(total {t_all:.2f} s)")
    with torch.cuda.stream(side):
        assert torch.equal(b[:, :, :Sw], golden[:, :, :Sw])
        assert int(status.sum().item()) == 0
    st = enc.worker_stats()
    assert st["served"] > 0 and calls_during > 0, st
    assert t_all < STREAM_BOUND_S, f"calls beside the busy worker took {t_all:.1f} s: {log}"
    enc.worker_stop()


def test_worker_busy_beside_user_pinned_alloc_free(gpu):
    """rsgpu_host_free / rsgpu_host_register / _unregister from the user (the
    Go shim's stage pool frees C-owned images) while the worker is busy:
    a free is held back until no worker kernel is resident and
    an unregister parks the workers around the device-synchronising call, so
    each returns promptly; the busy callers are declined to the stream path
    during a park and stay exact."""
    import ctypes
    enc = ia.New(K, P)
    enc.worker_start(nslots=8)
    L = ia._lib.load()
    log = []
    with _Busy(enc) as busy:
        assert not busy.errors, busy.errors[:2]
        t_start = time.monotonic()
        for i in range(20):
            p = ctypes.c_void_p()
            assert L.rsgpu_host_alloc(1 << 20, ctypes.byref(p)) == 0
            _timed(lambda: L.rsgpu_host_free(p), log, "host_free")
        arr = np.zeros(4 << 20, np.uint8)
        for i in range(5):
            _timed(lambda: ia.host_register(arr), log, "host_register")
            _timed(lambda: ia.host_unregister(arr), log, "host_unregister")
        t_all = time.monotonic() - t_start
        before = sum(busy.calls)
        time.sleep(0.2)  # the callers go on after the parks (the next call relaunches)
        after = sum(busy.calls)
    assert not busy.errors, busy.errors[:2]
    worst = max(t for _, t in log)
    print(f"user pinned-memory calls beside the busy worker: {len(log)} in {t_all:.2f} s, worst {worst * 1e3:.1f} ms")
    assert t_all < STREAM_BOUND_S, log
    assert after > before
    st = enc.worker_stats()
    assert st["served"] > 0 and st["launches"] >= 2, st  # parked and relaunched
    enc.worker_stop()


def test_worker_stop_start_while_calling(gpu):
    """stop and restart while 4 threads call.  A call
    that loaded the worker before the stop is declined (never served by a
    launch whose mailboxes are being freed); every result is exact."""
    enc = ia.New(K, P)
    enc.worker_start(nslots=4)
    with _Busy(enc) as busy:
        for r in range(12):
            enc.worker_stop()
            time.sleep(0.005)
            enc.worker_start(nslots=2 + r % 3, idle_us=2000 if r % 2 else 0)
            time.sleep(0.02)
    assert not busy.errors, busy.errors[:2]
    assert sum(busy.calls) > 100
    enc.worker_stop()
    # after the last stop: the stream path, exact
    full = _full(K, P, 103, 99)
    sh = [full[j].copy() if j < K else np.zeros(103, np.uint8) for j in range(N)]
    assert enc.EncodeVerify(sh)
    assert np.array_equal(sh[K], full[K])


def test_worker_two_contexts_one_stops(gpu):
    """Two contexts with workers on one device: stopping one (its pinned
    mailboxes are freed) must not wait for the other, which stays busy."""
    a, b = ia.New(K, P), ia.New(K, P)
    a.worker_start(nslots=4)
    b.worker_start(nslots=4)
    with _Busy(b):
        full = _full(K, P, 103, 5)
        sh = [full[j].copy() if j < K else np.zeros(103, np.uint8) for j in range(N)]
        assert a.EncodeVerify(sh)
        t0 = time.monotonic()
        a.worker_stop()
        dt = time.monotonic() - t0
    assert dt < 2.0, dt
    b.worker_stop()


def test_retired_frees_stay_bounded(gpu):
    """while a worker kernel is resident, the library's
    own frees (staging buffers that grew, contexts destroyed) are held back
    so they never wait for it — and what is held stays bounded: past
    kKeptCap (256 MiB) the workers are parked and everything held is freed
    (devmem.cpp relieve_retired).  Once no worker kernel is resident, the
    next free lets go of everything held; frees are held only while a kernel
    is resident, not merely while a worker is started."""
    import ctypes
    import gc
    cap = 256 << 20
    gc.collect()
    enc = ia.New(K, P)
    # a long idle exit (1 s): the kernel stays resident through the GIL gaps
    # of this thread's own work, so every destroy below happens beside it
    enc.worker_start(nslots=8, idle_us=1000000)
    L = ia._lib.load()
    peak = 0
    d0 = ia.retired_stats()["deferred"]
    with _Busy(enc) as busy:
        assert not busy.errors, busy.errors[:2]
        for i in range(10):
            c = ia.New(K, P)  # its staging grows to ~2 x 29 MB, freed (held) at destroy
            for size in (4 << 20, 24 << 20):
                obj = rn.splitmix64_bytes(0xB0B, 10 * i + size, size)
                sh = c.Split(obj)
                c.Encode(sh)
                e, want = oracle.encode(K, P, [bytes(s) for s in sh[:K]] + [bytes(len(sh[0]))] * P)
                assert e == 0 and all(np.array_equal(sh[K + r], want[K + r]) for r in range(P))
            del c  # (rsgpu_destroy: no reference cycle holds it)
            st = ia.retired_stats()
            peak = max(peak, st["bytes"])
            assert st["bytes"] <= cap + (128 << 20), st  # the cap plus one context's buffers
        held = ia.retired_stats()["deferred"] - d0
    assert not busy.errors, busy.errors[:2]
    assert held > 0  # the kernel was resident: frees were held back
    assert peak >= 32 << 20  # ... including the destroyed contexts' staging images
    # the busy callers stopped: the kernel leaves after idle_us (1 s); the
    # next free finds none resident and lets go of everything held
    time.sleep(1.5)
    p = ctypes.c_void_p()
    assert L.rsgpu_host_alloc(1 << 16, ctypes.byref(p)) == 0
    assert L.rsgpu_host_free(p) == 0
    st = ia.retired_stats()
    print(f"held back while resident: {held} frees, peak {peak >> 20} MiB; after idle: {st}")
    assert st["count"] == 0 and st["bytes"] == 0, st
    # started but idle: a free runs at once (nothing is held)
    d1 = st["deferred"]
    c = ia.New(K, P)
    sh = c.Split(rn.splitmix64_bytes(0xB0C, 1, 1 << 20))
    c.Encode(sh)
    del c
    gc.collect()
    st = ia.retired_stats()
    assert st["deferred"] == d1 and st["count"] == 0, st
    enc.worker_stop()


def test_user_free_held_is_counted_by_its_size(gpu):
    """a user's rsgpu_host_free held back while a worker kernel
    is resident counts toward the kept-bytes bound by the allocation's size
    (from the library's pin table; the runtime's address-range query does not
    know every hipHostMalloc'd pointer), so the bound also covers user frees."""
    import ctypes
    enc = ia.New(K, P)
    enc.worker_start(nslots=8, idle_us=1000000)
    L = ia._lib.load()
    nbytes = 24 << 20
    with _Busy(enc) as busy:
        time.sleep(0.05)  # the callers keep the kernel resident
        p = ctypes.c_void_p()
        assert L.rsgpu_host_alloc(nbytes, ctypes.byref(p)) == 0
        before = ia.retired_stats()
        assert L.rsgpu_host_free(p) == 0
        after = ia.retired_stats()
    assert not busy.errors, busy.errors[:2]
    assert after["deferred"] == before["deferred"] + 1, (before, after)  # held back: the kernel was resident
    assert after["bytes"] - before["bytes"] >= nbytes, (before, after)   # ... and counted by its size
    time.sleep(1.5)  # the kernel leaves after idle_us; the next free lets go of everything
    q = ctypes.c_void_p()
    assert L.rsgpu_host_alloc(1 << 16, ctypes.byref(q)) == 0
    assert L.rsgpu_host_free(q) == 0
    st = ia.retired_stats()
    assert st["count"] == 0 and st["bytes"] == 0, st
    enc.worker_stop()
