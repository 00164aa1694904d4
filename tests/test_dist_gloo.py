"""World-size-2, 3 and 8 CPU rehearsal of bench.py's multi-rank path with the
gloo backend: object sharding, the all_reduce start/finish barrier and the
MAX-over-ranks timing.  The per-rank step here codes its
objects with the CPU oracle so the partition can be checked end to end (a
checksum of checksums equals the single-process result); on GPUs the same
harness runs the HIP path with RCCL."""
import os
import socket
import time

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, nobj_total, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    import bench
    import oracle
    from oracle import rs_numpy as rn
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dctx = bench.DistCtx(world, rank, "cpu")
        start, count = bench.shard_objects(nobj_total, rank, world)
        e, m = oracle.build_matrix(10, 2)
        S = 1000
        digests = []

        def step(i):
            digests.clear()
            for o in range(start, start + count):
                data = rn.splitmix64_bytes(0x1F1C, o, 10 * S).reshape(10, S)
                par = oracle.code_fast(m[10:], [data[c] for c in range(10)])
                digests.append(int(np.bitwise_xor.reduce(np.concatenate(par).view(np.uint64))))
            time.sleep(0.05 * (rank + 1))  # rank skew: max-over-ranks must see the slowest

        el = bench.timed_run(step, steps=2, warmup=1, sync=lambda: None, dctx=dctx)
        total = dctx.sum(count)
        gathered = dctx.gather(float(rank) + 0.5)  # per-rank roofline fractions (bench.py)
        x = 0
        for d in digests:
            x ^= d
        q.put((rank, el, total, start, count, x, gathered))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_gloo_object_per_rank(world):
    nobj = 11
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, nobj, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    res.sort()
    els = {r[1] for r in res}
    assert len(els) == 1                       # every rank reports the same MAX
    assert min(els) >= 2 * 0.05 * world         # >= the slowest rank's two steps
    assert all(r[2] == nobj for r in res)       # all objects accounted exactly once
    assert all(r[6] == [i + 0.5 for i in range(world)] for r in res)  # gather: rank order
    spans = [(r[3], r[4]) for r in res]
    assert spans[0][0] == 0 and sum(c for _, c in spans) == nobj
    assert all(spans[i][0] + spans[i][1] == spans[i + 1][0] for i in range(world - 1))
    # checksum of checksums == single-process coding of all objects
    import oracle
    from oracle import rs_numpy as rn
    e, m = oracle.build_matrix(10, 2)
    want = 0
    for o in range(nobj):
        data = rn.splitmix64_bytes(0x1F1C, o, 10 * 1000).reshape(10, 1000)
        par = oracle.code_fast(m[10:], [data[c] for c in range(10)])
        want ^= int(np.bitwise_xor.reduce(np.concatenate(par).view(np.uint64)))
    got = 0
    for r in res:
        got ^= r[5]
    assert got == want


def test_shard_objects_cover_all():
    import bench
    for n in (0, 1, 7, 1024):
        for world in (1, 2, 3, 8):
            spans = [bench.shard_objects(n, r, world) for r in range(world)]
            assert sum(c for _, c in spans) == n
            assert max(c for _, c in spans) - min(c for _, c in spans) <= 1


def _one_rank(port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    import bench
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        d = bench.DistCtx(1, 0, "cpu", force=True)
        el = bench.timed_run(lambda i: time.sleep(0.01), steps=2, warmup=1, sync=lambda: None, dctx=d)
        q.put((el, d.sum(7), d.gather(0.25), d.calls))
    finally:
        dist.destroy_process_group()


def test_forced_collectives_at_world_one():
    """--collectives: DistCtx issues its collectives over a one-rank process
    group (the RCCL path of BENCH config 4 on a one-GPU box), same results
    as the short-circuited form."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_one_rank, args=(_free_port(), q))
    p.start()
    el, s, g, calls = q.get(timeout=120)
    p.join(60)
    assert p.exitcode == 0
    assert el >= 0.02 and s == 7 and g == [0.25]
    assert calls == 2 + 1 + 1 + 1  # timed_run's two barriers and MAX, the SUM, the gather
    import bench
    d0 = bench.DistCtx(1, 0, "cpu")
    assert not d0.on and d0.max(1.5) == 1.5 and d0.gather(2.0) == [2.0] and d0.calls == 0
