"""World-size 2 on the HIP path, on the one-GPU test box: bench.py's
multi-rank harness (DistCtx barrier + MAX-over-ranks timing, shard_objects)
driving librsgpu.so in each rank, with the ranks sharing cuda:0 over gloo
(RCCL refuses two ranks on one GPU).  BASELINE config 4 is the same harness
with one GPU per rank over RCCL (client/client.go:47-59 fans an object's
shards out from one process; here objects never cross ranks).

* test_gloo_ranks_hip_path: each rank encodes + erases + fused-decodes its
  own object range (strong split of one batch) with the HIP kernels inside
  bench.timed_run, then checks every object against the oracle; the parent
  checks the partition and a checksum of checksums.
* test_bench_two_ranks_shared_gpu: bench.py itself under torch.distributed.run
  with 2 ranks: one JSON line with n_gpus 2, the gloo backend named in the
  parallelism label, and the bit-exact work check of every rank's batch."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SEED = 0x1F1C


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _hip_worker(rank, world, port, nobj_total, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist

    import bench
    import infinicache_amd as ia
    import oracle
    from oracle import rs_numpy as rn
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        assert ia.device_ok(0)
        dctx = bench.DistCtx(world, rank, dev)
        start, count = bench.shard_objects(nobj_total, rank, world)
        k, p = 10, 2
        n = k + p
        S, pitch = 5003, 5120
        host = np.zeros((count, n, pitch), np.uint8)
        for j, o in enumerate(range(start, start + count)):
            host[j, :k, :S] = rn.splitmix64_bytes(SEED, 2000 + o, k * S).reshape(k, S)
        buf = torch.from_numpy(host).to(dev)
        bad = torch.full((count,), 3, dtype=torch.int32, device=dev)
        lost = (0, 5)
        present = [i not in lost for i in range(n)]
        enc = ia.New(k, p, device=0)
        stream = torch.cuda.current_stream(dev)

        def step(i):
            enc.encode_dev(buf, S, pitch, n * pitch, count, stream)
            buf[:, list(lost), :] = 0xEE  # the Get lost data shards 0 and 5
            enc.decode_dev(buf, present, S, pitch, n * pitch, count, bad, stream)

        el = bench.timed_run(step, steps=3, warmup=1, sync=lambda: torch.cuda.synchronize(dev), dctx=dctx)
        total = dctx.sum(count)
        out = buf.cpu().numpy()
        e, m = oracle.build_matrix(k, p)
        exact = not bool(bad.any())
        x = 0
        for j in range(count):
            par = oracle.apply(m[k:], [host[j, c, :S] for c in range(k)])
            exact &= all(np.array_equal(out[j, k + r, :S], par[r]) for r in range(p))
            exact &= all(np.array_equal(out[j, c, :S], host[j, c, :S]) for c in range(k))
            x ^= int(np.bitwise_xor.reduce(np.concatenate(par).view(np.uint8).astype(np.uint64)))
        q.put((rank, el, total, start, count, bool(exact), x, enc.device_calls()))
    finally:
        dist.destroy_process_group()


def test_gloo_ranks_hip_path(gpu):
    import torch.multiprocessing as mp

    import oracle
    from oracle import rs_numpy as rn
    world, nobj = 2, 9
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_hip_worker, args=(r, world, port, nobj, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = sorted(q.get(timeout=150) for _ in range(world))
    finally:
        for p in procs:
            p.join(60)
            if p.exitcode is None:
                p.kill()
    assert all(p.exitcode == 0 for p in procs)
    assert len({r[1] for r in res}) == 1          # one MAX over ranks
    assert all(r[2] == nobj for r in res)
    assert all(r[5] for r in res), "a rank's HIP output differs from the oracle"
    assert all(r[7][0] > 0 for r in res)          # the HIP library ran in each rank
    spans = [(r[3], r[4]) for r in res]
    assert spans[0][0] == 0 and spans[0][0] + spans[0][1] == spans[1][0] and sum(c for _, c in spans) == nobj
    e, m = oracle.build_matrix(10, 2)
    want = 0
    for o in range(nobj):
        d = rn.splitmix64_bytes(SEED, 2000 + o, 10 * 5003).reshape(10, 5003)
        par = oracle.apply(m[10:], [d[c] for c in range(10)])
        want ^= int(np.bitwise_xor.reduce(np.concatenate(par).view(np.uint8).astype(np.uint64)))
    got = 0
    for r in res:
        got ^= r[6]
    assert got == want


def test_bench_two_ranks_shared_gpu(gpu, tmp_path):
    env = dict(os.environ, BENCH_DIST_BACKEND="gloo", BENCH_SHARE_GPU="1", PYTHONUNBUFFERED="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "2",
           "--batch", "48", "--cpu-seconds", "2"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["batch_per_gpu"] == 48
    assert "gloo" in out["config"]["parallelism"] and "sharing one GPU" in out["config"]["parallelism"]
    assert out["decode_check"] == "bit-exact"
    assert out["work_check"]["encode"]["result"] == "bit-exact"
    assert out["value"] > 0
    # the CPU port is timed beside the GPU at every world size (VERDICT r03
    # next #3): the driver's N = 2/4/8 lines carry it too
    cpu = out["cpu_baseline"]
    assert cpu is not None and cpu["kind"] == "port" and cpu["value"] > 0 and cpu["cores"] >= 1
    assert "bit-exact vs GPU" in cpu["sample"] and cpu["sample"].endswith(": True"), cpu["sample"]
    assert out["roofline"]["traffic_source"].startswith(("committed profile", "none"))
    assert out["roofline"]["frac_per_rank"] and len(out["roofline"]["frac_per_rank"]) == 2
    # strong scaling beside the weak line: the 48-object
    # batch split 24 + 24 over the two ranks, every object coded once
    st = out["strong_scaling"]
    assert st["batch_total"] == 48 and st["objects_coded"] == 48 and st["objects_per_rank"] == [24, 24]
    assert st["value"] > 0 and st["ms_per_step"] > 0


def test_bench_four_ranks_shared_gpu_uneven(gpu):
    """N = 4 of bench.py's multi-rank path on the one-GPU box (gloo, ranks
    sharing cuda:0), with a batch that does not divide evenly: the strong
    block splits 50 objects 13 + 13 + 12 + 12 (shard_objects), every object
    coded once; each rank's weak batch is checked bit-exact; the per-rank
    roofline has 4 entries."""
    env = dict(os.environ, BENCH_DIST_BACKEND="gloo", BENCH_SHARE_GPU="1", PYTHONUNBUFFERED="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "4",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "4", "--steps", "3", "--warmup", "2",
           "--batch", "50", "--cpu-seconds", "2"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 4 and out["config"]["batch_per_gpu"] == 50
    assert all(v["result"] == "bit-exact" for v in out["work_check"].values())
    assert len(out["roofline"]["frac_per_rank"]) == 4 and min(out["roofline"]["frac_per_rank"]) > 0
    st = out["strong_scaling"]
    assert st["batch_total"] == 50 and st["objects_coded"] == 50
    assert st["objects_per_rank"] == [13, 13, 12, 12]
    assert out["work_check_ranks"] == [1, 1, 1, 1]
    assert out["cpu_baseline"] is not None and out["cpu_baseline"]["sample"].endswith(": True")


def test_bench_one_rank_rccl(gpu):
    """BASELINE config 4's collectives on the one-GPU box: bench.py under
    torch.distributed.run with ONE rank, the default nccl (RCCL) backend and
    the collectives forced on at world size 1: init_process_group with
    device_id, the device-tensor barrier, the float64 MAX-reduce, the int64
    SUM and the one-hot gather all execute over RCCL."""
    env = dict(os.environ, PYTHONUNBUFFERED="1")
    env.pop("BENCH_DIST_BACKEND", None)
    env.pop("BENCH_SHARE_GPU", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "1", "--collectives", "--steps", "5", "--warmup", "3",
           "--batch", "64", "--cpu-seconds", "2", "--no-pmc"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 1 and out["config"]["batch_per_gpu"] == 64
    assert "RCCL all_reduce barrier only" in out["config"]["parallelism"], out["config"]["parallelism"]
    # weak and strong regions: 2 barriers + MAX each, a SUM each, the strong
    # block's gather and the roofline gather
    assert out["collectives_issued"] >= 8
    assert out["decode_check"] == "bit-exact"
    assert all(v["result"] == "bit-exact" for v in out["work_check"].values())
    assert len(out["roofline"]["frac_per_rank"]) == 1 and out["roofline"]["frac_per_rank"][0] > 0
    st = out["strong_scaling"]
    assert st["objects_coded"] == 64 and st["objects_per_rank"] == [64]
    cpu = out["cpu_baseline"]
    assert cpu is not None and cpu["kind"] == "port" and cpu["value"] > 0
    assert cpu["sample"].endswith(": True"), cpu["sample"]
    dst = os.environ.get("BENCH_RCCL_JSON")
    if dst:  # the committed evidence (profiles/r05_bench_rccl_1rank.json)
        with open(dst, "w") as f:
            f.write(lines[0] + "\n")
