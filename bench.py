"""Benchmark: RS(10+2) encode+decode GiB/s, device-resident, 1 MiB objects.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload encdec|enc|dec4]
    torchrun --nproc-per-node N bench.py --gpus N ...      (one rank per GPU)

A step = one pass of the hot path over one batch: encode the batch (parity
rows <- M x data rows, Client.encode / ecRedis.go:390) then decode it
(reconstruct data shards {0, 5} from the first 10 present shards, the fused
Client.decode / ecRedis.go:406-420 with the proxy's first-d rule: exactly k
shards arrive).  Each rank owns its own batch of 1024 objects (object-per-
rank, weak scaling); RCCL all_reduce of one int is the start/finish barrier.
value = object bytes x ops of all ranks / max-over-ranks time.  At N > 1 (or
with --collectives) the same line carries a `strong_scaling` block: the
workload's one batch split over the ranks (shard_objects), timed after the
weak region with the same barriers.

Prints ONE JSON line (rank 0) with roofline (HIP-event kernel timing;
`traffic` measured in this run by two rocprofv3 --pmc child passes at N = 1,
else the committed summary, `traffic_source` says which) and cpu_baseline
(the oracle's AVX-512/AVX2 port of the Go path, timed on this host by rank 0
at every world size, after the timed region).

--collectives (or BENCH_COLLECTIVES=1) issues the collectives at world size 1
too: under `torch.distributed.run --nproc-per-node 1` that is one RCCL rank
running the barrier, MAX-reduce and gather of the multi-GPU path.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

GiB = float(1 << 30)
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)

WORKLOADS = {
    # name: (k, p, object bytes, batch per GPU, erased rows for decode, ops)
    "encdec": dict(k=10, p=2, nbytes=1 << 20, batch=1024, lost=(0, 5), ops=("encode", "decode"),
                   desc="RS(10+2) encode+decode, 1 MiB objects, batch 1024/GPU, device-resident"),
    # the same with a realistic Get batch: every object lost its own random
    # pair of shards (proxy first-d rule), decoded in one mixed-pattern launch
    "encdec_mixed": dict(k=10, p=2, nbytes=1 << 20, batch=1024, lost=(0, 5), ops=("encode", "decode"),
                         mixed=True,
                         desc="RS(10+2) encode+decode, 1 MiB objects, batch 1024/GPU, per-object "
                              "random erasure pair (device-resident present masks, patterns resolved on the GPU)"),
    # small objects (4 KiB): rows of 26 vectors, packed 9 objects per
    # workgroup; pitch = S rounded to 16 B (no padding traffic)
    "small": dict(k=10, p=2, nbytes=4 << 10, batch=256 << 10, lost=(0, 5), ops=("encode", "decode"),
                  palign=16,
                  desc="RS(10+2) encode+decode, 4 KiB objects, batch 262144/GPU, device-resident"),
    # the reference's own example object (client/example/main.go:15,26): 1 KiB,
    # S = 103; palign: row pitch rounded to 16 (112), 4 (104) or 1 (103,
    # byte-packed rows; the object stride is n * pitch either way)
    "small1k": dict(k=10, p=2, nbytes=1 << 10, batch=1 << 20, lost=(0, 5), ops=("encode", "decode"),
                    palign=16, desc="RS(10+2) encode+decode, 1 KiB objects, batch 1048576/GPU, pitch 112"),
    "small1k_p4": dict(k=10, p=2, nbytes=1 << 10, batch=1 << 20, lost=(0, 5), ops=("encode", "decode"),
                       palign=4, desc="RS(10+2) encode+decode, 1 KiB objects, batch 1048576/GPU, pitch 104"),
    "small1k_p1": dict(k=10, p=2, nbytes=1 << 10, batch=1 << 20, lost=(0, 5), ops=("encode", "decode"),
                       palign=1, desc="RS(10+2) encode+decode, 1 KiB objects, batch 1048576/GPU, "
                                      "byte-packed rows (pitch 103)"),
    # rows padded to whole 64/128-B sectors: every row piece is read and
    # written as whole sectors (no partial-sector writes), at the cost of
    # the padding bytes
    "small1k_p128": dict(k=10, p=2, nbytes=1 << 10, batch=1 << 20, lost=(0, 5), ops=("encode", "decode"),
                         palign=128, desc="RS(10+2) encode+decode, 1 KiB objects, batch 1048576/GPU, pitch 128"),
    "small_p64": dict(k=10, p=2, nbytes=4 << 10, batch=256 << 10, lost=(0, 5), ops=("encode", "decode"),
                      palign=64, desc="RS(10+2) encode+decode, 4 KiB objects, batch 262144/GPU, pitch 448"),
    "small_p128": dict(k=10, p=2, nbytes=4 << 10, batch=256 << 10, lost=(0, 5), ops=("encode", "decode"),
                       palign=128, desc="RS(10+2) encode+decode, 4 KiB objects, batch 262144/GPU, pitch 512"),
    # shard-major batches ([shard][object]: shard i of all objects back to
    # back, as InfiniCache ships shard i to Lambda node i): the batch is coded
    # as one object per shard row, whatever the object size
    "small1k_sm": dict(k=10, p=2, nbytes=1 << 10, batch=1 << 20, lost=(0, 5), ops=("encode", "decode"),
                       shard_major=True, oalign=1,
                       desc="RS(10+2) encode+decode, 1 KiB objects, batch 1048576/GPU, shard-major "
                            "(pieces back to back, S = 103)"),
    "small1k_sm_mixed": dict(k=10, p=2, nbytes=1 << 10, batch=1 << 20, lost=(0, 5), ops=("encode", "decode"),
                             shard_major=True, oalign=16, mixed=True,
                             desc="RS(10+2) encode+decode, 1 KiB objects, batch 1048576/GPU, shard-major "
                                  "(16-B aligned pieces), per-object random erasure pair (device-resident "
                                  "present masks)"),
    # the mixed 1 KiB shape as the library lays it out (rsgpu_shardmajor_layout:
    # whole 128-B line pieces for S = 103)
    "small1k_sm_mixed_a128": dict(k=10, p=2, nbytes=1 << 10, batch=1 << 20, lost=(0, 5), ops=("encode", "decode"),
                                  shard_major=True, oalign="library", mixed=True,
                                  desc="RS(10+2) encode+decode, 1 KiB objects, batch 1048576/GPU, shard-major "
                                       "in rsgpu_shardmajor_layout's geometry (128-B pieces: one line each), "
                                       "per-object random erasure pair (device-resident present masks)"),
    "small_sm": dict(k=10, p=2, nbytes=4 << 10, batch=256 << 10, lost=(0, 5), ops=("encode", "decode"),
                     shard_major=True, oalign=1,
                     desc="RS(10+2) encode+decode, 4 KiB objects, batch 262144/GPU, shard-major"),
    "small_mixed": dict(k=10, p=2, nbytes=4 << 10, batch=256 << 10, lost=(0, 5), ops=("encode", "decode"),
                        palign=16, mixed=True,
                        desc="RS(10+2) encode+decode, 4 KiB objects, batch 262144/GPU, per-object "
                             "random erasure pair (device-resident present masks, patterns resolved on the GPU)"),
    # upstream Get semantics, unfused (reported separately, not
    # the headline): Reconstruct, then a full Verify pass over all k+p rows
    "encdec_upstream": dict(k=10, p=2, nbytes=1 << 20, batch=1024, lost=(0, 5), ops=("encode", "decode"),
                            upstream_get=True,
                            desc="RS(10+2) encode+decode, 1 MiB objects, batch 1024/GPU, decode as upstream "
                                 "Client.decode: Reconstruct then a separate full Verify pass"),
    "enc": dict(k=10, p=2, nbytes=1 << 20, batch=1024, lost=(), ops=("encode",),
                desc="RS(10+2) encode, 1 MiB objects, batch 1024/GPU, device-resident"),
    # a healthy RS(10+4) Get receives exactly k = 10 bodies (proxy first-d
    # rule): data {0,5} and parity {12,13} absent; ReconstructData rebuilds
    # the 2 data shards from the 10 survivors
    # a wide code (K > 16: the generic kernel, inputs coded in triples);
    # the Get receives k = 20 bodies, data {0,5} and parity {22,23} absent
    "wide": dict(k=20, p=4, nbytes=1 << 20, batch=1024, lost=(0, 5), absent=(22, 23),
                 ops=("encode", "decode"),
                 desc="RS(20+4) encode+decode, 1 MiB objects, batch 1024/GPU, device-resident "
                      "(generic kernel)"),
    "dec4": dict(k=10, p=4, nbytes=4 << 20, batch=512, lost=(0, 5), absent=(12, 13),
                 ops=("decode",), data_only=True,
                 desc="RS(10+4) ReconstructData, data shards {0,5} missing (10 of 14 present), "
                      "4 MiB objects, batch 512/GPU"),
    # BASELINE config 3 as the reference's Client.decode runs it
    # (client/ecRedis.go:404-427): with 2 data shards lost, 12 of 14 shards
    # are present, so the Get rebuilds {0,5} from the first 10 present and
    # verifies the whole object, which checks the 2 extra parity shards
    #   dec4_get:      one fused launch: 12 rows in, 2 rows written, 2 parity
    #                  rows checked in registers (rsgpu_decode_dev)
    #   dec4_upstream: upstream's passes as they are: Reconstruct (10 rows in,
    #                  2 written), then a full Verify (14 rows in, 4 checked)
    "dec4_get": dict(k=10, p=4, nbytes=4 << 20, batch=512, lost=(0, 5), ops=("decode",),
                     desc="RS(10+4) Get as Client.decode runs it: 12 of 14 shards present, data {0,5} "
                          "rebuilt from the first 10 and the 2 extra parity shards verified, fused in one "
                          "pass, 4 MiB objects, batch 512/GPU"),
    "dec4_upstream": dict(k=10, p=4, nbytes=4 << 20, batch=512, lost=(0, 5), ops=("decode",),
                          upstream_get=True,
                          desc="RS(10+4) Get as Client.decode runs it, unfused: Reconstruct of data {0,5} "
                               "from the first 10 of 12 present shards, then a separate full Verify pass "
                               "over all 14 rows, 4 MiB objects, batch 512/GPU"),
}
METRICS = {
    "encdec": "RS(10+2) encode+decode GiB/s (device-resident), 1 MB objects, 1/2/4/8 GPU",
    "encdec_mixed": "RS(10+2) encode+decode GiB/s (device-resident, mixed erasure patterns), 1 MB objects",
    "enc": "RS(10+2) encode GiB/s (device-resident), 1 MB objects",
    "encdec_upstream": "RS(10+2) encode+decode GiB/s (device-resident, unfused Reconstruct+Verify Get), 1 MB objects",
    "small": "RS(10+2) encode+decode GiB/s (device-resident), 4 KiB objects",
    "wide": "RS(20+4) encode+decode GiB/s (device-resident), 1 MB objects",
    "small_mixed": "RS(10+2) encode+decode GiB/s (device-resident, mixed erasure patterns), 4 KiB objects",
    "small1k": "RS(10+2) encode+decode GiB/s (device-resident), 1 KiB objects",
    "small1k_sm": "RS(10+2) encode+decode GiB/s (device-resident, shard-major batch), 1 KiB objects",
    "small1k_sm_mixed": "RS(10+2) encode+decode GiB/s (device-resident, shard-major batch, mixed erasure "
                        "patterns), 1 KiB objects",
    "small1k_sm_mixed_a128": "RS(10+2) encode+decode GiB/s (device-resident, shard-major batch, mixed erasure "
                             "patterns), 1 KiB objects",
    "small_sm": "RS(10+2) encode+decode GiB/s (device-resident, shard-major batch), 4 KiB objects",
    "small1k_p4": "RS(10+2) encode+decode GiB/s (device-resident), 1 KiB objects",
    "small1k_p1": "RS(10+2) encode+decode GiB/s (device-resident), 1 KiB objects",
    "small1k_p128": "RS(10+2) encode+decode GiB/s (device-resident), 1 KiB objects",
    "small_p64": "RS(10+2) encode+decode GiB/s (device-resident), 4 KiB objects",
    "small_p128": "RS(10+2) encode+decode GiB/s (device-resident), 4 KiB objects",
    "dec4": "RS(10+4) decode (2 missing data shards) GiB/s, 4 MB objects",
    "dec4_get": "RS(10+4) decode (2 missing data shards, Client.decode Reconstruct+Verify fused) GiB/s, "
                "4 MB objects",
    "dec4_upstream": "RS(10+4) decode (2 missing data shards, Client.decode Reconstruct then Verify, "
                     "unfused) GiB/s, 4 MB objects",
}


def pass_symbol(K, R, KI, S, shard_major=False):
    """Kernel a uniform K-input, R-row pass of the library runs (KI trailing
    identity inputs, shard length S): gf_apply_tri for the shapes
    infinicache_amd/csrc/gf_kernels.hip tri_shape lists, on rows longer than
    128 16-B vectors of an object-major batch; gf_apply_kernel otherwise."""
    tri = {(12, 4, 2), (11, 4, 1), (10, 4, 0), (14, 4, 4), (13, 3, 3), (16, 4, 4)}
    if (K, R, KI) in tri and (S + 15) // 16 * 2 > 256 and not shard_major:
        return f"gf_apply_tri<{K},{R}>"
    return f"gf_apply_kernel<{K},{R}>"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_baseline(w, sample, gpu_sample, m, inv_rows, budget_s=10.0, threads=16, windows=3, fused_checks=0):
    """Time the oracle's port of the Go path (upstream galMulAVX2Xor /
    codeSomeShardsAvx512 SIMD coders) over a bounded sample laid out like the
    GPU batch, bit-compare with the GPU output.  Headline form: object-
    parallel (one object per task, as many concurrent EcSet/EcGet calls would
    run) on `threads` threads (the box's cgroup share) and on 1 thread, each
    the MEDIAN of `windows` timing windows (1-core and all-core);
    the per-object codeSomeShardsP split form (maxGoroutines 32, minSplitSize
    1024, client/example/main.go:22) is timed beside it for reference.

    A decode that verifies (the Get of dec4_get / *_upstream: 12 of 14 shards
    present, or upstream's separate Verify) is timed the way the Go path runs
    it: Reconstruct, then Verify re-encoding every parity row from the data
    rows and comparing (client/ecRedis.go:414-420); with fused_checks > 0 the
    fused form (the extra shards checked from the survivors in the decode's
    own pass) is timed beside it."""
    import ctypes

    import oracle
    from oracle import rs_numpy as rn
    k, p = w["k"], w["p"]
    n = k + p
    S = (w["nbytes"] + k - 1) // k
    ns, _, pitch = sample.shape
    lost = list(w["lost"])
    present = [i for i in range(n) if i not in lost and i not in w.get("absent", ())]
    surv = present[:k]
    base = sample.reshape(-1)
    verifies = "decode" in w["ops"] and (w.get("upstream_get") or fused_checks > 0)
    extras = present[k:]
    fused_coef = None
    if fused_checks > 0:  # check rows of the extra shards, over the survivors
        fused_coef = np.concatenate([inv_rows, rn.matmul(m[extras], rn.invert(m[surv]))])
    verified = [True]

    def one_pass(nt, nobj, form="upstream"):
        if "encode" in w["ops"]:
            oracle.code_batch(m[k:], list(range(k)), list(range(k, n)), base, n * pitch, pitch, S,
                              nobj, nthreads=nt)
        if "decode" in w["ops"]:
            if form == "fused":  # rebuilt rows written, extra shards compared, one pass per object
                oracle.code_batch(inv_rows, surv, lost, base, n * pitch, pitch, S, nobj, nthreads=nt)
                ok = oracle.verify_batch(fused_coef[len(lost):], surv, extras, base, n * pitch, pitch, S,
                                         nobj, nthreads=nt)
                verified[0] &= bool(ok.all())
                return
            oracle.code_batch(inv_rows, surv, lost, base, n * pitch, pitch, S, nobj, nthreads=nt)
            if verifies:  # upstream Verify: all parity re-encoded from the data rows, compared
                ok = oracle.verify_batch(m[k:], list(range(k)), list(range(k, n)), base, n * pitch, pitch,
                                         S, nobj, nthreads=nt)
                verified[0] &= bool(ok.all())

    def rate(nt, nobj, secs, form="upstream"):
        """median GiB/s over `windows` windows of ~secs each"""
        one_pass(nt, nobj, form)  # warm the pool and the pages
        vals = []
        for _ in range(windows):
            reps, t0 = 0, time.perf_counter()
            while True:
                one_pass(nt, nobj, form)
                reps += 1
                el = time.perf_counter() - t0
                if el >= secs:
                    break
            vals.append(nobj * reps * w["nbytes"] * len(w["ops"]) / el / GiB)
        return float(np.median(vals)), vals

    all_v, all_w = rate(threads, ns, budget_s * 0.5 / windows)
    one_v, one_w = rate(1, ns, budget_s * 0.3 / windows)  # same sample: beyond the host's L3
    fused_v = None
    if fused_coef is not None:
        fused_v, _ = rate(threads, ns, budget_s * 0.2 / windows, form="fused")
    exact = bool(np.array_equal(sample[:, :, :S], gpu_sample[:, :, :S])) and verified[0]
    if "encode" in w["ops"] and "decode" in w["ops"]:
        # the encode pass above needs the data rows, so the rows the GPU
        # rebuilt are checked by a separate CPU decode: erase them again and
        # rebuild them on the CPU from the GPU's survivors
        dsample = gpu_sample.copy()
        dsample[:, lost] = 0
        oracle.code_batch(inv_rows, surv, lost, dsample.reshape(-1), n * pitch, pitch, S, ns, nthreads=threads)
        exact = exact and bool(np.array_equal(dsample[:, :, :S], gpu_sample[:, :, :S]))
    # per-object codeSomeShardsP form, ~budget/5 s
    sreps, t1 = 0, time.perf_counter()
    while time.perf_counter() - t1 < budget_s / 5:
        for o in range(ns):
            if "encode" in w["ops"]:
                oracle.code_fast(m[k:], [sample[o, c, :S] for c in range(k)], nthreads=threads,
                                 max_goroutines=32)
            if "decode" in w["ops"]:
                oracle.code_fast(inv_rows, [sample[o, c, :S] for c in surv], nthreads=threads,
                                 max_goroutines=32)
                if verifies:
                    oracle.code_fast(m[k:], [sample[o, c, :S] for c in range(k)], nthreads=threads,
                                     max_goroutines=32)
        sreps += 1
    split_val = ns * sreps * w["nbytes"] * len(w["ops"]) / (time.perf_counter() - t1) / GiB
    # the host's one-thread memory rate beside it: the 1-core coder figure
    # follows it from box to box (r02 runs: 17-36 GiB/s on the same code)
    src = np.ones(1 << 28, np.uint8)
    dst = np.empty_like(src)
    np.copyto(dst, src)
    creps, t2 = 0, time.perf_counter()
    while time.perf_counter() - t2 < 0.5:
        np.copyto(dst, src)
        creps += 1
    copy_gbps = 2 * src.nbytes * creps / (time.perf_counter() - t2) / 1e9
    del src, dst
    L = oracle.lib()
    L.orc_cpu_isa.restype = ctypes.c_char_p
    isa = L.orc_cpu_isa().decode()
    cpu_model = ""
    try:
        cpu_model = next(l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo")
                         if l.startswith("model name"))
    except Exception:
        pass
    return {
        "value": round(all_v, 3),
        "unit": "GiB/s",
        "cores": threads,
        "kind": "port",
        "windows_GiBps": [round(v, 2) for v in all_w],
        "one_core": {"value": round(one_v, 3), "cores": 1, "windows_GiBps": [round(v, 2) for v in one_w]},
        "per_object_split_form_GiBps": round(split_val, 3),
        **({"decode_form": "Reconstruct then Verify of all parity rows (the Go path, client/ecRedis.go:414-420)",
            "fused_form_GiBps": round(fused_v, 3) if fused_v is not None else None} if verifies else {}),
        "host_copy_GBps_1thread": round(copy_gbps, 1),
        "sample": f"{ns} x {w['nbytes'] >> 10} KiB objects ({' + '.join(w['ops'])}), object-parallel; value = "
                  f"median of {windows} windows on {threads} threads (the box's cgroup share), one_core = "
                  f"median of {windows} windows on 1 thread, same sample; {isa} coder "
                  f"(oracle/rs_oracle.c restating upstream's SIMD path; Go toolchain and "
                  f"klauspost/reedsolomon unavailable offline); per-object codeSomeShardsP split "
                  f"form {split_val:.2f} GiB/s; host CPU: {cpu_model}; bit-exact vs GPU (parity, and the rows "
                  f"the GPU rebuilt from garbage in the work check): {exact}",
    }


class DistCtx:
    """The only cross-rank traffic of the path: an all_reduce of one int as
    the start/finish barrier (RCCL over xGMI on GPUs, gloo on CPU) and one
    MAX-reduce of the elapsed time.  Objects never cross ranks.

    force: issue the collectives at world size 1 as well (a process group
    of one rank must exist), so the RCCL path runs on a one-GPU box."""

    def __init__(self, world, rank, device, force=False):
        self.world, self.rank, self.device = world, rank, device
        self.on = world > 1 or force
        self.calls = 0  # collectives issued (the 1-rank RCCL test checks them)

    def barrier(self):
        if self.on:
            import torch
            import torch.distributed as dist
            t = torch.ones(1, dtype=torch.int32, device=self.device)
            dist.all_reduce(t)
            self.calls += 1

    def max(self, x: float) -> float:
        if not self.on:
            return x
        import torch
        import torch.distributed as dist
        t = torch.tensor([x], dtype=torch.float64, device=self.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        self.calls += 1
        return float(t.item())

    def sum(self, x: int) -> int:
        if not self.on:
            return x
        import torch
        import torch.distributed as dist
        t = torch.tensor([x], dtype=torch.int64, device=self.device)
        dist.all_reduce(t)
        self.calls += 1
        return int(t.item())

    def gather(self, x: float) -> list:
        """Every rank's value of x, in rank order (a SUM-reduce of one-hot
        vectors: the same collective as the barrier, no payload besides)."""
        if not self.on:
            return [x]
        import torch
        import torch.distributed as dist
        t = torch.zeros(self.world, dtype=torch.float64, device=self.device)
        t[self.rank] = x
        dist.all_reduce(t)
        self.calls += 1
        return [float(v) for v in t.cpu()]


def shard_objects(nobj_total: int, rank: int, world: int):
    """Contiguous object range of `rank` for strong scaling (objects are
    independent units: object i's shards never leave its rank's GPU)."""
    base, rem = divmod(nobj_total, world)
    start = rank * base + min(rank, rem)
    return start, base + (1 if rank < rem else 0)


def timed_run(step, steps, warmup, sync, dctx: DistCtx):
    """W untimed warmup steps; barrier + sync; K timed steps; sync + barrier +
    sync; returns the MAX over ranks of the elapsed seconds."""
    for _ in range(warmup):
        step(None)
    sync()
    dctx.barrier()
    sync()
    t0 = time.perf_counter()
    for i in range(steps):
        step(i)
    sync()
    dctx.barrier()
    sync()
    return dctx.max(time.perf_counter() - t0)


def pmc_traffic(kernel_key, workload, alg_bytes):
    """HBM bytes per launch from the committed rocprofv3 PMC summary (separate
    --pmc passes; gfx950 FETCH_SIZE x2 correction, MI355X_MICROARCH.md §HBM),
    only when that summary was taken on this same workload and launch size.
    Returns (bytes or None, where they came from): the counters are NOT
    collected inside this run (a --pmc pass is its own rocprofv3 process)."""
    path = os.path.join(ROOT, "profiles", f"pmc_traffic_{workload}.json")
    if not os.path.exists(path):
        path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    rel = os.path.relpath(path, ROOT)
    try:
        d = json.load(open(path))
        if d.get("workload", "encdec") != workload:
            return None, f"none: {rel} is for another workload"
        k = d["kernels"][kernel_key]
        if k.get("algorithmic_bytes_per_launch") != alg_bytes:
            return None, f"none: {rel} is for another launch size"
        src = (f"committed profile {rel} (rocprofv3 --pmc passes of this workload and launch size, "
               f"{d.get('source', 'see the file')}); not measured in this run")
        return k["hbm_bytes_per_launch"], src
    except Exception:
        return None, f"none: no committed PMC summary for {kernel_key}"


def under_profiler() -> bool:
    """True when this process runs under rocprofv3 (its tool library is
    preloaded): a child rocprofv3 run would nest profilers."""
    return any(k.startswith(("ROCPROF", "ROCP_")) for k in os.environ) or \
        "rocprof" in os.environ.get("LD_PRELOAD", "")


def _pmc_child(args, counters, timeout=90, warmup=3):
    """One rocprofv3 --pmc child run of this same workload (`warmup` warm-up +
    3 timed steps, same batch rotation, no CPU leg, no nested passes), started
    after this process's timed region as a separate process (never an exec),
    its process group killed past `timeout` (a refused counter set hangs past
    SIGTERM).  Returns (path of its counter CSV copy or None, note); the
    output directory goes whatever happens to the pass."""
    import glob
    import shutil
    import signal
    import subprocess
    import tempfile
    exe = shutil.which("rocprofv3")
    if not exe:
        return None, "rocprofv3 not on PATH"
    # the children are plain one-process runs: no process group of their own
    child_env = {kk: v for kk, v in os.environ.items() if kk != "BENCH_COLLECTIVES"}
    child_env["BENCH_PMC_CHILD"] = "1"
    with tempfile.TemporaryDirectory(prefix="bench_pmc_", dir=os.environ.get("TMPDIR", "/tmp")) as out:
        cmd = [exe, "--pmc", *counters, "-d", out, "-o", "run", "--output-format", "csv", "--",
               sys.executable, os.path.abspath(__file__), "--workload", args.workload, "--no-cpu",
               "--no-pmc", "--steps", "3", "--warmup", str(warmup), "--copies", str(args.copies)]
        if args.batch:
            cmd += ["--batch", str(args.batch)]
        p = subprocess.Popen(cmd, env=child_env, stdout=subprocess.DEVNULL,
                             stderr=subprocess.DEVNULL, start_new_session=True)
        try:
            rc = p.wait(timeout=timeout)
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGKILL)
            p.wait()
            return None, f"rocprofv3 --pmc {' '.join(counters)} pass timed out ({timeout} s)"
        files = glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True)
        if rc != 0 or not files:
            return None, f"rocprofv3 --pmc {' '.join(counters)} pass failed (rc {rc})"
        keep = tempfile.NamedTemporaryFile(prefix="bench_pmc_", suffix=".csv", delete=False,
                                           dir=os.environ.get("TMPDIR", "/tmp"))
        keep.close()
        shutil.copyfile(files[0], keep.name)
        return keep.name, "ok"


def pmc_traffic_live(args, kernel_key, alg_bytes):
    """HBM bytes per launch of `kernel_key` measured in THIS run: two child
    runs of this same workload under `rocprofv3 --pmc FETCH_SIZE` and `--pmc
    WRITE_SIZE` (separate passes: the TCC block cannot hold both,
    MI355X_MICROARCH.md §rocprofv3 PMC slots), each averaged over that
    kernel's dispatches; read = 2 x FETCH_SIZE (the gfx950 correction of
    MI355X_MICROARCH.md §HBM), write = WRITE_SIZE, both KiB.  Returns (bytes or
    None, source note)."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from pmc_traffic import per_kernel, short
    key = short(kernel_key)
    got = {}
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        path, note = _pmc_child(args, [counter])
        if path is None:
            return None, note
        try:
            val = per_kernel(path, counter).get(key)
        finally:
            os.unlink(path)
        if not val:
            return None, f"rocprofv3 --pmc {counter}: no dispatch of {key}"
        got[counter] = val
    rd = 2.0 * got["FETCH_SIZE"][0] * 1024
    wr = got["WRITE_SIZE"][0] * 1024
    return int(rd + wr), (f"measured in this run: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE child passes of this "
                          f"workload ({got['FETCH_SIZE'][1]} / {got['WRITE_SIZE'][1]} dispatches of {key}), "
                          f"read 2 x FETCH_SIZE = {int(rd)} B + write {int(wr)} B per launch, "
                          f"{(rd + wr) / alg_bytes:.4f} x algorithmic")


SQ_COUNTERS = ["SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_WAIT_ANY",
               "SQ_WAIT_INST_ANY", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "GRBM_GUI_ACTIVE", "GRBM_COUNT"]


def pmc_issue_live(args, kernel_key):
    """Where the dominant kernel's waves spend their cycles, measured in THIS
    run: one child run under `rocprofv3 --pmc` with 8 SQ and 2 GRBM counters
    (one pass: the SQ block holds 8, MI355X_MICROARCH.md §rocprofv3 PMC
    slots), summarised by tools/pmc_sq.py: VALU instructions per wave,
    VALUBusy (SQ_ACTIVE_INST_VALU x 4 over every SIMD's cycles), the waves'
    parked (WAIT_ANY) and issue-stalled (WAIT_INST_ANY) shares of their
    cycles, and the clock the chip held in the pass (GRBM_GUI_ACTIVE / 8 /
    dispatch time; a profiled pass runs a few % off the unprofiled clock,
    §DVFS give-back).  Returns a dict or None and a note."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from pmc_sq import per_dispatch, summarise
    from pmc_traffic import short
    key = short(kernel_key)
    # 100 warm-up steps: the shader clock ramps over the first ~0.1 s of load;
    # the summary takes the last dispatches (the child's timed steps)
    path, note = _pmc_child(args, SQ_COUNTERS, warmup=100)
    if path is None:
        return None, note
    try:
        ds = per_dispatch(path).get(key)
    finally:
        os.unlink(path)
    if not ds:
        return None, f"SQ pass: no dispatch of {key}"
    ds = ds[-6:]  # 3 timed steps x at most 2 launches of the kernel per step
    sm = summarise(ds)
    out = {"kernel": key, "dispatches": sm["dispatches"]}
    for src, dst in (("valu_insts_per_wave", "valu_insts_per_wave"),
                     ("valu_active_share_of_simd_cycles", "valu_busy"),
                     ("wait_any_over_wave_cycles", "wait_any_share"),
                     ("wait_inst_any_over_wave_cycles", "wait_inst_any_share"),
                     ("active_inst_any_over_wave_cycles", "issuing_share"),
                     ("clock_GHz_pass_duration", "clock_GHz_in_pass")):
        if src in sm:
            out[dst] = sm[src]
    out["source"] = ("measured in this run: one rocprofv3 --pmc child pass (" + " ".join(SQ_COUNTERS) +
                     ") of this workload, tools/pmc_sq.py")
    return out, "ok"


def run_trace(args):
    """BASELINE config 5: mixed 4 KiB-100 MiB objects (log-uniform, numpy
    PCG64 seed 20200225, 512 objects, ~5 GiB), RS(10+2), one MI355X, host <->
    device copies INCLUDED: objects live in pinned host memory in Split
    layout; a step = encode_batch (H2D data rows -> kernel -> D2H parity) +
    decode_batch with data shards {0,5} missing (H2D 10 survivors -> kernel ->
    D2H 2 rows).  Prints one JSON line (this is a DESIGN.md measurement, not
    the headline metric)."""
    import torch

    import infinicache_amd as ia

    k, p = 10, 2
    n = k + p
    rng = np.random.Generator(np.random.PCG64(20200225))
    nobj = args.trace_objects
    sizes = np.exp(rng.uniform(np.log(4096), np.log(100 << 20), nobj)).astype(np.int64)
    S = (sizes + k - 1) // k
    offs = np.concatenate([[0], np.cumsum(n * S)])
    total_obj = int(sizes.sum())
    # --devices N (N > 1): one multi-device context, as the Go shim's
    # NewEncoder builds it: object o -> GPU o mod N, one pipeline and PCIe
    # link per GPU, all in this one process
    ndev = max(1, args.devices)
    if ndev > torch.cuda.device_count():
        raise SystemExit(f"--devices {ndev} but {torch.cuda.device_count()} GPU(s) visible")
    enc = ia.New(k, p, devices=list(range(ndev))) if ndev > 1 else ia.New(k, p)
    host = ia.host_alloc(int(offs[-1]))
    # random object bytes: one 256 MiB device random block, copied around
    rnd = torch.randint(0, 256, (256 << 20,), dtype=torch.uint8, device="cuda").cpu().numpy()
    objs = []
    for o in range(nobj):
        base = host[offs[o]:offs[o + 1]]
        nb = int(sizes[o])
        st = (o * 7919 * 4096) % (len(rnd) - (100 << 20) - 1)
        base[:nb] = rnd[st:st + nb]
        base[nb:] = 0
        objs.append([base[i * S[o]:(i + 1) * S[o]] for i in range(n)])
    lost = (0, 5)
    present = [[i not in lost for i in range(n)]] * nobj
    golden = [[objs[o][i].copy() for i in lost] for o in range(0, nobj, 37)]

    # the link's own rate, measured in this process before the timed region:
    # one pinned 1D copy of 512 MiB per direction (best of 5), the same kind
    # of memory the trace's objects live in (hipHostMalloc'd), GPU 0
    def link_rate(h2d):
        nb = 512 << 20
        hbuf = ia.host_alloc(nb)
        hbuf[:] = 1
        ht = torch.from_numpy(hbuf)
        dt = torch.empty(nb, dtype=torch.uint8, device="cuda")
        best = 0.0
        for _ in range(6):
            torch.cuda.synchronize()
            t = time.perf_counter()
            if h2d:
                dt.copy_(ht, non_blocking=True)
            else:
                ht.copy_(dt, non_blocking=True)
            torch.cuda.synchronize()
            best = max(best, nb / (time.perf_counter() - t) / 1e9)
        del ht, dt, hbuf
        return best
    link_h2d_gbs, link_d2h_gbs = link_rate(True), link_rate(False)
    # bytes each step moves over the link (encode_batch: data rows in, parity
    # out; decode_batch: the first k present rows in, the 2 rebuilt rows out)
    h2d_step = int(sum(2 * k * int(x) for x in S))
    d2h_step = int(sum((p + len(lost)) * int(x) for x in S))

    def step():
        enc.encode_batch(objs)
        oks = enc.decode_batch(objs, present=present)
        assert all(oks)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    el = time.perf_counter() - t0
    for j, o in enumerate(range(0, nobj, 37)):
        for g, i in zip(golden[j], lost):
            assert np.array_equal(objs[o][i], g), "decode did not restore the data rows"
    e2e = 2 * total_obj * args.steps / el / GiB
    h2d_gbs = h2d_step * args.steps / el / 1e9
    d2h_gbs = d2h_step * args.steps / el / 1e9

    # the same trace device-resident (kernel + launch only, no PCIe)
    pitches = [(int(x) + 255) // 256 * 256 for x in S]
    doffs = np.concatenate([[0], np.cumsum([n * pp for pp in pitches])])
    dev = torch.zeros(int(doffs[-1]), dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream()
    pres = [i not in lost for i in range(n)]
    bad = torch.zeros(1, dtype=torch.int32, device="cuda")

    def dstep_per_object():  # round 2's form: one launch per object and op
        for o in range(nobj):
            b = dev.data_ptr() + int(doffs[o])
            enc.encode_dev(b, int(S[o]), pitches[o], n * pitches[o], 1, stream)
            enc.decode_dev(b, pres, int(S[o]), pitches[o], n * pitches[o], 1, bad, stream)

    # one launch per op over the whole trace (variable-size table)
    dobjs = [(dev.data_ptr() + int(doffs[o]), int(S[o]), pitches[o]) for o in range(nobj)]
    badv = torch.zeros(nobj, dtype=torch.int32, device="cuda")

    def dstep():
        enc.encode_dev_objs(dobjs, stream)
        enc.decode_dev_objs(dobjs, pres, badv, stream)

    def time_dev(fn):
        fn()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(args.steps):
            fn()
        torch.cuda.synchronize()
        return time.perf_counter() - t1

    # device-resident work check: garbage into the lost rows of every object,
    # one decode, compare with the rows before
    dgen = torch.Generator(device="cuda").manual_seed(3)
    dev.copy_(torch.randint(0, 256, dev.shape, dtype=torch.uint8, device="cuda", generator=dgen))
    enc.encode_dev_objs(dobjs, stream)
    ref = dev.clone()
    for o in range(nobj):
        for i in lost:
            a = int(doffs[o]) + i * pitches[o]
            dev[a:a + int(S[o])] = 0xA5
    badv.fill_(7)
    enc.decode_dev_objs(dobjs, pres, badv, stream)
    torch.cuda.synchronize()
    dev_check = "bit-exact" if (not bool(badv.any()) and torch.equal(dev, ref)) else "MISMATCH"
    del ref
    if dev_check != "bit-exact":
        raise SystemExit("trace device-resident decode check failed")
    dev_el = time_dev(dstep)
    dev_rate = 2 * total_obj * args.steps / dev_el / GiB
    per_obj_el = time_dev(dstep_per_object)
    per_obj_rate = 2 * total_obj * args.steps / per_obj_el / GiB

    cpu = None
    if not args.no_cpu:
        import oracle
        from oracle import rs_numpy as rn
        m = enc.matrix()
        surv = [i for i in range(n) if i not in lost][:k]
        inv_rows = rn.invert(m[surv])[list(lost)]
        threads = int(os.environ.get("BENCH_CPU_THREADS", "16"))
        t2 = time.perf_counter()
        done = 0
        for o in range(nobj):
            sh = objs[o]
            oracle.code_fast(m[k:], sh[:k], nthreads=threads, max_goroutines=32)
            oracle.code_fast(inv_rows, [sh[i] for i in surv], nthreads=threads, max_goroutines=32)
            done += 2 * int(sizes[o])
            if time.perf_counter() - t2 > args.cpu_seconds:
                break
        cel = time.perf_counter() - t2
        cpu = {"value": round(done / cel / GiB, 3), "unit": "GiB/s", "cores": threads,
               "kind": "port",
               "sample": f"per-object codeSomeShardsP (maxGoroutines 32) encode+decode over "
                         f"{o + 1} trace objects ({done / GiB:.2f} GiB), host memory, no PCIe"}
    out = {
        "metric": "RS(10+2) encode+decode GiB/s, mixed 4 KiB-100 MiB trace, host<->device copies included",
        "value": round(e2e, 2),
        "unit": "GiB/s",
        "n_gpus": ndev,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(el / args.steps * 1e3, 2),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic: log-uniform sizes (PCG64 seed 20200225), random bytes, pinned host memory",
        "config": {"workload": "config 5 mixed trace, e2e (pinned H2D -> gf_apply -> D2H, 4 slots/streams)",
                   "devices_in_process": ndev, "objects": nobj, "total_object_bytes": total_obj,
                   "size_min": int(sizes.min()), "size_max": int(sizes.max()),
                   "size_median": int(np.median(sizes))},
        "device_resident_same_trace_GiBps": round(dev_rate, 2),
        "device_resident_form": "rsgpu_encode_dev_objs + rsgpu_decode_dev_objs: one launch per op "
                                "over the whole trace (variable-size object table)",
        "device_resident_check": dev_check,
        "device_resident_per_object_launches_GiBps": round(per_obj_rate, 2),
        "kernel_fraction_of_e2e_time": round(dev_el / el, 4),
        # the e2e path is bound by the PCIe link's host-to-device direction:
        # achieved = H2D bytes the step moves / step time, peak = the pinned
        # 1D H2D copy rate measured in this process before the timed region
        # (D2H runs concurrently on the other direction of the link)
        "roofline": {
            "bound": "pcie-h2d",
            "achieved": round(h2d_gbs, 2),
            "peak": round(link_h2d_gbs, 2),
            "unit": "GB/s",
            "frac": round(h2d_gbs / link_h2d_gbs, 4),
            "traffic": h2d_step,
            "traffic_note": "H2D bytes per step (2 x k x shard_len per object: the encode's data rows and the "
                            "decode's k survivors); per-step, not per kernel launch",
            "d2h": {"achieved": round(d2h_gbs, 2), "peak": round(link_d2h_gbs, 2),
                    "frac": round(d2h_gbs / link_d2h_gbs, 4), "bytes_per_step": d2h_step,
                    "share_of_link_bytes": round(d2h_step / (h2d_step + d2h_step), 4)},
            "peak_source": "pinned 1D copy of 512 MiB per direction, hipHostMalloc'd host memory, best of 6, "
                           "this process, before the timed region",
        },
        **({"winner": ("gpu_e2e" if e2e > cpu["value"] else "cpu_port"),
            "gpu_e2e_over_cpu": round(e2e / cpu["value"], 3)} if cpu else {}),
        "cpu_baseline": cpu,
    }
    print(json.dumps(out), flush=True)


def run_latency(args):
    """The per-object path the Go shim takes (one EcSet / EcGet at a time,
    host buffers in and out): Client.encode = Encode + Verify
    (ecRedis.go:382-402) and Client.decode = Reconstruct + Verify of 2 lost
    data shards, fused (ecRedis.go:404-427), on RS(10+2) objects of
    --obj-bytes (1 MiB), from Python (the C ABI's own figures: tools/lat_bench).
    Reports per-op latency percentiles beside the CPU port's per-object
    codeSomeShardsP latency.  A DESIGN.md measurement, not the headline."""
    import infinicache_amd as ia
    import oracle
    from oracle import rs_numpy as rn
    k, p, nb = 10, 2, args.obj_bytes
    enc = ia.New(k, p)
    if args.worker:
        enc.worker_start(nslots=args.worker)
    rng = np.random.default_rng(7)
    nobj = 64
    objs = [rng.integers(0, 256, nb, dtype=np.uint8) for _ in range(nobj)]
    res = {}
    for pinned in (False, True):
        lat_e, lat_d = [], []
        for it in range(args.steps + args.warmup):
            o = objs[it % nobj]
            if pinned:
                buf = ia.host_alloc((k + p) * ((nb + k - 1) // k))
                S = len(buf) // (k + p)
                buf[:nb] = o
                buf[nb:] = 0
                sh = [buf[i * S:(i + 1) * S] for i in range(k + p)]
            else:
                sh = enc.Split(o)
            t0 = time.perf_counter()
            ok = enc.EncodeVerify(sh)  # Client.encode's Encode+Verify, one round trip
            t1 = time.perf_counter()
            assert ok
            got = [None if i in (0, 5) else sh[i] for i in range(k + p)]
            t2 = time.perf_counter()
            ok = enc.DecodeVerify(got)
            t3 = time.perf_counter()
            assert ok and np.array_equal(got[0], sh[0])
            if it >= args.warmup:
                lat_e.append(t1 - t0)
                lat_d.append(t3 - t2)
        key = "pinned" if pinned else "pageable"
        res[key] = {
            "encode_verify_us_p50": round(float(np.percentile(lat_e, 50)) * 1e6, 1),
            "encode_verify_us_p99": round(float(np.percentile(lat_e, 99)) * 1e6, 1),
            "decode_us_p50": round(float(np.percentile(lat_d, 50)) * 1e6, 1),
            "decode_us_p99": round(float(np.percentile(lat_d, 99)) * 1e6, 1),
        }
    # CPU port, same ops per object (codeSomeShardsP, 16 threads)
    m = enc.matrix()
    inv = rn.invert(m[[1, 2, 3, 4, 6, 7, 8, 9, 10, 11]])[[0, 5]]
    threads = int(os.environ.get("BENCH_CPU_THREADS", "16"))
    ce, cd = [], []
    for it in range(args.steps + args.warmup):
        sh = rn.split(objs[it % nobj].tobytes(), k, p)
        t0 = time.perf_counter()
        par = oracle.code_fast(m[k:], sh[:k], nthreads=threads, max_goroutines=32)
        chk = oracle.code_fast(m[k:], sh[:k], nthreads=threads, max_goroutines=32)  # Verify
        t1 = time.perf_counter()
        surv = [sh[i] for i in (1, 2, 3, 4, 6, 7, 8, 9)] + par
        oracle.code_fast(inv, surv, nthreads=threads, max_goroutines=32)
        t2 = time.perf_counter()
        if it >= args.warmup:
            ce.append(t1 - t0)
            cd.append(t2 - t1)
    from infinicache_amd import ec
    out = {
        "metric": f"RS(10+2) per-object host-API latency (Client.encode / Client.decode), {nb} B objects, "
                  f"from Python",
        "python_marshalling": "C (csrc/pyshards.c)" if ec._pyshards is not None else "ctypes",
        "worker_mailboxes": args.worker,
        "worker_stats": enc.worker_stats() if args.worker else None,
        "gpu": res,
        "cpu_port_16_threads": {
            "encode_verify_us_p50": round(float(np.percentile(ce, 50)) * 1e6, 1),
            "decode_us_p50": round(float(np.percentile(cd, 50)) * 1e6, 1)},
        "ops": args.steps,
    }
    print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=None,
                    help="untimed steps (default 300 for the device-resident workloads: the shader "
                         "clock ramps over the first ~0.1 s of load; 3 for trace/latency)")
    ap.add_argument("--workload", default="encdec", choices=sorted(WORKLOADS) + ["trace", "latency"])
    ap.add_argument("--trace-objects", type=int, default=512)
    ap.add_argument("--obj-bytes", type=int, default=1 << 20, help="latency: object size")
    ap.add_argument("--worker", type=int, default=0, help="latency: resident worker mailboxes (0: stream path)")
    ap.add_argument("--devices", type=int, default=1,
                    help="trace: GPUs driven by ONE process through a multi-device context")
    ap.add_argument("--batch", type=int, default=0, help="objects per GPU (default: workload's)")
    ap.add_argument("--strong", action="store_true",
                    help="strong scaling: the workload's batch is the TOTAL, split over ranks")
    ap.add_argument("--collectives", action="store_true",
                    help="issue the barrier / MAX / gather collectives at world size 1 too (one RCCL "
                         "rank under torch.distributed.run; also BENCH_COLLECTIVES=1)")
    ap.add_argument("--copies", type=int, default=3,
                    help="distinct batches per GPU, step i codes batch i %% copies (cold Infinity Cache)")
    ap.add_argument("--warm", action="store_true",
                    help="also time K steps re-coding one batch (warm Infinity Cache; comparison only)")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--cpu-seconds", type=float, default=20.0)
    ap.add_argument("--no-pmc", action="store_true",
                    help="take roofline.traffic from the committed PMC summary instead of two rocprofv3 "
                         "--pmc child passes of this workload (the default at N = 1 when rocprofv3 is present)")
    args = ap.parse_args()
    if args.warmup is None:
        # ~0.1-0.2 s of untimed steps: the HBM-bound workloads time the same
        # with 3 or 1000 (the headline: 4,530-4,555 GiB/s), but the VALU-
        # heavier passes read slow until the shader clock has ramped (wide
        # RS(20+4) -10 %, 4 KiB mixed patterns -6 %; profiles/r02_bench_warmup*.txt)
        args.warmup = 3 if args.workload in ("trace", "latency") else 300

    if args.workload == "trace":
        return run_trace(args)
    if args.workload == "latency":
        return run_latency(args)

    import torch
    import torch.distributed as dist

    import infinicache_amd as ia

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: launch N > 1 ranks with "
                         f"python -m torch.distributed.run --nproc-per-node N bench.py --gpus N")
    # BENCH_DIST_BACKEND=gloo + BENCH_SHARE_GPU=1: rehearse the N-rank path on
    # a one-GPU box (ranks share cuda:0; RCCL refuses two ranks on one GPU).
    # The driver's multi-GPU runs use the defaults: RCCL, one GPU per rank.
    backend = os.environ.get("BENCH_DIST_BACKEND", "nccl")
    if os.environ.get("BENCH_SHARE_GPU") == "1":
        local = local % max(1, torch.cuda.device_count())
    force_coll = args.collectives or os.environ.get("BENCH_COLLECTIVES") == "1"
    dist_on = world > 1 or force_coll
    if dist_on:
        os.environ.setdefault("MASTER_PORT", "29517")
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", rank=rank, world_size=world,
                                    device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend, rank=rank, world_size=world)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    if not ia.device_ok(local):
        raise SystemExit(f"rank {rank}: no usable gfx950 device at cuda:{local}")

    w = WORKLOADS[args.workload]
    k, p = w["k"], w["p"]
    n = k + p
    batch_total = args.batch or w["batch"]
    nobj = batch_total
    if args.strong:
        nobj = shard_objects(nobj, rank, world)[1]
    S = (w["nbytes"] + k - 1) // k
    if w.get("shard_major"):  # [shard][object]: object o's piece of shard i at i*pitch + o*stride
        if w.get("oalign") == "library":  # the geometry rsgpu_shardmajor_layout chooses
            stride, pitch = ia.shardmajor_layout(S, nobj)
        else:
            oal = w.get("oalign", 1)
            stride = (S + oal - 1) // oal * oal
            pitch = (nobj * stride + 255) // 256 * 256
    else:                     # [object][shard][pitch]
        pal = w.get("palign", 256)
        pitch = (S + pal - 1) // pal * pal
        stride = n * pitch
    enc = ia.New(k, p, device=local)
    stream = torch.cuda.current_stream(dev)

    # synthetic objects: uniform random bytes, generated on device per rank.
    # `copies` distinct batches, step i codes batch i % copies: a batch is
    # re-read only after (copies-1) x 1.3+ GB of other traffic, so none of it
    # is left in the 256 MiB Infinity Cache (MALL) and the timed rate is the
    # HBM rate.  Re-coding ONE batch every step instead lets that cache absorb
    # the repeated parity rewrites (kbench KB_ROT sweep); that
    # warm rate is reported beside it as `warm_repeat`, never as `value`.
    copies = max(1, args.copies)
    g = torch.Generator(device=dev).manual_seed(0x1F1C + rank)
    if w.get("shard_major"):
        allbuf = torch.randint(0, 256, (copies, n, pitch), dtype=torch.uint8, device=dev, generator=g)
        allbuf[..., nobj * stride:] = 0
        if stride > S:  # zero pads between the pieces
            allbuf[..., :nobj * stride].view(copies, n, nobj, stride)[..., S:] = 0
    else:
        allbuf = torch.randint(0, 256, (copies, nobj, n, pitch), dtype=torch.uint8, device=dev, generator=g)
        allbuf[..., S:] = 0
    bufs = [allbuf[j] for j in range(copies)]
    bad = torch.zeros(nobj, dtype=torch.int32, device=dev)
    present = [i not in w["lost"] and i not in w.get("absent", ()) for i in range(n)]
    if "encode" not in w["ops"]:  # decode-only workload: start from valid parity
        enc.encode_dev(allbuf, S, pitch, stride, nobj * copies, stream)
    if w.get("mixed"):  # per-object random erasure pair (seeded)
        prs = np.random.default_rng(20200225 + rank)
        pres_m = np.ones((nobj, n), dtype=np.uint8)
        if nobj <= 4096:
            for o in range(nobj):
                pres_m[o, prs.choice(n, p, replace=False)] = 0
        else:  # vectorised: the p smallest of n uniform keys per object
            np.put_along_axis(pres_m, np.argsort(prs.random((nobj, n)), axis=1)[:, :p], 0, axis=1)
        # the arrival bitmaps live in HBM next to the shards (bit i: shard i
        # arrived); the decode resolves each object's pattern on the device
        masks_np = (pres_m.astype(np.int64) << np.arange(n)).sum(axis=1).astype(np.int32)
        masks_dev = torch.from_numpy(masks_np).to(dev)

    # each op codes the first `cnt` objects of a batch (default: all of them;
    # the strong-scaling block codes this rank's share of one batch)
    def op_encode(buf, cnt=None):
        enc.encode_dev(buf, S, pitch, stride, nobj if cnt is None else cnt, stream)

    def op_decode(buf, cnt=None):
        c = nobj if cnt is None else cnt
        if w.get("upstream_get"):
            enc.reconstruct_dev(buf, present, S, pitch, stride, c, data_only=False, stream=stream)
            enc.verify_dev(buf, S, pitch, stride, c, bad, stream)
        elif w.get("mixed"):
            enc.decode_dev_masks(buf, masks_dev, S, pitch, stride, c, bad, stream)
        elif w.get("data_only"):
            enc.reconstruct_dev(buf, present, S, pitch, stride, c, data_only=True, stream=stream)
        else:
            enc.decode_dev(buf, present, S, pitch, stride, c, bad, stream)

    op_fns = {"encode": op_encode, "decode": op_decode}

    # timing units: each op, except the unfused upstream Get, which is timed
    # (and profiled) as its two launches
    def op_reconstruct(buf, cnt=None):
        enc.reconstruct_dev(buf, present, S, pitch, stride, nobj if cnt is None else cnt, data_only=False,
                            stream=stream)

    def op_verify(buf, cnt=None):
        enc.verify_dev(buf, S, pitch, stride, nobj if cnt is None else cnt, bad, stream)

    units = []
    for op in w["ops"]:
        if op == "decode" and w.get("upstream_get"):
            units += [("decode:reconstruct", op_reconstruct), ("decode:verify", op_verify)]
        else:
            units.append((op, op_fns[op]))

    # rows of the decode: present shards, rows it writes, and the extra present
    # shards (beyond the first k) the fused Get checks in the same pass
    n_present = sum(present)
    e_rows = len(w["lost"]) + (0 if w.get("data_only") else len(w.get("absent", ())))
    fused_checks = 0 if (w.get("data_only") or w.get("upstream_get") or w.get("mixed")) else n_present - k
    # the row the corruption check flips: a present parity row that the decode
    # verifies (fused: an extra shard; upstream: Verify reads every row)
    check_row = None
    if "decode" in w["ops"] and (fused_checks > 0 or (w.get("upstream_get") and n_present > k)) \
            and not w.get("shard_major"):
        check_row = max(i for i in range(n) if present[i])

    # rows each op writes, per (object, shard row)
    written = {}
    if "encode" in w["ops"]:
        e_enc = torch.zeros((nobj, n), dtype=torch.bool, device=dev)
        e_enc[:, k:] = True
        written["encode"] = e_enc
    if "decode" in w["ops"]:
        if w.get("mixed"):
            e_dec = torch.from_numpy(pres_m == 0).to(dev)
        else:
            rows = list(w["lost"]) + ([] if w.get("data_only") else list(w.get("absent", ())))
            e_dec = torch.zeros((nobj, n), dtype=torch.bool, device=dev)
            e_dec[:, rows] = True
        written["decode"] = e_dec

    def check_ops(buf):
        """Garbage into every row the op writes, the op, then a bit-exact
        compare of those rows' shard_len bytes with the copy taken before."""
        out = {}
        gg = torch.Generator(device=dev).manual_seed(0xBAD + rank)
        for op in w["ops"]:
            ref = buf.clone()
            E = written[op]
            if w.get("shard_major"):
                pieces = buf[:, :nobj * stride].view(n, nobj, stride)
                Et = E.t().contiguous()
                pieces[Et] = torch.randint(0, 256, (int(Et.sum()), stride), dtype=torch.uint8, device=dev,
                                           generator=gg)
            else:
                buf[E] = torch.randint(0, 256, (int(E.sum()), pitch), dtype=torch.uint8, device=dev, generator=gg)
            flags = op == "decode" and not w.get("data_only")  # the decode sets every object's flag
            if flags:
                bad.fill_(7)
            op_fns[op](buf)
            torch.cuda.synchronize(dev)
            if flags and int(bad.sum()) != 0:
                raise SystemExit(f"{op} check: decode reported a mismatch / error status")
            if w.get("shard_major"):
                same = torch.equal(buf[:, :nobj * stride].view(n, nobj, stride)[..., :S],
                                   ref[:, :nobj * stride].view(n, nobj, stride)[..., :S])
            else:
                same = torch.equal(buf[..., :S], ref[..., :S])
            del ref
            if not same:
                raise SystemExit(f"{op} check FAILED: rewritten rows differ from the rows before")
            out[op] = {"result": "bit-exact", "objects": nobj, "rows_rewritten": int(E.sum()),
                       "bytes_compared": int(E.sum()) * S}
            if op == "decode" and check_row is not None:
                # one corrupted byte in a checked parity row of one object:
                # the decode must flag exactly that object (and still rebuild
                # every object's lost rows bit-exact)
                o = nobj // 2
                buf[o, check_row, S - 1] ^= 0x5A
                ref = buf.clone()
                buf[E] = 0
                bad.fill_(7)
                op_fns[op](buf)
                torch.cuda.synchronize(dev)
                flagged = torch.nonzero(bad).flatten().tolist()
                same = torch.equal(buf[..., :S], ref[..., :S])
                buf[o, check_row, S - 1] ^= 0x5A
                del ref
                if flagged != [o] or not same:
                    raise SystemExit(f"{op} corruption check FAILED: flagged {flagged[:8]}, expected [{o}]; "
                                     f"rebuilt rows {'equal' if same else 'DIFFER'}")
                out[op]["corruption_check"] = {"object": o, "row": check_row, "byte": S - 1,
                                               "flagged": flagged, "result": "exactly that object flagged"}
        return out

    turn = [0]

    def step(fixed=None):
        buf = bufs[turn[0] % copies] if fixed is None else bufs[fixed]
        turn[0] += 1
        for op in w["ops"]:
            op_fns[op](buf)

    def kernel_ms(fixed=None):
        """Per-op launch time: HIP events around an UNINTERRUPTED run of K
        launches of that op alone (batches in the same rotation), on the
        stream the kernels run on.  No marker packets between the launches,
        so the average is the kernel's own time plus launch gaps; the timed
        steps above carry no events at all."""
        out = {}
        for name, fn in units:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            fn(bufs[0 if fixed is not None else 1 % copies])  # untimed: same launch shape warm
            e0.record(stream)
            for i in range(args.steps):
                fn(bufs[fixed if fixed is not None else i % copies])
            e1.record(stream)
            e1.synchronize()
            out[name] = e0.elapsed_time(e1) / args.steps
        return out

    dctx = DistCtx(world, rank, dev, force=force_coll)
    elapsed = timed_run(lambda i: step(), args.steps, args.warmup, lambda: torch.cuda.synchronize(dev), dctx)
    objs_all = dctx.sum(nobj)
    if int(bad.sum()) != 0:
        raise SystemExit("decode reported a verify mismatch on synthetic data")

    # Strong scaling beside the weak line ("strong
    # scaling of 1024 total"): the workload's ONE batch split over the ranks
    # by shard_objects, each rank coding its share (a prefix of its own
    # batches, same rotation) under the same barriers and MAX-over-ranks
    # timing.  Timed after the weak region; not the line's `value`.
    strong = None
    if dist_on and not args.strong:
        s_start, s_cnt = shard_objects(batch_total, rank, world)
        sturn = [0]

        def sstep(i):
            buf = bufs[sturn[0] % copies]
            sturn[0] += 1
            for op in w["ops"]:
                op_fns[op](buf, s_cnt)

        s_el = timed_run(sstep, args.steps, max(3, args.warmup // 10), lambda: torch.cuda.synchronize(dev), dctx)
        if int(bad.sum()) != 0:
            raise SystemExit("decode reported a verify mismatch on synthetic data (strong block)")
        s_objs = dctx.sum(s_cnt)
        s_counts = [int(round(c)) for c in dctx.gather(float(s_cnt))]
        strong = {
            "value": round(s_objs * w["nbytes"] * len(w["ops"]) * args.steps / s_el / GiB, 2),
            "unit": "GiB/s",
            "ms_per_step": round(s_el / args.steps * 1e3, 4),
            "batch_total": batch_total,
            "objects_coded": s_objs,
            "objects_per_rank": s_counts,
            "note": "the workload's one batch split over the ranks (shard_objects), max-over-ranks time, "
                    "same barriers; timed after the weak region, not the line's value",
        }
        if s_objs != batch_total:
            raise SystemExit(f"strong block coded {s_objs} objects, batch is {batch_total}")
    # Untimed proof that the timed ops did their work: on batch 0, overwrite
    # every row an op writes (encode: the parity rows; decode: each object's
    # erased rows) with random garbage, run the op, and compare the rows'
    # shard_len bytes with a copy taken before (client/ecRedis.go:390,404-427).
    work_check = check_ops(bufs[0])
    # every rank's own check passed (a failing rank exits before this point):
    # 1 per rank, in rank order
    wc_ranks = [int(round(x)) for x in dctx.gather(1.0)]
    kms_alone = kernel_ms()
    # Each op's share of the timed step comes from its uninterrupted run; run
    # alone an op can be a little slower than inside the step (there a decode
    # re-reads rows its batch's encode just streamed, partly still in the
    # Infinity Cache), so the shares are scaled to the measured step when
    # they add up to more: kernel time x launches never exceeds ms_per_step.
    ms_per_step_meas = elapsed / args.steps * 1e3
    scale = min(1.0, ms_per_step_meas / max(sum(kms_alone.values()), 1e-9))
    kms = {op: t * scale for op, t in kms_alone.items()}
    ops = len(w["ops"])

    # --warm: the same K steps on ONE batch (warm Infinity Cache), for
    # comparison only (off by default so a rocprofv3 run of the default
    # command averages the cold launches alone)
    if args.warm:
        warm_el = timed_run(lambda i: step(fixed=0), args.steps, args.warmup,
                            lambda: torch.cuda.synchronize(dev), dctx)
        if int(bad.sum()) != 0:
            raise SystemExit("decode reported a verify mismatch on synthetic data")
        warm_ms = kernel_ms(fixed=0)
    total_obj_bytes = objs_all * w["nbytes"] * ops * args.steps
    value = total_obj_bytes / elapsed / GiB
    ms_per_step = elapsed / args.steps * 1e3

    # algorithmic bytes per launch: encode k*S read + p*S write;
    # decode: every row it reads (the first k present, plus the extra present
    # shards a fused Get checks) + every row it writes (each missing row, parity
    # included (upstream Reconstruct, ecRedis.go:415), unless ReconstructData);
    # upstream's separate Verify reads all k+p rows
    dec_in = k + fused_checks
    sm = bool(w.get("shard_major"))
    enc_sym = pass_symbol(k, p, 0, S, sm)
    dec_sym = pass_symbol(dec_in, e_rows + fused_checks, fused_checks, S, sm)
    if k > 16:  # generic kernel, one launch per <= 8 rows
        enc_sym, dec_sym = f"gf_apply_generic<{min(p, 8)}>", f"gf_apply_generic<{e_rows}>"
    if w.get("mixed"):  # device-resolved patterns: KMAX = n inputs (gf_masked.h)
        dec_sym = f"gf_apply_{'lanes' if ((S + 15) // 16) * 2 <= 256 else 'masked'}<{n},{min(p, 4)}>"
    # unit -> (kernel symbol, algorithmic bytes per launch, bytes read per launch)
    unit_info = {
        "encode": (enc_sym, nobj * n * S, nobj * k * S),
        "decode": (dec_sym, nobj * (dec_in + e_rows) * S, nobj * dec_in * S),
        "decode:reconstruct": (pass_symbol(k, e_rows, 0, S, sm), nobj * (k + e_rows) * S, nobj * k * S),
        "decode:verify": (pass_symbol(n, p, p, S, sm), nobj * n * S, nobj * n * S),
    }
    # launches grouped by kernel symbol: encode and the uniform-pattern decode
    # of RS(10+2) are the same kernel (gf_apply_kernel<10,2>) with the same
    # algorithmic bytes per launch, so its average duration is over both, as
    # rocprofv3 --stats reports it
    per_op = {name: (*unit_info[name], kms[name]) for name, _ in units}
    groups = {}
    for op, (sym, b, rb, ms) in per_op.items():
        groups.setdefault((sym, b, rb), []).append((op, ms))
    # dominant: the kernel with the most time per step
    (kernel_key, dom_bytes, dom_read), members = max(groups.items(), key=lambda kv: sum(m for _, m in kv[1]))
    dom_ms = float(np.mean([m for _, m in members]))
    dom = "+".join(op for op, _ in members)
    achieved = dom_bytes / (dom_ms * 1e-3) / 1e9
    # every rank's own kernel rate (N > 1: each GPU codes its own objects)
    frac_ranks = [round(a / HBM_PEAK_GBS, 4) for a in dctx.gather(achieved)]
    traffic, traffic_src = None, None
    # HBM traffic of the dominant kernel measured in this run (rank 0 of a
    # one-GPU run; N > 1 ranks and profiled runs use the committed summary)
    if world == 1 and not args.no_pmc and not os.environ.get("BENCH_PMC_CHILD") and "+" not in kernel_key \
            and not under_profiler():
        traffic, traffic_src = pmc_traffic_live(args, kernel_key, dom_bytes)
        if traffic is None:
            log(f"PMC traffic not measured: {traffic_src}")
            note = traffic_src
            traffic, traffic_src = pmc_traffic(kernel_key, args.workload, dom_bytes)
            traffic_src = f"{traffic_src} (live passes: {note})"
    if traffic_src is None:
        traffic, traffic_src = pmc_traffic(kernel_key, args.workload, dom_bytes)
    # the dominant kernel's issue / wait / clock counters, same conditions
    issue = None
    if world == 1 and not args.no_pmc and not os.environ.get("BENCH_PMC_CHILD") and not under_profiler():
        issue, note = pmc_issue_live(args, kernel_key)
        if issue is None:
            log(f"SQ counters not measured: {note}")
    roofline = {
        "bound": "hbm",
        "achieved": round(achieved, 1),
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 4),
        "traffic": traffic,
        "traffic_source": traffic_src,
        "kernel": f"{kernel_key} ({dom} launches), {dom_bytes} algorithmic B/launch, "
                  f"{dom_ms * 1e3:.1f} us avg (HIP events around {args.steps} back-to-back launches "
                  f"per op after the timed steps, scaled x{scale:.4f} to the timed step)",
        "kernel_ms_per_step": round(sum(kms.values()), 4),
        "kernel_ms_alone": {op: round(t, 4) for op, t in kms_alone.items()},
        "per_kernel_GBps": {op: round(b / (ms * 1e-3) / 1e9, 1) for op, (_, b, _rb, ms) in per_op.items()},
        "per_kernel_symbol": {op: sym for op, (sym, _b, _rb, _ms) in per_op.items()},
        # the read side alone (the input rows per object and launch), SURVEY §8d
        "read_only": {"achieved": round(dom_read / (dom_ms * 1e-3) / 1e9, 1),
                      "frac": round(dom_read / (dom_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)},
        # achieved / peak of the same kernel on each rank's GPU (rank order);
        # achieved and frac above are rank 0's
        "frac_per_rank": frac_ranks,
        **({"issue": issue} if issue else {}),
    }

    warm = None
    if args.warm:
        warm = {
            "value": round(objs_all * w["nbytes"] * ops * args.steps / warm_el / GiB, 2),
            "frac": round(dom_bytes / (float(np.mean([warm_ms[op] for op, _ in members])) * 1e-3)
                          / 1e9 / HBM_PEAK_GBS, 4),
            "note": "one batch re-coded every step: its parity rewrites hit the 256 MiB Infinity "
                    "Cache, so this is not an HBM rate (reported for comparison, not the value)",
        }

    # The CPU baseline at every world size (north_star: "next to the Go CPU
    # path ... in the same run"): rank 0 times the CPU port after the timed
    # region and its barriers, on its own batch 0 (bit-compared with its GPU).
    cpu = None
    if rank == 0 and not args.no_cpu and not w.get("shard_major"):
        from oracle import rs_numpy as rn
        ns = min(256, nobj)  # 256 x 1.26 MB: well beyond the host's last-level cache
        # final GPU state of the sampled objects: batch 0 after check_ops, so
        # its parity rows and erased rows are the ones the GPU rewrote from garbage
        gpu_sample = bufs[0][:ns].cpu().numpy()
        sample = gpu_sample.copy()
        if "encode" in w["ops"]:
            sample[:, k:] = 0           # CPU recomputes parity from the same data rows
        else:
            sample[:, list(w["lost"])] = 0  # CPU reconstructs the erased rows
        m = enc.matrix()
        surv = [i for i in range(n) if present[i]][:k]
        inv_rows = rn.invert(m[surv])[list(w["lost"])] if w["lost"] else None
        cpu = cpu_baseline(w, sample, gpu_sample, m, inv_rows, budget_s=args.cpu_seconds,
                           threads=int(os.environ.get("BENCH_CPU_THREADS", "16")), fused_checks=fused_checks)

    if rank == 0:
        out = {
            "metric": METRICS[args.workload],
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "strong" if args.strong else "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": f"synthetic: uniform random bytes (torch.randint on device, seeded per rank), "
                    f"{copies} distinct batches coded in rotation",
            "config": {
                "workload": w["desc"],
                "k": k, "p": p,
                "object_bytes": w["nbytes"],
                "shard_len": S,
                "pitch": pitch,
                "obj_stride": stride,
                "layout": "shard-major" if w.get("shard_major") else "object-major",
                "batch_per_gpu": nobj,
                "batch_copies": copies,
                "decode_erasures": list(w["lost"]),
                "parallelism": (f"object-per-rank x{world} "
                                + ("(one process, no collective)" if not dist_on else
                                   f"({'RCCL' if backend == 'nccl' else backend} all_reduce barrier only"
                                   + (", ranks sharing one GPU)" if os.environ.get("BENCH_SHARE_GPU") == "1"
                                      else ")"))),
            },
            "roofline": roofline,
            **({"decode_check": work_check["decode"]["result"]} if "decode" in work_check else {}),
            "work_check": work_check,
            "work_check_ranks": wc_ranks,
            **({"warm_repeat": warm} if warm else {}),
            **({"strong_scaling": strong} if strong else {}),
            **({"collectives_issued": dctx.calls} if dist_on else {}),
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if dist_on:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
