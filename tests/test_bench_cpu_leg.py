"""bench.py's CPU-baseline leg for the checked Get of BASELINE config 3
(dec4_get / dec4_upstream), no GPU: the oracle's batch Verify
(oracle.verify_batch, upstream Verify / checkSomeShards) and the CPU decode
forms bench.py times beside the GPU line.

  * verify_batch flags exactly the objects whose stored rows differ from the
    recomputed ones (upstream Verify: every parity row re-encoded from the
    data rows; the fused Get: the extra shards from the survivors);
  * cpu_baseline on a small RS(10+4) batch with 12 of 14 shards present
    rebuilds data {0,5} bit-exact and reports both forms (Reconstruct+Verify,
    client/ecRedis.go:414-420, and the fused one)."""
import numpy as np

import bench
import oracle
from oracle import rs_numpy as rn


def _batch(k, p, nobj, S, pitch, seed):
    n = k + p
    rng = np.random.default_rng(seed)
    b = np.zeros((nobj, n, pitch), dtype=np.uint8)
    b[:, :k, :S] = rng.integers(0, 256, (nobj, k, S), dtype=np.uint8)
    m = rn.build_matrix(k, p)
    oracle.code_batch(m[k:], list(range(k)), list(range(k, n)), b.reshape(-1), n * pitch, pitch, S, nobj)
    return b, m


def test_verify_batch_flags_exactly_the_corrupt_objects():
    k, p, nobj, S, pitch = 10, 4, 7, 1000, 1024
    n = k + p
    b, m = _batch(k, p, nobj, S, pitch, 1)
    ok = oracle.verify_batch(m[k:], list(range(k)), list(range(k, n)), b.reshape(-1), n * pitch, pitch, S,
                             nobj, nthreads=4)
    assert ok.tolist() == [1] * nobj
    b[3, 13, S - 1] ^= 1   # parity row, last byte
    b[5, 2, 0] ^= 0x80     # a data row: every parity row disagrees
    ok = oracle.verify_batch(m[k:], list(range(k)), list(range(k, n)), b.reshape(-1), n * pitch, pitch, S,
                             nobj, nthreads=4)
    assert ok.tolist() == [1, 1, 1, 0, 1, 0, 1]
    # the fused Get's checks: extra shards 12, 13 from the survivors
    surv = [1, 2, 3, 4, 6, 7, 8, 9, 10, 11]
    b, m = _batch(k, p, nobj, S, pitch, 2)
    coef = rn.matmul(m[[12, 13]], rn.invert(m[surv]))
    b[6, 12, 500] ^= 0x11
    ok = oracle.verify_batch(coef, surv, [12, 13], b.reshape(-1), n * pitch, pitch, S, nobj, nthreads=2)
    assert ok.tolist() == [1] * 6 + [0]


def test_cpu_baseline_checked_get_forms():
    w = dict(bench.WORKLOADS["dec4_get"])
    w["nbytes"] = 40 << 10
    k, p = w["k"], w["p"]
    n = k + p
    S = (w["nbytes"] + k - 1) // k
    pitch = (S + 255) // 256 * 256
    gpu_sample, m = _batch(k, p, 6, S, pitch, 3)
    sample = gpu_sample.copy()
    sample[:, list(w["lost"])] = 0
    surv = [i for i in range(n) if i not in w["lost"]][:k]
    inv_rows = rn.invert(m[surv])[list(w["lost"])]
    cpu = bench.cpu_baseline(w, sample, gpu_sample, m, inv_rows, budget_s=0.5, threads=2, windows=1,
                             fused_checks=2)
    assert cpu["kind"] == "port" and cpu["value"] > 0
    assert cpu["fused_form_GiBps"] > 0
    assert "Reconstruct then Verify" in cpu["decode_form"]
    assert "bit-exact vs GPU (parity, and the rows the GPU rebuilt from garbage in the work check): True" \
        in cpu["sample"]


def test_pass_symbol_follows_the_library_dispatch():
    """bench.py names the kernel a pass runs as gf_kernels.hip dispatches it:
    gf_apply_tri for its (K, R, KI) shapes on rows past 128 16-B vectors of an
    object-major batch, gf_apply_kernel otherwise (the names rocprofv3 and the
    live PMC passes match on)."""
    S4 = (4 << 20) // 10 + 1
    assert bench.pass_symbol(12, 4, 2, S4) == "gf_apply_tri<12,4>"      # dec4_get
    assert bench.pass_symbol(14, 4, 4, S4) == "gf_apply_tri<14,4>"      # upstream Verify
    assert bench.pass_symbol(10, 2, 0, 104858) == "gf_apply_kernel<10,2>"  # headline
    assert bench.pass_symbol(12, 4, 2, 2048) == "gf_apply_kernel<12,4>"   # 128 vectors: small form
    assert bench.pass_symbol(12, 4, 2, 2049) == "gf_apply_tri<12,4>"
    assert bench.pass_symbol(12, 4, 2, S4, shard_major=True) == "gf_apply_kernel<12,4>"
    assert bench.pass_symbol(12, 4, 1, S4) == "gf_apply_kernel<12,4>"     # not an instantiated shape


def test_pmc_sq_summary_from_a_counter_csv(tmp_path):
    """tools/pmc_sq.py (bench.py's live SQ pass and the committed r06_sq_*
    summaries): per-dispatch counters folded per kernel, VALUBusy = VALU
    quad-cycles x 4 over 1024 SIMDs' cycles, the held clock = GRBM_GUI_ACTIVE
    / 8 / dispatch time."""
    import csv
    import sys
    sys.path.insert(0, str(bench.ROOT) + "/tools")
    from pmc_sq import per_dispatch, summarise
    name = "void rsgpu::gf_apply_tri<12, 4, 2, 4>(rsgpu::TriArgs<12>)"
    vals = {"SQ_WAVES": 1000, "SQ_WAVE_CYCLES": 4_000_000, "SQ_ACTIVE_INST_ANY": 1_200_000,
            "SQ_ACTIVE_INST_VALU": 1_024_000, "SQ_WAIT_ANY": 2_000_000, "SQ_WAIT_INST_ANY": 800_000,
            "SQ_INSTS_VALU": 976_000, "SQ_INSTS_SALU": 90_000, "GRBM_GUI_ACTIVE": 8 * 4000, "GRBM_COUNT": 8 * 4000}
    f = tmp_path / "run_counter_collection.csv"
    with open(f, "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value", "Start_Timestamp",
                    "End_Timestamp"])
        for disp in (1, 2):
            for c, v in vals.items():
                w.writerow([disp, name, c, v, 1000, 1000 + 2000])  # 2 us per dispatch
    d = per_dispatch(str(f))
    assert list(d) == ["gf_apply_tri<12,4>"] and len(d["gf_apply_tri<12,4>"]) == 2
    sm = summarise(d["gf_apply_tri<12,4>"])
    assert sm["valu_insts_per_wave"] == 976.0
    assert sm["valu_active_share_of_simd_cycles"] == round(4 * 1_024_000 / (1024 * 4000), 4)  # 1.0
    assert sm["wait_any_over_wave_cycles"] == 0.5
    assert sm["clock_GHz_pass_duration"] == 2.0  # 4000 cycles / 2000 ns
