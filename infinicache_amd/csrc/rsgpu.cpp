// rsgpu.cpp — host side of the C ABI in include/rsgpu.h.
//
// Mirrors reedsolomon.Encoder v1.9.3 (the interface Client.EC holds,
// /root/reference/client/client.go:38; factory /root/reference/client/ec.go:14-24):
//   * rsgpu_create       <- reedsolomon.New (buildMatrix; ErrInvShardNum /
//                           ErrMaxShardNum checks)
//   * rsgpu_encode       <- Encode           (ecRedis.go:390)
//   * rsgpu_verify       <- Verify           (ecRedis.go:395,406,420)
//   * rsgpu_reconstruct  <- Reconstruct / ReconstructData (ecRedis.go:415)
//   * rsgpu_decode       <- Client.decode's Verify->Reconstruct->Verify
//                           (ecRedis.go:404-427), fused into one pass
//   * rsgpu_update       <- Update
// Argument checks follow upstream precedence (length check, then
// checkShards).  All GF arithmetic runs in gf_kernels.hip; this file only
// derives per-operation coefficient matrices (including upstream's
// per-erasure-pattern inverse cache, inversionTree) and moves bytes.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/rsgpu.h"
#include "gf256.h"
#include "gf_apply.h"
#include "gf_masked.h"
#include "gf_worker.h"

namespace rsgpu {

const GF &gf() {
    static const GF g;
    return g;
}

bool gf_invert(const uint8_t *in, int n, uint8_t *out) {
    const GF &g = gf();
    const int cols = 2 * n;
    std::vector<uint8_t> w((size_t)n * cols, 0);
    for (int r = 0; r < n; ++r) {
        std::memcpy(&w[(size_t)r * cols], in + (size_t)r * n, n);
        w[(size_t)r * cols + n + r] = 1;
    }
    for (int r = 0; r < n; ++r) {
        uint8_t *row = &w[(size_t)r * cols];
        if (row[r] == 0) {
            for (int rb = r + 1; rb < n; ++rb)
                if (w[(size_t)rb * cols + r]) {
                    std::swap_ranges(row, row + cols, &w[(size_t)rb * cols]);
                    break;
                }
        }
        if (row[r] == 0) return false;
        const uint8_t s = g.div(1, row[r]);
        for (int c = 0; c < cols; ++c) row[c] = g.mul(row[c], s);
        for (int rb = 0; rb < n; ++rb) {
            if (rb == r) continue;
            uint8_t *o = &w[(size_t)rb * cols];
            const uint8_t f = o[r];
            if (f)
                for (int c = 0; c < cols; ++c) o[c] ^= g.mul(f, row[c]);
        }
    }
    for (int r = 0; r < n; ++r) std::memcpy(out + (size_t)r * n, &w[(size_t)r * cols + n], n);
    return true;
}

bool gf_build_matrix(int k, int p, unsigned kind, std::vector<uint8_t> &out) {
    const GF &g = gf();
    const int n = k + p;
    out.assign((size_t)n * k, 0);
    if (kind == RSGPU_MATRIX_CAUCHY || kind == RSGPU_MATRIX_PAR1) {
        for (int r = 0; r < n; ++r)
            for (int c = 0; c < k; ++c)
                out[(size_t)r * k + c] = r < k ? (uint8_t)(r == c)
                                       : kind == RSGPU_MATRIX_CAUCHY ? g.div(1, (uint8_t)(r ^ c))
                                                                     : g.pow((uint8_t)(c + 1), r - k);
        return true;
    }
    std::vector<uint8_t> vm((size_t)n * k), inv((size_t)k * k);
    for (int r = 0; r < n; ++r)
        for (int c = 0; c < k; ++c) vm[(size_t)r * k + c] = g.pow((uint8_t)r, c);
    if (!gf_invert(vm.data(), k, inv.data())) return false;
    for (int r = 0; r < n; ++r)
        for (int c = 0; c < k; ++c) {
            uint8_t a = 0;
            for (int i = 0; i < k; ++i) a ^= g.mul(vm[(size_t)r * k + i], inv[(size_t)i * k + c]);
            out[(size_t)r * k + c] = a;
        }
    return true;
}

}  // namespace rsgpu

#include "ctx.h"

using namespace rsgpu;

// Multi-device contexts forward every compute call to one of their per-device
// contexts: per-object host calls round-robin (concurrent EcSet/EcGet callers
// spread over the GPUs and their PCIe links), device-resident calls to the
// device that owns the memory.
#define RSGPU_FORWARD_RR(fn, ...) \
    if (ctx && ctx->multi()) return fn(ctx->pick(), __VA_ARGS__)
#define RSGPU_FORWARD_DEV(fn, ptr, ...)                  \
    if (ctx && ctx->multi()) {                           \
        rsgpu_ctx *sub_ = ctx->sub_for(ptr);             \
        if (!sub_) return RSGPU_ERR_INVALID_ARG;         \
        return fn(sub_, __VA_ARGS__);                    \
    }

namespace rsgpu {

// upstream checkShards(shards, nilok): size = first non-empty length
int check_shards(const size_t *lens, int n, bool nilok, size_t *size) {
    size_t s = 0;
    for (int i = 0; i < n; ++i)
        if (lens[i]) { s = lens[i]; break; }
    if (s == 0) return RSGPU_ERR_SHARD_NO_DATA;
    for (int i = 0; i < n; ++i)
        if (lens[i] != s && (lens[i] != 0 || !nilok)) return RSGPU_ERR_SHARD_SIZE;
    *size = s;
    return RSGPU_OK;
}

}  // namespace rsgpu

namespace {

#ifdef RSGPU_MEASURE_DMA_SPLIT
// The copy-engine share of a split per-object call, percent of the columns
// (run_host_once; RSGPU_DMA_SPLIT, read once; 0 = off), for objects whose
// shards are at least kDmaSplitMin bytes.  A measurement build only
// (make HIPFLAGS+=-DRSGPU_MEASURE_DMA_SPLIT): measured 4x slower and not kept.
constexpr size_t kDmaSplitMin = (size_t)64 << 10;
int dma_split_pct() {
    static const int v = [] {
        const char *e = std::getenv("RSGPU_DMA_SPLIT");
        const int x = e ? std::atoi(e) : 0;
        return x > 0 && x < 100 ? x : 0;
    }();
    return v;
}
#endif

// Runs `plan` over one object staged from host buffers.  in_src[c] is the
// host source of staging row plan.in_rows[c]; out_dst[r] receives written
// row r.  Returns the mismatch flag in *bad when the plan has check rows.
// One object through the device: inputs H2D, the plan's pass, written rows
// D2H, the check flag.  The device image is byte-packed (row i at i*size, the
// pass's packed mode, gf_device.h store_row), so host rows move as plain 1D
// copies with no device-side repack:
//   * inputs inside one pinned range at base + row*size (Split's layout) are
//     read by the pass itself over PCIe (zero-copy, no H2D command) when the
//     range is readable up to the last row's final 16-B vector, else go as
//     ONE DMA of the row span;
//   * written rows at their Split positions in one pinned range are stored
//     by the pass straight into it (zero-copy, no D2H command);
//   * other pinned rows go as one DMA per run of rows consecutive in both the
//     object and host memory;
//   * pageable rows are staged into the slot's pinned buffer (same packed
//     layout) and go as one DMA;
//   * written rows come back the same way (pinned: straight into the caller's
//     buffers).
//   * `then` (optional): a second plan run on the same device image after the
//     first one's rows went back, whose check flag lands in *then_bad
//     (Client.encode's Verify right after Encode: no second upload).
int run_host_once(rsgpu_ctx *ctx, Plan &plan, int nrows_staged, size_t size,
                  const std::vector<const uint8_t *> &in_src, const std::vector<uint8_t *> &out_dst,
                  uint32_t *bad, Plan *then, uint32_t *then_bad) {
    if (then && (plan.nw < plan.R || then->nw != 0)) return RSGPU_ERR_INVALID_ARG;  // see `then` above
    // row offsets are 32-bit inside the pass (Pass::in_off / out_off)
    if ((size_t)nrows_staged * size + 16 >= ((size_t)1 << 32)) return RSGPU_ERR_INVALID_ARG;
    std::unique_ptr<Slot> s;
    int e = ctx->get_slot(round_up((size_t)nrows_staged * size + 16, 256), s);
    if (e) return e;
    bool pin_in = true, pin_out = true;
    for (int c = 0; c < plan.K && pin_in; ++c) pin_in = host_pinned(in_src[c], size);
    for (int r = 0; r < plan.nw && pin_out; ++r) pin_out = host_pinned(out_dst[r], size);
    int rlo = plan.in_rows[0], rhi = plan.in_rows[0];
    for (int c = 1; c < plan.K; ++c) {
        rlo = std::min(rlo, plan.in_rows[c]);
        rhi = std::max(rhi, plan.in_rows[c]);
    }
    const size_t span = (size_t)(rhi - rlo + 1) * size;
    // rows [i, j) of a list form a run: consecutive object rows at
    // consecutive host addresses
    auto run_end = [&](const std::vector<int> &rows, size_t i, auto host) {
        size_t j = i + 1;
        while (j < rows.size() && rows[j] == rows[j - 1] + 1 && host(j) == host(j - 1) + size) ++j;
        return j;
    };
    hipError_t he = hipSuccess;
    [[maybe_unused]] bool staged_in = false;  // the inputs were copied into the slot's pinned image s->h (the DMA-split measurement reads it)
    const uint8_t *span0 = in_src[0] - (size_t)(plan.in_rows[0] - rlo) * size;
    bool split = pin_in;
    for (int c = 0; c < plan.K && split; ++c)
        split = in_src[c] == span0 + (size_t)(plan.in_rows[c] - rlo) * size;
    split = split && host_pinned(span0, span);
    // Zero-copy inputs: a pinned Split-layout input span is read by the pass
    // itself over PCIe (no H2D command).  The last 16-B vector of a row may
    // run up to 15 bytes past it, so the pinned range must be readable up to
    // rhi*size + roundup16(size) (rsgpu_host_alloc leaves that slack).  A
    // following plan (`then`) reads the image, so the pass copies the input
    // rows into it as well.
    Layout L{s->d, 0, size, size, 1};
    L.slack = true;  // the slot holds nrows_staged*size + 16 bytes at least
    if (split && plan.K <= kRedirectMaxK) {
        const size_t first = (size_t)rlo * size, need = (size_t)rhi * size + round_up(size, 16);
        if (const uint8_t *d = (const uint8_t *)host_device_ptr(span0, need - first)) {
            L.in_base = d - first;
            L.in_span = need;
            L.copy_in = then != nullptr;
        }
    }
    if (L.in_base) {
        // nothing to copy
    } else if (split) {
        he = hipMemcpyAsync(s->d + (size_t)rlo * size, span0, span, hipMemcpyHostToDevice, s->stream);
    } else if (pin_in) {
        auto src = [&](size_t c) { return in_src[c]; };
        for (size_t i = 0; i < (size_t)plan.K && he == hipSuccess;) {
            const size_t j = run_end(plan.in_rows, i, src);
            he = hipMemcpyAsync(s->d + (size_t)plan.in_rows[i] * size, in_src[i], (j - i) * size,
                                hipMemcpyHostToDevice, s->stream);
            i = j;
        }
    } else {
        std::vector<CopyJob> cp((size_t)plan.K);
        for (int c = 0; c < plan.K; ++c) cp[c] = {s->h + (size_t)plan.in_rows[c] * size, in_src[c], size};
        copy_rows(cp.data(), cp.size());
        staged_in = true;
        if (plan.K <= kRedirectMaxK && s->hdev) {
            // the pass reads the pinned staging image in place (zero-copy);
            // the slot holds nrows_staged*size + 16 bytes at least
            L.in_base = s->hdev;
            L.in_span = (size_t)rhi * size + round_up(size, 16);
            L.copy_in = then != nullptr;
        } else {
            he = hipMemcpyAsync(s->d + (size_t)rlo * size, s->h + (size_t)rlo * size, span,
                                hipMemcpyHostToDevice, s->stream);
        }
    }
    // The check flag is a mapped pinned word: zeroed here, written by the
    // kernels over PCIe, read after the sync (no memset, no D2H command).
    *s->h_bad = 0;
    // Zero-copy outputs: when every written row lies in one pinned range at
    // its Split position (row r at obase + r*size, the image's own layout),
    // the pass stores straight into it over PCIe and the D2H commands go
    // away.  A following plan (`then`) reads the image, so the rows are then
    // stored to the image as well.
    std::vector<int> orows(plan.out_rows.begin(), plan.out_rows.begin() + plan.nw);
    if (pin_out && plan.nw > 0 && plan.K <= kRedirectMaxK) {
        const uint8_t *ob = out_dst[0] - (size_t)orows[0] * size;
        int lo = orows[0], hi = orows[0];
        bool split_out = true;
        for (size_t r = 0; r < orows.size() && split_out; ++r) {
            split_out = out_dst[r] == ob + (size_t)orows[r] * size;
            lo = std::min(lo, orows[r]);
            hi = std::max(hi, orows[r]);
        }
        if (split_out) {
            if (uint8_t *d = (uint8_t *)host_device_ptr(ob + (size_t)lo * size, (size_t)(hi - lo + 1) * size)) {
                L.out_base = d - (size_t)lo * size;
                L.out_dual = then != nullptr;
            }
        }
    } else if (!pin_out && plan.nw > 0 && plan.K <= kRedirectMaxK && s->hdev) {
        // pageable outputs: the pass stores into the pinned staging image in
        // place (zero-copy), copied out to the caller after the sync
        L.out_base = s->hdev;
        L.out_dual = then != nullptr;
    }
#ifdef RSGPU_MEASURE_DMA_SPLIT
    bool two = false;
    // Copy engine beside the zero-copy pass (RSGPU_DMA_SPLIT=<percent>; a
    // measurement build only, not in the product library): the input rows' last columns [cb, size)
    // go H2D on a second stream and a second pass codes them from HBM while
    // the first pass codes columns [0, cb) over PCIe.  Measured 4x slower at
    // 1 MiB — each row slice's copy command carries a fixed ~10-14 us — and
    // not kept (profiles/r05_dma_split_not_kept/).  Every operation is a byte-column map.  The second share is
    // whole 16-B vectors, so its last vector ends at the row's end; the first
    // share's last vector may reach into the second's first vector, where
    // both passes store the same bytes (the coding of the same input
    // columns).  Both passes set the same mapped check flag.
    if (he == hipSuccess && L.in_base && size >= kDmaSplitMin && dma_split_pct() > 0) {
        const size_t blen = (size * (size_t)dma_split_pct() / 100) & ~(size_t)15;
        if (blen >= 4096 && blen + 16 <= size) {
            const size_t cb = size - blen;
            if (!s->stream2 && (he = hipStreamCreateWithFlags(&s->stream2, hipStreamNonBlocking)) != hipSuccess)
                s->stream2 = nullptr;
            if (he == hipSuccess && !s->ev2 && (he = hipEventCreateWithFlags(&s->ev2, hipEventDisableTiming)) != hipSuccess)
                s->ev2 = nullptr;
            for (int c = 0; c < plan.K && he == hipSuccess; ++c) {
                const size_t ro = (size_t)plan.in_rows[c] * size;
                const uint8_t *src = staged_in ? s->h + ro : in_src[c];
                he = hipMemcpyAsync(s->d + ro + cb, src + cb, blen, hipMemcpyHostToDevice, s->stream2);
            }
            if (he == hipSuccess) {
                Layout B{s->d + cb, 0, size, blen, 1};
                B.slack = true;
                if (L.out_base) {
                    B.out_base = L.out_base + cb;
                    B.out_dual = L.out_dual;
                }
                he = launch_plan(plan, B, s->m_bad, s->stream2);
            }
            if (he == hipSuccess) {
                L.shard_len = cb;
                two = true;
            }
        }
    }
#endif
    if (he == hipSuccess) he = launch_plan(plan, L, s->m_bad, s->stream);
    // what follows on the slot's stream (D2H of written rows, the `then`
    // pass over the image) waits for the second share
#ifdef RSGPU_MEASURE_DMA_SPLIT
    if (two && he == hipSuccess && (!L.out_base || then)) {
        he = hipEventRecord(s->ev2, s->stream2);
        if (he == hipSuccess) he = hipStreamWaitEvent(s->stream, s->ev2, 0);
    }
#endif
    auto dst = [&](size_t r) {
        return pin_out ? (const uint8_t *)out_dst[r] : (const uint8_t *)s->h + (size_t)orows[r] * size;
    };
    for (size_t i = 0; i < orows.size() && he == hipSuccess && !L.out_base;) {
        const size_t j = run_end(orows, i, dst);
        he = hipMemcpyAsync((void *)dst(i), s->d + (size_t)orows[i] * size, (j - i) * size,
                            hipMemcpyDeviceToHost, s->stream);
        i = j;
    }
    if (then && he == hipSuccess) {  // check-only plan (nw == 0) on the image as it stands
        // the first plan has no check rows (run_host's contract with `then`):
        // its pass already cleared the flag.  (Running the written rows' D2H
        // on a side stream to overlap this kernel was measured slower: 67.5 ->
        // 85.7 us per fused encode+verify; the cross-stream event and second
        // sync cost more than the overlap.)
        Layout img{s->d, 0, size, size, 1};
        img.slack = true;
        he = launch_plan(*then, img, s->m_bad, s->stream);
    }
#ifdef RSGPU_MEASURE_DMA_SPLIT
    if (he == hipSuccess && two) he = hipStreamSynchronize(s->stream2);
#endif
    if (he == hipSuccess) he = hipStreamSynchronize(s->stream);
    if (he != hipSuccess) {
        (void)hipStreamSynchronize(s->stream);  // nothing in flight may touch a pooled slot
#ifdef RSGPU_MEASURE_DMA_SPLIT
        if (s->stream2) (void)hipStreamSynchronize(s->stream2);
#endif
        ctx->put_slot(std::move(s));
        return hip_fail(he, "run_host");
    }
    if (!pin_out) {
        std::vector<CopyJob> cp((size_t)plan.nw);
        for (int r = 0; r < plan.nw; ++r) cp[r] = {out_dst[r], s->h + (size_t)orows[r] * size, size};
        copy_rows(cp.data(), cp.size());
    }
    if (bad) *bad = plan.nw < plan.R ? *s->h_bad : 0;
    if (then_bad) *then_bad = *s->h_bad;
    ctx->put_slot(std::move(s));
    return RSGPU_OK;
}

// run_host_once for objects of any size.  Every operation is a byte-column
// map (output byte b of a row depends on byte b of the input rows only), so
// an object whose staged image would pass slab_bytes() — or the 4 GiB a
// pass can address — is coded as consecutive column slabs [b0, b0 + L) of
// every row, each one run_host_once on the rows' pointers offset by b0.
// Upstream codes shards of any length (reedsolomon.Encoder has no size
// limit); the slabs also bound the staging slot a huge object takes.  Check
// flags are OR-ed over the slabs (Verify fails if any column mismatches).
int run_host(rsgpu_ctx *ctx, Plan &plan, int nrows_staged, size_t size,
             const std::vector<const uint8_t *> &in_src, const std::vector<uint8_t *> &out_dst,
             uint32_t *bad, Plan *then = nullptr, uint32_t *then_bad = nullptr) {
    const size_t lim = slab_bytes();
    if ((size_t)nrows_staged * size + 16 <= lim)
        return run_host_once(ctx, plan, nrows_staged, size, in_src, out_dst, bad, then, then_bad);
    const size_t L = std::max<size_t>(4096, ((lim - 16) / (size_t)nrows_staged) & ~(size_t)4095);
    std::vector<const uint8_t *> in(in_src.size());
    std::vector<uint8_t *> out(out_dst.size());
    uint32_t bad_all = 0, then_all = 0;
    for (size_t b0 = 0; b0 < size; b0 += L) {
        const size_t l = std::min(L, size - b0);
        for (size_t i = 0; i < in.size(); ++i) in[i] = in_src[i] ? in_src[i] + b0 : nullptr;
        for (size_t i = 0; i < out.size(); ++i) out[i] = out_dst[i] ? out_dst[i] + b0 : nullptr;
        uint32_t b = 0, tb = 0;
        const int e = run_host_once(ctx, plan, nrows_staged, l, in, out, bad ? &b : nullptr, then,
                                    then_bad ? &tb : nullptr);
        if (e) return e;
        bad_all |= b;
        then_all |= tb;
    }
    if (bad) *bad = bad_all;
    if (then_bad) *then_bad = then_all;
    return RSGPU_OK;
}

// ------------------------------------------------- device pattern atlas
// Every erasure pattern of the code, for one operation, as the device kernels
// of gf_masked.h read it: the pattern table over all 2^n present masks, one
// PatRec per (pattern, sub-pass) and its [kmax][R] kernel tables.  Built once
// per context and mode (upstream's inversionTree holds the same inverses,
// filled lazily), uploaded, then immutable.
constexpr size_t kAtlasMaxBytes = (size_t)256 << 20;      // *_dev_masks: no other path
constexpr size_t kAtlasHostFlagBytes = (size_t)32 << 20;  // *_dev_multi: host-planned path beyond

int build_atlas_host(rsgpu_ctx *ctx, AtlasMode mode, Atlas &A) {
    const int n = ctx->n, k = ctx->k;
    const bool check = mode == kAtlasDecode, data_only = mode == kAtlasData;
    // refuse before enumerating 2^n patterns whose tables could not be kept
    if (atlas_estimate(k, ctx->p, check) > kAtlasMaxBytes) return RSGPU_ERR_NOT_IMPLEMENTED;
    const size_t nm = (size_t)1 << n;
    struct Ent {
        int K, R, nw, ki;
        std::vector<uint8_t> coef;
        std::vector<int> out_rows, in_rows;
    };
    std::vector<int32_t> pat(nm);
    std::vector<Ent> ents;
    std::vector<uint8_t> present(n);
    int maxR = 0;
    for (size_t mask = 0; mask < nm; ++mask) {
        const int np = __builtin_popcountll(mask);
        if (np < k) {
            pat[mask] = kPatTooFew;
            continue;
        }
        for (int i = 0; i < n; ++i) present[i] = (mask >> i) & 1;
        Plan pl;
        if (np == n) {
            if (!check) {  // Reconstruct with every shard present: nothing to do
                pat[mask] = kPatNothing;
                continue;
            }
            ctx->build_verify(pl);  // Client.decode's first Verify
        } else {
            const int e = ctx->build_reconstruct(present.data(), data_only, check, pl);
            if (e == RSGPU_ERR_SINGULAR) {
                pat[mask] = kPatSingular;
                continue;
            }
            if (e) return e;
        }
        if (pl.R == 0) {  // ReconstructData with only parity missing
            pat[mask] = kPatNothing;
            continue;
        }
        pat[mask] = (int32_t)ents.size();
        ents.push_back({pl.K, pl.R, pl.nw, pl.identity_inputs(), pl.coef, pl.out_rows, pl.in_rows});
        maxR = std::max(maxR, pl.R);
    }
    const int R = std::max(1, std::min(4, maxR)), nsub = std::max(1, (maxR + 3) / 4);
    const int kmax = check ? n : k;
    const size_t nrec = ents.size() * (size_t)nsub, tw = (size_t)kmax * R * kCoefWords;
    if (nrec * tw * 4 > kAtlasMaxBytes) return RSGPU_ERR_NOT_IMPLEMENTED;  // bound the atlas
    std::vector<uint32_t> ct(256 * kCoefWords);
    for (int c = 0; c < 256; ++c) coef_tables((uint8_t)c, &ct[(size_t)c * kCoefWords]);
    std::vector<PatRec> recs(std::max<size_t>(nrec, 1));
    std::memset(recs.data(), 0, recs.size() * sizeof(PatRec));
    std::vector<uint32_t> tabs(std::max<size_t>(nrec * tw, 1), 0);
    for (size_t i = 0; i < ents.size(); ++i) {
        const Ent &e = ents[i];
        int nchk = 0;
        for (int s = 0; s < nsub; ++s) {
            const int nr = std::max(0, std::min(4, e.R - 4 * s)), nw = std::max(0, std::min(nr, e.nw - 4 * s));
            nchk += nw < nr;
        }
        for (int s = 0; s < nsub; ++s) {
            const int r0 = 4 * s;
            const int nr = std::max(0, std::min(4, e.R - r0)), nw = std::max(0, std::min(nr, e.nw - r0));
            PatRec &rc = recs[i * nsub + s];
            rc.kact = (uint8_t)e.K;
            rc.nr = (uint8_t)nr;
            rc.nw = (uint8_t)nw;
            // identity inputs feed the plan's last rows: usable in its last sub-pass
            rc.ki = (uint8_t)(nr > 0 && r0 + nr == e.R ? std::min(e.ki, nr) : 0);
            rc.nchk = (uint8_t)nchk;
            for (int c = 0; c < e.K; ++c) rc.in_row[c] = (uint8_t)e.in_rows[c];
            uint32_t *tb = &tabs[(i * nsub + s) * tw];
            for (int r = 0; r < nr; ++r) {
                if (r < nw) rc.out_row[r] = (uint8_t)e.out_rows[r0 + r];
                for (int c = 0; c < e.K; ++c) {
                    const uint8_t cf = e.coef[(size_t)(r0 + r) * e.K + c];
                    rc.coef[r][c] = cf;
                    std::memcpy(&tb[((size_t)c * R + r) * kCoefWords], &ct[(size_t)cf * kCoefWords], kCoefWords * 4);
                }
            }
        }
    }
    A.h_pat = std::move(pat);
    A.h_recs.resize(recs.size() * sizeof(PatRec));
    std::memcpy(A.h_recs.data(), recs.data(), A.h_recs.size());
    A.h_tabs = std::move(tabs);
    AtlasView &v = A.view;
    v.n = n;
    v.kmax = kmax;
    v.R = R;
    v.nsub = nsub;
    v.kfix = check ? 0 : k;
    v.kcap = k;
    return RSGPU_OK;
}

// Uploads the host atlas H (this context's own, or its parent's when shared)
// into D, this context's device copy.  On failure nothing stays allocated.
int upload_atlas(rsgpu_ctx *ctx, const Atlas &H, Atlas &D) {
    hipError_t e = hipMalloc(&D.d_pat, H.h_pat.size() * 4);
    if (e == hipSuccess) e = upload(D.d_pat, H.h_pat.data(), H.h_pat.size() * 4);
    if (e == hipSuccess) e = hipMalloc(&D.d_recs, H.h_recs.size());
    if (e == hipSuccess) e = upload(D.d_recs, H.h_recs.data(), H.h_recs.size());
    if (e == hipSuccess) e = hipMalloc(&D.d_tabs, H.h_tabs.size() * 4);
    if (e == hipSuccess) e = upload(D.d_tabs, H.h_tabs.data(), H.h_tabs.size() * 4);
    if (e != hipSuccess) {
        D.free_dev();
        return hip_fail(e, "atlas upload");
    }
    D.view = H.view;
    D.view.pat = D.d_pat;
    D.view.recs = D.d_recs;
    D.view.tabs = D.d_tabs;
    D.view.ctab = ctx->d_ctab;
    return RSGPU_OK;
}

// huge: the caller codes objects whose rows span 4 GiB or more (launch_plan
// codes them in column slabs); the mixed-pattern calls do not
int check_layout(const rsgpu_ctx *ctx, const void *base, size_t shard_len, size_t pitch,
                 size_t obj_stride, int nobj, bool huge = false) {
    if (!base || nobj < 0) return RSGPU_ERR_INVALID_ARG;
    if (shard_len == 0) return RSGPU_ERR_SHARD_NO_DATA;
    // any alignment: a pitch below 16 * ceil(S / 16) stores the last vector
    // of a row in 8/4/2/1-byte pieces (store_row); 16-B aligned rows and
    // objects are the fast path
    if (pitch < shard_len) return RSGPU_ERR_INVALID_ARG;
    if (!huge && (size_t)ctx->n * pitch >= ((size_t)1 << 32)) return RSGPU_ERR_INVALID_ARG;
    // objects must not overlap: object-major ([object][shard]: each object's
    // rows within its stride) or shard-major ([shard][object]: each shard row
    // holds every object's piece)
    if (nobj > 1 && obj_stride < (size_t)ctx->n * pitch &&
        !(obj_stride >= shard_len && pitch >= (size_t)(nobj - 1) * obj_stride + shard_len))
        return RSGPU_ERR_INVALID_ARG;
    return RSGPU_OK;
}

}  // namespace

rsgpu_ctx *rsgpu_ctx::sub_for(const void *dev_ptr) {
    hipPointerAttribute_t at;
    if (!dev_ptr || hipPointerGetAttributes(&at, dev_ptr) != hipSuccess) return nullptr;
    // a device listed several times: its entries take turns
    const unsigned start = rr.fetch_add(1, std::memory_order_relaxed);
    for (size_t i = 0; i < subs.size(); ++i) {
        rsgpu_ctx *c = subs[(start + i) % subs.size()].get();
        if (c->device == at.device) return c;
    }
    return nullptr;
}

size_t rsgpu::atlas_estimate(int k, int p, bool check) {
    const int n = k + p;
    double npat = 0, c = 1;  // sum over j >= k of C(n, j)
    for (int j = 0; j <= n; ++j) {
        if (j >= k) npat += c;
        c = c * (n - j) / (j + 1);
    }
    const int R = std::min(4, p), nsub = (p + 3) / 4, kmax = check ? n : k;
    const double b = npat * nsub * ((double)kmax * R * kCoefWords * 4 + sizeof(PatRec));
    return b > 1e18 ? (size_t)-1 : (size_t)b;
}

int rsgpu_ctx::atlas_host(AtlasMode mode, const Atlas *&out) {
    if (n > kAtlasMaxN) return RSGPU_ERR_NOT_IMPLEMENTED;
    rsgpu_ctx *owner = parent ? parent : this;  // one host build per code
    Atlas &A = owner->atlas[mode];
    std::call_once(A.host_once, [&] { A.host_err = build_atlas_host(owner, mode, A); });
    out = &A;
    return A.host_err;
}

int rsgpu_ctx::atlas_view(AtlasMode mode, AtlasView &out) {
    const Atlas *ah;
    int e = atlas_host(mode, ah);
    if (e) return e;
    {
        std::lock_guard<std::mutex> g(ctab_mu);
        if (!d_ctab) {
            std::vector<uint32_t> t(256 * kCtabStride, 0);
            for (int c = 0; c < 256; ++c) coef_tables((uint8_t)c, &t[(size_t)c * kCtabStride]);
            uint32_t *d = nullptr;
            hipError_t he = hipMalloc(&d, t.size() * 4);
            if (he == hipSuccess) he = upload(d, t.data(), t.size() * 4);
            if (he != hipSuccess) {
                retire(d, false);
                return hip_fail(he, "atlas coefficient table");  // retried by the next call
            }
            d_ctab = d;
        }
    }
    Atlas &D = atlas[mode];
    std::lock_guard<std::mutex> g(D.dev_mu);
    if (!D.dev_done) {
        if ((e = upload_atlas(this, *ah, D))) return e;  // retried by the next call
        D.dev_done = true;
        // a context of its own (no sub-contexts share its host atlas) drops
        // the host images once they are on the device
        if (ah == &D && subs.empty() && !parent) {
            std::vector<uint8_t>().swap(D.h_recs);
            std::vector<uint32_t>().swap(D.h_tabs);
        }
    }
    out = D.view;
    return RSGPU_OK;
}

namespace {

// launch_masked with the multi-reporter status scratch the decode needs
int run_masked(rsgpu_ctx *ctx, const AtlasView &A, AtlasMode mode, const Layout &L, const uint32_t *d_masks,
               uint32_t *d_status, hipStream_t st) {
    if (mode != kAtlasDecode) {
        HIP_TRY(launch_masked(A, L, d_masks, d_status, nullptr, nullptr, st));
        return RSGPU_OK;
    }
    // Inside a stream capture (a HIP graph): the scratch ring's event waits
    // and first-use allocations are not capturable, and a replay must not
    // share a ring slot with later calls; the counters then come from a
    // stream-ordered allocation the graph owns (alloc + memset + free nodes)
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cs) == hipSuccess && cs == hipStreamCaptureStatusActive) {
        uint32_t *tmp = nullptr;
        HIP_TRY(hipMallocAsync((void **)&tmp, (size_t)L.nobj * 2 * sizeof(uint32_t), st));
        hipError_t e = hipMemsetAsync(tmp, 0, (size_t)L.nobj * 2 * sizeof(uint32_t), st);
        if (e == hipSuccess) e = launch_masked(A, L, d_masks, d_status, tmp, tmp + L.nobj, st);
        const hipError_t f = hipFreeAsync(tmp, st);
        if (e != hipSuccess) return hip_fail(e, "launch_masked (capture)");
        if (f != hipSuccess) return hip_fail(f, "status scratch (capture)");
        return RSGPU_OK;
    }
    StatusScratch::Slot *sc = nullptr;
    HIP_TRY(ctx->scratch.acquire((size_t)L.nobj, st, sc));
    const hipError_t e = launch_masked(A, L, d_masks, d_status, sc->d, sc->d + sc->cap, st);
    const hipError_t e2 = ctx->scratch.release(sc, st, e == hipSuccess);
    if (e != hipSuccess) return hip_fail(e, "launch_masked");
    if (e2 != hipSuccess) return hip_fail(e2, "status scratch");
    return RSGPU_OK;
}

// *_dev_masks for codes without a device atlas (17-32 shards, or an atlas
// past its size bound, e.g. RS(2+14)): the masks come to the host (one
// stream synchronisation), objects are grouped by pattern with the same
// per-object statuses as the atlas (too few shards 2, singular 3, untouched),
// and the groups are coded by the host-planned mixed-pattern launches.
int dev_masks_host(rsgpu_ctx *ctx, const Layout &L, const uint32_t *d_masks, AtlasMode mode, uint32_t *d_status,
                   hipStream_t st) {
    const int n = ctx->n, nobj = L.nobj;
    const uint32_t nmask = n >= 32 ? ~0u : ((1u << n) - 1);
    std::vector<uint32_t> masks((size_t)nobj), status((size_t)nobj, kStatusOk);
    HIP_TRY(hipMemcpyAsync(masks.data(), d_masks, (size_t)nobj * 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    const bool check = mode == kAtlasDecode, data_only = mode == kAtlasData;
    std::unordered_map<uint32_t, int> slot_of;  // pattern -> plan index, or -1 - status
    std::vector<std::shared_ptr<Plan>> owned;
    std::vector<Plan *> plans;
    std::vector<int> plan_of((size_t)nobj, -1);
    std::vector<uint8_t> pr((size_t)n);
    for (int o = 0; o < nobj; ++o) {
        const uint32_t m = masks[o] & nmask;
        auto ins = slot_of.emplace(m, 0);
        if (ins.second) {  // first object with this pattern
            const int np = __builtin_popcount(m);
            int slot = -1 - (int)kStatusOk;
            if (np < ctx->k) {
                slot = -1 - (int)kStatusTooFew;
            } else if (np < n || check) {
                for (int i = 0; i < n; ++i) pr[i] = (uint8_t)((m >> i) & 1u);
                std::shared_ptr<Plan> p;
                int e = np == n ? (p = ctx->plan_verify(), RSGPU_OK) : ctx->plan_reconstruct(pr.data(), data_only, check, p);
                if (e == RSGPU_ERR_SINGULAR) {
                    slot = -1 - (int)kStatusSingular;
                } else if (e) {
                    return e;
                } else if (p->R > 0) {
                    slot = (int)plans.size();
                    owned.push_back(p);
                    plans.push_back(p.get());
                }
            }
            ins.first->second = slot;
        }
        const int s = ins.first->second;
        if (s >= 0) plan_of[o] = s;
        else status[o] = (uint32_t)(-1 - s);
    }
    // statuses of the objects no launch touches; the coded ones start at 0
    // and the check rows raise theirs to 1
    if (d_status) {  // on the call's stream (ordered with its launches), never the null stream
        HIP_TRY(hipMemcpyAsync(d_status, status.data(), (size_t)nobj * 4, hipMemcpyHostToDevice, st));
        HIP_TRY(hipStreamSynchronize(st));  // `status` is a local
    }
    if (plans.empty()) return RSGPU_OK;
    HIP_TRY(launch_plans_multi(plans, plan_of, L, check ? d_status : nullptr, st, ctx->multi_ws));
    return RSGPU_OK;
}

int dev_masks(rsgpu_ctx *ctx, void *d_base, const uint32_t *d_masks, size_t shard_len, size_t pitch,
              size_t obj_stride, int nobj, AtlasMode mode, uint32_t *d_status, void *stream) {
    if (!ctx || (nobj > 0 && !d_masks)) return RSGPU_ERR_INVALID_ARG;
    int e = check_layout(ctx, d_base, shard_len, pitch, obj_stride, nobj);
    if (e) return e;
    if (((uintptr_t)d_base & 15) || (pitch & 15) || (obj_stride & 15)) return RSGPU_ERR_INVALID_ARG;
    if (ctx->n > 32) return RSGPU_ERR_NOT_IMPLEMENTED;  // masks are 32-bit words
    DeviceGuard dg_;
    if ((e = ctx->use_device(dg_))) return e;
    if (nobj == 0) return RSGPU_OK;
    Layout L{(uint8_t *)d_base, obj_stride, pitch, shard_len, nobj};
    AtlasView A;
    if (ctx->n <= kAtlasMaxN) {
        e = ctx->atlas_view(mode, A);
        if (e == RSGPU_OK) return run_masked(ctx, A, mode, L, d_masks, d_status, (hipStream_t)stream);
        if (e != RSGPU_ERR_NOT_IMPLEMENTED) return e;
    }
    return dev_masks_host(ctx, L, d_masks, mode, d_status, (hipStream_t)stream);
}

}  // namespace

// ============================================================== C ABI

extern "C" {

int rsgpu_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int rsgpu_device_ok(int device) {
    const int n = rsgpu_device_count();
    if (device < 0 || device >= n) return 0;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return 0;
    return std::strncmp(prop.gcnArchName, "gfx950", 6) == 0 ? 1 : 0;
}

const char *rsgpu_strerror(int code) {
    switch (code) {
        case RSGPU_OK: return "ok";
        case RSGPU_ERR_INV_SHARD_NUM: return "cannot create Encoder with zero or less data/parity shards";
        case RSGPU_ERR_MAX_SHARD_NUM: return "cannot create Encoder with more than 256 data+parity shards";
        case RSGPU_ERR_TOO_FEW_SHARDS: return "too few shards given";
        case RSGPU_ERR_SHARD_NO_DATA: return "no shard data";
        case RSGPU_ERR_SHARD_SIZE: return "shard sizes do not match";
        case RSGPU_ERR_SINGULAR: return "matrix is singular";
        case RSGPU_ERR_SHORT_DATA: return "not enough data to fill the number of requested shards";
        case RSGPU_ERR_RECONSTRUCT_REQUIRED: return "reconstruction required as one or more required data shards are nil";
        case RSGPU_ERR_INVALID_INPUT: return "invalid input";
        case RSGPU_ERR_NOT_IMPLEMENTED: return "Not implemented";
        case RSGPU_ERR_INVALID_ARG: return "rsgpu: invalid argument";
        case RSGPU_ERR_NO_DEVICE: return "rsgpu: no usable gfx950 device";
        case RSGPU_ERR_HIP: return "rsgpu: HIP runtime error";
        case RSGPU_ERR_NOMEM: return "rsgpu: out of memory";
        default: return "rsgpu: unknown error";
    }
}

int rsgpu_create(int data_shards, int parity_shards, int device, unsigned flags, rsgpu_ctx **out) {
    if (!out) return RSGPU_ERR_INVALID_ARG;
    *out = nullptr;
    if (data_shards <= 0 || parity_shards <= 0) return RSGPU_ERR_INV_SHARD_NUM;
    if (data_shards + parity_shards > 256) return RSGPU_ERR_MAX_SHARD_NUM;
    const unsigned kind = flags & RSGPU_MATRIX_MASK;
    if (kind > RSGPU_MATRIX_PAR1 || (flags & ~RSGPU_MATRIX_MASK)) return RSGPU_ERR_INVALID_ARG;
    if (device == RSGPU_ALL_DEVICES) {
        // every visible gfx950 device; none: a single-device context on
        // device 0 whose compute calls return RSGPU_ERR_NO_DEVICE
        std::vector<int> devs;
        for (int d = 0; d < rsgpu_device_count(); ++d)
            if (rsgpu_device_ok(d)) devs.push_back(d);
        if (!devs.empty()) return rsgpu_create_multi(data_shards, parity_shards, devs.data(), (int)devs.size(), flags, out);
        device = 0;
    }
    if (device < 0) return RSGPU_ERR_INVALID_ARG;
    std::unique_ptr<rsgpu_ctx> c(new (std::nothrow) rsgpu_ctx());
    if (!c) return RSGPU_ERR_NOMEM;
    c->k = data_shards;
    c->p = parity_shards;
    c->n = data_shards + parity_shards;
    c->kind = kind;
    c->device = device;
    if (!gf_build_matrix(c->k, c->p, kind, c->m)) return RSGPU_ERR_SINGULAR;
    *out = c.release();
    return RSGPU_OK;
}

int rsgpu_create_multi(int data_shards, int parity_shards, const int *devices, int ndev, unsigned flags,
                       rsgpu_ctx **out) {
    if (!out) return RSGPU_ERR_INVALID_ARG;
    *out = nullptr;
    if (!devices || ndev <= 0) return RSGPU_ERR_INVALID_ARG;
    rsgpu_ctx *parent = nullptr;
    int e = rsgpu_create(data_shards, parity_shards, devices[0] < 0 ? -2 : devices[0], flags, &parent);
    if (e) return e;
    std::unique_ptr<rsgpu_ctx> P(parent);
    // a device may be listed more than once: each entry is an independent
    // single-device context (its own streams, staging slots and pipeline)
    for (int i = 0; i < ndev; ++i) {
        rsgpu_ctx *c = nullptr;
        if ((e = rsgpu_create(data_shards, parity_shards, devices[i] < 0 ? -2 : devices[i], flags, &c))) return e;
        c->parent = P.get();
        P->subs.emplace_back(c);
    }
    *out = P.release();
    return RSGPU_OK;
}

int rsgpu_devices(const rsgpu_ctx *ctx, int *out, int cap) {
    if (!ctx || cap < 0 || (cap > 0 && !out)) return RSGPU_ERR_INVALID_ARG;
    if (!ctx->multi()) {
        if (cap > 0) out[0] = ctx->device;
        return 1;
    }
    for (int i = 0; i < (int)ctx->subs.size() && i < cap; ++i) out[i] = ctx->subs[i]->device;
    return (int)ctx->subs.size();
}

int rsgpu_device_calls(const rsgpu_ctx *ctx, uint64_t *out, int cap) {
    if (!ctx || cap < 0 || (cap > 0 && !out)) return RSGPU_ERR_INVALID_ARG;
    if (!ctx->multi()) {
        if (cap > 0) out[0] = ctx->calls.load(std::memory_order_relaxed);
        return 1;
    }
    for (int i = 0; i < (int)ctx->subs.size() && i < cap; ++i)
        out[i] = ctx->subs[i]->calls.load(std::memory_order_relaxed);
    return (int)ctx->subs.size();
}

void rsgpu_destroy(rsgpu_ctx *ctx) {
    if (!ctx) return;
    (void)rsgpu_worker_stop(ctx);  // the resident kernel reads this context's tables
    for (auto &c : ctx->subs) rsgpu_destroy(c.release());  // each on its own device
    DeviceGuard g;  // frees its device memory on its device, then restores the caller's
    int cur = -1;
    if (ctx->dev_state == 1 && hipGetDevice(&cur) == hipSuccess && cur != ctx->device &&
        hipSetDevice(ctx->device) == hipSuccess)
        g.prev = cur;
    delete ctx;
    relieve_retired();  // what a resident worker held back stays bounded (devmem.cpp)
}

int rsgpu_data_shards(const rsgpu_ctx *ctx) { return ctx ? ctx->k : RSGPU_ERR_INVALID_ARG; }
int rsgpu_parity_shards(const rsgpu_ctx *ctx) { return ctx ? ctx->p : RSGPU_ERR_INVALID_ARG; }

int rsgpu_matrix(const rsgpu_ctx *ctx, uint8_t *out) {
    if (!ctx || !out) return RSGPU_ERR_INVALID_ARG;
    std::memcpy(out, ctx->m.data(), ctx->m.size());
    return RSGPU_OK;
}

int rsgpu_encode(rsgpu_ctx *ctx, uint8_t *const *shards, const size_t *lens, int nshards) {
    RSGPU_FORWARD_RR(rsgpu_encode, shards, lens, nshards);
    if (!ctx || !shards || !lens) return RSGPU_ERR_INVALID_ARG;
    if (nshards != ctx->n) return RSGPU_ERR_TOO_FEW_SHARDS;
    size_t size;
    int e = check_shards(lens, nshards, false, &size);
    if (e) return e;
    DeviceGuard dg_;
    if ((e = ctx->use_device(dg_))) return e;
    uint32_t wbad = 0;
    if ((e = worker_run(ctx, kWopEncode, size, 0, shards, &wbad)) != kWorkerDeclined) return e;
    auto plan = ctx->plan_encode();
    std::vector<const uint8_t *> in(shards, shards + ctx->k);
    std::vector<uint8_t *> out(shards + ctx->k, shards + ctx->n);
    return run_host(ctx, *plan, ctx->n, size, in, out, nullptr);
}

int rsgpu_encode_verify(rsgpu_ctx *ctx, uint8_t *const *shards, const size_t *lens, int nshards, int *ok) {
    RSGPU_FORWARD_RR(rsgpu_encode_verify, shards, lens, nshards, ok);
    if (!ctx || !shards || !lens || !ok) return RSGPU_ERR_INVALID_ARG;
    *ok = 0;
    if (nshards != ctx->n) return RSGPU_ERR_TOO_FEW_SHARDS;
    size_t size;
    int e = check_shards(lens, nshards, false, &size);
    if (e) return e;
    DeviceGuard dg_;
    if ((e = ctx->use_device(dg_))) return e;
    uint32_t wbad = 0;
    if ((e = worker_run(ctx, kWopEncodeVerify, size, 0, shards, &wbad)) != kWorkerDeclined) {
        if (e == RSGPU_OK) *ok = wbad == 0;
        return e;
    }
    auto enc = ctx->plan_encode();
    auto ver = ctx->plan_verify();
    std::vector<const uint8_t *> in(shards, shards + ctx->k);
    std::vector<uint8_t *> out(shards + ctx->k, shards + ctx->n);
    uint32_t bad = 1;
    e = run_host(ctx, *enc, ctx->n, size, in, out, nullptr, ver.get(), &bad);
    if (e) return e;
    *ok = bad == 0;
    return RSGPU_OK;
}

int rsgpu_verify(rsgpu_ctx *ctx, const uint8_t *const *shards, const size_t *lens, int nshards, int *ok) {
    RSGPU_FORWARD_RR(rsgpu_verify, shards, lens, nshards, ok);
    if (!ctx || !shards || !lens || !ok) return RSGPU_ERR_INVALID_ARG;
    *ok = 0;
    if (nshards != ctx->n) return RSGPU_ERR_TOO_FEW_SHARDS;
    size_t size;
    int e = check_shards(lens, nshards, false, &size);
    if (e) return e;
    DeviceGuard dg_;
    if ((e = ctx->use_device(dg_))) return e;
    uint32_t wbad = 0;
    if ((e = worker_run(ctx, kWopVerify, size, 0, const_cast<uint8_t *const *>(shards), &wbad)) != kWorkerDeclined) {
        if (e == RSGPU_OK) *ok = wbad == 0;
        return e;
    }
    auto plan = ctx->plan_verify();
    std::vector<const uint8_t *> in(shards, shards + ctx->n);
    uint32_t bad = 1;
    e = run_host(ctx, *plan, ctx->n, size, in, {}, &bad);
    if (e) return e;
    *ok = bad == 0;
    return RSGPU_OK;
}

static int reconstruct_common(rsgpu_ctx *ctx, uint8_t *const *shards, const size_t *lens,
                              int nshards, bool data_only, bool check, int *ok) {
    if (!ctx || !shards || !lens) return RSGPU_ERR_INVALID_ARG;
    if (nshards != ctx->n) return RSGPU_ERR_TOO_FEW_SHARDS;
    size_t size;
    int e = check_shards(lens, nshards, true, &size);
    if (e) return e;
    std::vector<uint8_t> present(ctx->n);
    int np = 0;
    for (int i = 0; i < ctx->n; ++i) np += (present[i] = lens[i] != 0);
    if (np == ctx->n) {
        if (!check) return RSGPU_OK;
        return rsgpu_verify(ctx, shards, lens, nshards, ok);
    }
    if (np < ctx->k) return RSGPU_ERR_TOO_FEW_SHARDS;
    std::shared_ptr<Plan> plan;
    if ((e = ctx->plan_reconstruct(present.data(), data_only, check, plan))) return e;
    for (int r = 0; r < plan->nw; ++r)
        if (!shards[plan->out_rows[r]]) return RSGPU_ERR_INVALID_ARG;
    DeviceGuard dg_;
    if ((e = ctx->use_device(dg_))) return e;
    if (ctx->worker_raw.load(std::memory_order_relaxed)) {
        // the worker writes every missing row it rebuilds through rows[i]:
        // each needs a buffer (ReconstructData: the missing data rows only)
        bool bufs = true;
        uint32_t mask = 0;
        for (int i = 0; i < ctx->n; ++i) {
            mask |= (uint32_t)present[i] << i;
            if (!present[i] && !shards[i] && (!data_only || i < ctx->k)) bufs = false;
        }
        uint32_t wbad = 0;
        if (bufs && (e = worker_run(ctx, check ? kWopDecode : data_only ? kWopReconstructData : kWopReconstruct, size,
                                    mask, shards, &wbad)) != kWorkerDeclined) {
            if (e == RSGPU_OK && ok) *ok = wbad == 0;
            return e;
        }
    }
    std::vector<const uint8_t *> in;
    for (int row : plan->in_rows) in.push_back(shards[row]);
    std::vector<uint8_t *> out;
    for (int r = 0; r < plan->nw; ++r) out.push_back(shards[plan->out_rows[r]]);
    uint32_t bad = 0;
    e = run_host(ctx, *plan, ctx->n, size, in, out, &bad);
    if (e) return e;
    if (ok) *ok = bad == 0;
    return RSGPU_OK;
}

int rsgpu_reconstruct(rsgpu_ctx *ctx, uint8_t *const *shards, const size_t *lens, int nshards,
                      int data_only) {
    RSGPU_FORWARD_RR(rsgpu_reconstruct, shards, lens, nshards, data_only);
    return reconstruct_common(ctx, shards, lens, nshards, data_only != 0, false, nullptr);
}

int rsgpu_decode(rsgpu_ctx *ctx, uint8_t *const *shards, const size_t *lens, int nshards, int *ok) {
    RSGPU_FORWARD_RR(rsgpu_decode, shards, lens, nshards, ok);
    if (!ok) return RSGPU_ERR_INVALID_ARG;
    *ok = 0;
    return reconstruct_common(ctx, shards, lens, nshards, false, true, ok);
}

int rsgpu_update(rsgpu_ctx *ctx, uint8_t *const *shards, const size_t *lens, int nshards,
                 const uint8_t *const *newdata, const size_t *new_lens, int nnew) {
    RSGPU_FORWARD_RR(rsgpu_update, shards, lens, nshards, newdata, new_lens, nnew);
    if (!ctx || !shards || !lens || !newdata || !new_lens) return RSGPU_ERR_INVALID_ARG;
    const int k = ctx->k, n = ctx->n;
    if (nshards != n) return RSGPU_ERR_TOO_FEW_SHARDS;
    if (nnew != k) return RSGPU_ERR_TOO_FEW_SHARDS;
    size_t size, size2;
    int e = check_shards(lens, nshards, true, &size);
    if (e) return e;
    if ((e = check_shards(new_lens, nnew, true, &size2))) return e;
    for (int i = 0; i < k; ++i)
        if (new_lens[i] != 0 && lens[i] == 0) return RSGPU_ERR_INVALID_INPUT;
    for (int i = k; i < n; ++i)
        if (lens[i] == 0) return RSGPU_ERR_INVALID_INPUT;
    if (size2 != size) return RSGPU_ERR_SHARD_SIZE;
    std::vector<int> changed;
    for (int c = 0; c < k; ++c)
        if (new_lens[c]) changed.push_back(c);
    if (changed.empty()) return RSGPU_OK;
    DeviceGuard dg_;
    if ((e = ctx->use_device(dg_))) return e;
    // staging rows: [0,n) shards, [n, n+k) new data, [n+k, n+k+|C|+p) outputs
    const int nc = (int)changed.size();
    Plan plan;
    for (int c : changed) plan.in_rows.push_back(c);
    for (int c : changed) plan.in_rows.push_back(n + c);
    for (int r = k; r < n; ++r) plan.in_rows.push_back(r);
    plan.K = (int)plan.in_rows.size();
    for (int i = 0; i < nc; ++i) {  // delta_c = old_c ^ new_c
        plan.out_rows.push_back(n + k + i);
        for (int c = 0; c < plan.K; ++c) plan.coef.push_back(c == i || c == nc + i);
    }
    for (int r = 0; r < ctx->p; ++r) {  // parity_r ^= M[k+r][c] (old_c ^ new_c)
        plan.out_rows.push_back(n + k + nc + r);
        for (int i = 0; i < nc; ++i) plan.coef.push_back(ctx->row(k + r)[changed[i]]);
        for (int i = 0; i < nc; ++i) plan.coef.push_back(ctx->row(k + r)[changed[i]]);
        for (int j = 0; j < ctx->p; ++j) plan.coef.push_back(j == r);
    }
    plan.R = plan.nw = nc + ctx->p;
    plan.build_tables();
    std::vector<const uint8_t *> in;
    for (int c : changed) in.push_back(shards[c]);
    for (int c : changed) in.push_back(newdata[c]);
    for (int r = k; r < n; ++r) in.push_back(shards[r]);
    std::vector<uint8_t *> out;
    for (int c : changed) out.push_back(shards[c]);
    for (int r = k; r < n; ++r) out.push_back(shards[r]);
    return run_host(ctx, plan, n + k + nc + ctx->p, size, in, out, nullptr);
}

// ------------------------------------------- contiguous-image host calls
// Thin forms of the pointer-table calls for Split's contiguous layout: the
// table is built here, on the C side, so a cgo caller passes one pointer.

namespace {

int image_table(const rsgpu_ctx *ctx, const uint8_t *base, size_t shard_len, int nshards, uint64_t present,
                std::vector<uint8_t *> &ptrs, std::vector<size_t> &lens) {
    if (!ctx || !base) return RSGPU_ERR_INVALID_ARG;
    if (nshards <= 0 || nshards > 64) return nshards != ctx->n ? RSGPU_ERR_TOO_FEW_SHARDS : RSGPU_ERR_INVALID_ARG;
    ptrs.resize(nshards);
    lens.resize(nshards);
    for (int i = 0; i < nshards; ++i) {
        ptrs[i] = const_cast<uint8_t *>(base) + (size_t)i * shard_len;
        lens[i] = (present >> i) & 1 ? shard_len : 0;
    }
    return RSGPU_OK;
}

}  // namespace

extern "C" {

int rsgpu_encode_image(rsgpu_ctx *ctx, uint8_t *base, size_t shard_len, int nshards) {
    std::vector<uint8_t *> p;
    std::vector<size_t> l;
    int e = image_table(ctx, base, shard_len, nshards, ~0ull, p, l);
    return e ? e : rsgpu_encode(ctx, p.data(), l.data(), nshards);
}

int rsgpu_encode_verify_image(rsgpu_ctx *ctx, uint8_t *base, size_t shard_len, int nshards, int *ok) {
    std::vector<uint8_t *> p;
    std::vector<size_t> l;
    int e = image_table(ctx, base, shard_len, nshards, ~0ull, p, l);
    return e ? e : rsgpu_encode_verify(ctx, p.data(), l.data(), nshards, ok);
}

int rsgpu_verify_image(rsgpu_ctx *ctx, const uint8_t *base, size_t shard_len, int nshards, int *ok) {
    std::vector<uint8_t *> p;
    std::vector<size_t> l;
    int e = image_table(ctx, base, shard_len, nshards, ~0ull, p, l);
    return e ? e : rsgpu_verify(ctx, (const uint8_t *const *)p.data(), l.data(), nshards, ok);
}

int rsgpu_reconstruct_image(rsgpu_ctx *ctx, uint8_t *base, size_t shard_len, int nshards, uint64_t present,
                            int data_only) {
    std::vector<uint8_t *> p;
    std::vector<size_t> l;
    int e = image_table(ctx, base, shard_len, nshards, present, p, l);
    return e ? e : rsgpu_reconstruct(ctx, p.data(), l.data(), nshards, data_only);
}

int rsgpu_decode_image(rsgpu_ctx *ctx, uint8_t *base, size_t shard_len, int nshards, uint64_t present, int *ok) {
    std::vector<uint8_t *> p;
    std::vector<size_t> l;
    int e = image_table(ctx, base, shard_len, nshards, present, p, l);
    return e ? e : rsgpu_decode(ctx, p.data(), l.data(), nshards, ok);
}

}  // extern "C"

// ---------------------------------------------------- device-resident API

int rsgpu_encode_dev(rsgpu_ctx *ctx, void *d_base, size_t shard_len, size_t pitch,
                     size_t obj_stride, int nobj, void *stream) {
    RSGPU_FORWARD_DEV(rsgpu_encode_dev, d_base, d_base, shard_len, pitch, obj_stride, nobj, stream)
    if (!ctx) return RSGPU_ERR_INVALID_ARG;
    int e = check_layout(ctx, d_base, shard_len, pitch, obj_stride, nobj, true);
    if (e) return e;
    DeviceGuard dg_;
    if ((e = ctx->use_device(dg_))) return e;
    auto plan = ctx->plan_encode();
    Layout L{(uint8_t *)d_base, obj_stride, pitch, shard_len, nobj};
    HIP_TRY(launch_plan(*plan, L, nullptr, (hipStream_t)stream));
    return RSGPU_OK;
}

int rsgpu_verify_dev(rsgpu_ctx *ctx, const void *d_base, size_t shard_len, size_t pitch,
                     size_t obj_stride, int nobj, uint32_t *d_bad, void *stream) {
    RSGPU_FORWARD_DEV(rsgpu_verify_dev, d_base, d_base, shard_len, pitch, obj_stride, nobj, d_bad, stream)
    if (!ctx || !d_bad) return RSGPU_ERR_INVALID_ARG;
    int e = check_layout(ctx, d_base, shard_len, pitch, obj_stride, nobj, true);
    if (e) return e;
    DeviceGuard dg_;
    if ((e = ctx->use_device(dg_))) return e;
    auto plan = ctx->plan_verify();
    Layout L{(uint8_t *)d_base, obj_stride, pitch, shard_len, nobj};
    HIP_TRY(hipMemsetAsync(d_bad, 0, (size_t)nobj * 4, (hipStream_t)stream));
    HIP_TRY(launch_plan(*plan, L, d_bad, (hipStream_t)stream));
    return RSGPU_OK;
}

static int recon_dev(rsgpu_ctx *ctx, void *d_base, const uint8_t *present, size_t shard_len,
                     size_t pitch, size_t obj_stride, int nobj, bool data_only, bool check,
                     uint32_t *d_bad, void *stream) {
    if (!ctx || !present) return RSGPU_ERR_INVALID_ARG;
    int e = check_layout(ctx, d_base, shard_len, pitch, obj_stride, nobj, true);
    if (e) return e;
    int np = 0;
    for (int i = 0; i < ctx->n; ++i) np += present[i] != 0;
    if (np < ctx->k) return RSGPU_ERR_TOO_FEW_SHARDS;
    DeviceGuard dg_;
    if ((e = ctx->use_device(dg_))) return e;
    if (np == ctx->n) {
        if (!check) return RSGPU_OK;
        return rsgpu_verify_dev(ctx, d_base, shard_len, pitch, obj_stride, nobj, d_bad, stream);
    }
    std::shared_ptr<Plan> plan;
    if ((e = ctx->plan_reconstruct(present, data_only, check, plan))) return e;
    Layout L{(uint8_t *)d_base, obj_stride, pitch, shard_len, nobj};
    // with check rows the flags are OR-ed by the kernel and need a memset
    // first; without, the kernel clears them itself (no extra launch)
    if (check && plan->nw < plan->R)
        HIP_TRY(hipMemsetAsync(d_bad, 0, (size_t)nobj * 4, (hipStream_t)stream));
    HIP_TRY(launch_plan(*plan, L, check ? d_bad : nullptr, (hipStream_t)stream));
    return RSGPU_OK;
}

// Bitmask of the nonzero bytes of flags[0, n), n <= 64: eight flags per
// word (OR-fold each byte onto its low bit, then gather the low bits).
static uint64_t present_mask(const uint8_t *flags, int n) {
    uint64_t mask = 0;
    int i = 0;
    for (; i + 8 <= n; i += 8) {
        uint64_t w;
        std::memcpy(&w, flags + i, 8);
        w |= w >> 4;
        w |= w >> 2;
        w |= w >> 1;
        w &= 0x0101010101010101ull;
        mask |= ((w * 0x0102040810204080ull) >> 56) << i;
    }
    for (; i < n; ++i) mask |= (uint64_t)(flags[i] != 0) << i;
    return mask;
}

// mask -> plan index (-1: not yet planned): a direct table for n <= 16
// shards, else open addressing with load <= 1/2
struct PatternTable {
    explicit PatternTable(int n) : direct(n <= 16 ? (size_t)1 << n : 0, -1) {
        if (direct.empty()) keys.resize(256), vals.resize(256), used.resize(256);
    }
    int &operator[](uint64_t k) { return direct.empty() ? find_or_insert(k) : direct[k]; }

  private:
    std::vector<int> direct;
    std::vector<uint64_t> keys;
    std::vector<int> vals;
    std::vector<uint8_t> used;
    size_t count = 0;
    static size_t hash(uint64_t k) { return (size_t)((k * 0x9E3779B97F4A7C15ull) >> 32); }
    int &find_or_insert(uint64_t k) {
        if (2 * (count + 1) > keys.size()) grow();
        size_t m = keys.size() - 1, h = hash(k) & m;
        while (used[h] && keys[h] != k) h = (h + 1) & m;
        if (!used[h]) {
            used[h] = 1;
            keys[h] = k;
            vals[h] = -1;
            ++count;
        }
        return vals[h];
    }
    void grow() {
        std::vector<uint64_t> k2(keys.size() * 2);
        std::vector<int> v2(keys.size() * 2);
        std::vector<uint8_t> u2(keys.size() * 2);
        std::swap(k2, keys);
        std::swap(v2, vals);
        std::swap(u2, used);
        count = 0;
        for (size_t i = 0; i < k2.size(); ++i)
            if (u2[i]) find_or_insert(k2[i]) = v2[i];
    }
};

// Mixed erasure patterns: present is nobj x (data+parity).  Objects are
// grouped by pattern (one cached plan each) and coded by one launch per
// (K, R) class (launch_plans_multi).
// Host present flags -> masks, uploaded from a pinned ring slot on a side
// stream (no host wait), then the device-resolved passes (n <= 16).  Argument
// errors (too few shards, a singular pattern) are returned before any launch.
static int recon_dev_multi_atlas(rsgpu_ctx *ctx, void *d_base, const uint8_t *present, size_t shard_len,
                                 size_t pitch, size_t obj_stride, int nobj, AtlasMode mode,
                                 uint32_t *d_bad, void *stream) {
    const int n = ctx->n;
    const Atlas *ah;
    int e = ctx->atlas_host(mode, ah);
    if (e) return e;
    MultiWorkspace &ws = ctx->multi_ws;
    std::lock_guard<std::mutex> g(ws.mu);
    // argument errors first (upstream precedence), without a device
    std::vector<uint32_t> &hm = ws.masks;
    hm.resize((size_t)nobj);
    for (int o = 0; o < nobj; ++o) {
        const uint32_t mask = (uint32_t)present_mask(present + (size_t)o * n, n);
        const int32_t slot = ah->h_pat[mask];
        if (slot == kPatTooFew) return RSGPU_ERR_TOO_FEW_SHARDS;
        if (slot == kPatSingular) return RSGPU_ERR_SINGULAR;
        hm[o] = mask;
    }
    DeviceGuard dg_;
    if ((e = ctx->use_device(dg_))) return e;
    AtlasView A;
    if ((e = ctx->atlas_view(mode, A))) return e;
    const unsigned si = ws.next++ % MultiWorkspace::kRing;
    MultiWorkspace::Slot &w = ws.slot[si];
    if (!ws.upload) HIP_TRY(hipStreamCreateWithFlags(&ws.upload, hipStreamNonBlocking));
    if (!ws.uploaded[si]) HIP_TRY(hipEventCreateWithFlags(&ws.uploaded[si], hipEventDisableTiming));
    if (w.done) HIP_TRY(hipEventSynchronize(w.done));  // the kernels that read it kRing calls ago
    else HIP_TRY(hipEventCreateWithFlags(&w.done, hipEventDisableTiming));
    const size_t bytes = (size_t)nobj * 4;
    if (w.cap < bytes) {
        retire(w.d, false, w.cap);  // (held while a worker kernel is resident: devmem.cpp)
        retire(w.h, true, w.cap);
        w.d = nullptr;
        w.h = nullptr;
        w.cap = 0;
        const size_t cap = std::max<size_t>(bytes * 2, 1 << 16);
        HIP_TRY(hipMalloc(&w.d, cap));
        HIP_TRY(hipHostMalloc(&w.h, cap, hipHostMallocDefault));
        w.cap = cap;
    }
    std::memcpy(w.h, hm.data(), bytes);
    HIP_TRY(hipMemcpyAsync(w.d, w.h, bytes, hipMemcpyHostToDevice, ws.upload));
    HIP_TRY(hipEventRecord(ws.uploaded[si], ws.upload));
    HIP_TRY(hipStreamWaitEvent((hipStream_t)stream, ws.uploaded[si], 0));
    Layout L{(uint8_t *)d_base, obj_stride, pitch, shard_len, nobj};
    e = run_masked(ctx, A, mode, L, (const uint32_t *)w.d, mode == kAtlasDecode ? d_bad : nullptr,
                   (hipStream_t)stream);
    // the slot is reused only after these kernels finished with the masks
    const hipError_t he = hipEventRecord(w.done, (hipStream_t)stream);
    if (e) return e;
    if (he != hipSuccess) return hip_fail(he, "multi ring event");
    return RSGPU_OK;
}

static int recon_dev_multi(rsgpu_ctx *ctx, void *d_base, const uint8_t *present, size_t shard_len,
                           size_t pitch, size_t obj_stride, int nobj, bool data_only, bool check,
                           uint32_t *d_bad, void *stream) {
    if (!ctx || (nobj > 0 && !present)) return RSGPU_ERR_INVALID_ARG;
    int e = check_layout(ctx, d_base, shard_len, pitch, obj_stride, nobj);
    if (e) return e;
    const int n = ctx->n;
    if (nobj == 0) return RSGPU_OK;
    // the device-resolved kernels for codes whose atlas is modest (RS(10+2):
    // 30 KB; RS(12+4): ~1 MB); wider atlases (e.g. RS(4+12), RS(2+14)) keep the
    // host-planned path below rather than building tens of thousands of
    // patterns on the first call
    if (n <= kAtlasMaxN && !((uintptr_t)d_base & 15) && !(pitch & 15) && !(obj_stride & 15) &&
        atlas_estimate(ctx->k, ctx->p, check) <= kAtlasHostFlagBytes) {
        e = recon_dev_multi_atlas(ctx, d_base, present, shard_len, pitch, obj_stride, nobj,
                                  check ? kAtlasDecode : data_only ? kAtlasData : kAtlasReconstruct, d_bad, stream);
        if (e != RSGPU_ERR_NOT_IMPLEMENTED) return e;
    }
    // pattern key: the present bitmask (n <= 64: one word, looked up in a
    // PatternTable — a Get batch of 4 KiB objects holds 10^5+ objects, and
    // this loop is host time in front of the launch; else a byte string)
    PatternTable idx64(n);
    std::map<std::string, int> idx_str;
    std::vector<std::shared_ptr<Plan>> owned;
    std::vector<Plan *> plans;
    std::vector<int> plan_of(nobj, -1);
    bool any_checks = false;
    for (int o = 0; o < nobj; ++o) {
        const uint8_t *pr = present + (size_t)o * n;
        uint64_t mask = 0;
        int np;
        if (n <= 64) {
            mask = present_mask(pr, n);
            np = __builtin_popcountll(mask);
        } else {
            np = 0;
            for (int i = 0; i < n; ++i) np += pr[i] != 0;
        }
        if (np < ctx->k) return RSGPU_ERR_TOO_FEW_SHARDS;
        if (np == n && !check) continue;  // nothing to reconstruct
        int *slot_idx;
        if (n <= 64) {
            slot_idx = &idx64[mask];
        } else {
            std::string key(n, '0');
            for (int i = 0; i < n; ++i) key[i] = pr[i] ? '1' : '0';
            auto ins = idx_str.emplace(key, -1);
            slot_idx = &ins.first->second;
        }
        if (*slot_idx < 0) {
            std::shared_ptr<Plan> p;
            if (np == n) p = ctx->plan_verify();
            else if ((e = ctx->plan_reconstruct(pr, data_only, check, p))) return e;
            any_checks |= p->nw < p->R;
            *slot_idx = (int)plans.size();
            owned.push_back(p);
            plans.push_back(p.get());
        }
        plan_of[o] = *slot_idx;
    }
    DeviceGuard dg_;
    if ((e = ctx->use_device(dg_))) return e;
    if (check && any_checks)
        HIP_TRY(hipMemsetAsync(d_bad, 0, (size_t)nobj * 4, (hipStream_t)stream));
    Layout L{(uint8_t *)d_base, obj_stride, pitch, shard_len, nobj};
    HIP_TRY(launch_plans_multi(plans, plan_of, L, check ? d_bad : nullptr, (hipStream_t)stream,
                               ctx->multi_ws));
    return RSGPU_OK;
}

int rsgpu_reconstruct_dev_multi(rsgpu_ctx *ctx, void *d_base, const uint8_t *present,
                                size_t shard_len, size_t pitch, size_t obj_stride, int nobj,
                                int data_only, void *stream) {
    RSGPU_FORWARD_DEV(rsgpu_reconstruct_dev_multi, d_base, d_base, present, shard_len, pitch, obj_stride, nobj,
                      data_only, stream)
    return recon_dev_multi(ctx, d_base, present, shard_len, pitch, obj_stride, nobj, data_only != 0,
                           false, nullptr, stream);
}

int rsgpu_decode_dev_multi(rsgpu_ctx *ctx, void *d_base, const uint8_t *present, size_t shard_len,
                           size_t pitch, size_t obj_stride, int nobj, uint32_t *d_bad, void *stream) {
    RSGPU_FORWARD_DEV(rsgpu_decode_dev_multi, d_base, d_base, present, shard_len, pitch, obj_stride, nobj, d_bad,
                      stream)
    if (!d_bad) return RSGPU_ERR_INVALID_ARG;
    return recon_dev_multi(ctx, d_base, present, shard_len, pitch, obj_stride, nobj, false, true, d_bad,
                           stream);
}

int rsgpu_decode_dev_masks(rsgpu_ctx *ctx, void *d_base, const uint32_t *d_masks, size_t shard_len,
                           size_t pitch, size_t obj_stride, int nobj, uint32_t *d_status, void *stream) {
    RSGPU_FORWARD_DEV(rsgpu_decode_dev_masks, d_base, d_base, d_masks, shard_len, pitch, obj_stride, nobj, d_status,
                      stream)
    return dev_masks(ctx, d_base, d_masks, shard_len, pitch, obj_stride, nobj, kAtlasDecode, d_status, stream);
}

int rsgpu_reconstruct_dev_masks(rsgpu_ctx *ctx, void *d_base, const uint32_t *d_masks, size_t shard_len,
                                size_t pitch, size_t obj_stride, int nobj, int data_only, uint32_t *d_status,
                                void *stream) {
    RSGPU_FORWARD_DEV(rsgpu_reconstruct_dev_masks, d_base, d_base, d_masks, shard_len, pitch, obj_stride, nobj,
                      data_only, d_status, stream)
    return dev_masks(ctx, d_base, d_masks, shard_len, pitch, obj_stride, nobj,
                     data_only ? kAtlasData : kAtlasReconstruct, d_status, stream);
}

// ---------------------------------------------- variable-size device batches

static_assert(sizeof(rsgpu_dev_obj) == sizeof(DevObj) && offsetof(rsgpu_dev_obj, shard_len) == offsetof(DevObj, shard_len) &&
                  offsetof(rsgpu_dev_obj, pitch) == offsetof(DevObj, pitch),
              "rsgpu_dev_obj and DevObj share one layout");

// Argument checks of a variable-size table; multi-device contexts: the
// entry that owns the objects' memory (all on one device)
static int objs_prepare(rsgpu_ctx *&ctx, const rsgpu_dev_obj *objs, int nobj) {
    if (!ctx || nobj < 0 || (nobj > 0 && !objs)) return RSGPU_ERR_INVALID_ARG;
    for (int o = 0; o < nobj; ++o) {
        const rsgpu_dev_obj &d = objs[o];
        if (!d.base) return RSGPU_ERR_INVALID_ARG;
        if (d.shard_len == 0) return RSGPU_ERR_SHARD_NO_DATA;
        if (d.pitch < (d.shard_len + 15) / 16 * 16) return RSGPU_ERR_INVALID_ARG;
        if ((size_t)ctx->n * d.pitch >= ((size_t)1 << 32)) return RSGPU_ERR_INVALID_ARG;
    }
    if (ctx->multi() && nobj > 0) {
        rsgpu_ctx *sub = ctx->sub_for(objs[0].base);
        if (!sub) return RSGPU_ERR_INVALID_ARG;
        for (int o = 1; o < nobj; ++o) {
            hipPointerAttribute_t at;
            if (hipPointerGetAttributes(&at, objs[o].base) != hipSuccess || at.device != sub->device)
                return RSGPU_ERR_INVALID_ARG;
        }
        ctx = sub;
    }
    return RSGPU_OK;
}

int rsgpu_encode_dev_objs(rsgpu_ctx *ctx, const rsgpu_dev_obj *objs, int nobj, void *stream) {
    int e = objs_prepare(ctx, objs, nobj);
    if (e) return e;
    DeviceGuard dg_;
    if ((e = ctx->use_device(dg_))) return e;
    if (nobj == 0) return RSGPU_OK;
    auto plan = ctx->plan_encode();
    HIP_TRY(launch_plan_objs(*plan, (const DevObj *)objs, nobj, nullptr, (hipStream_t)stream, ctx->multi_ws));
    return RSGPU_OK;
}

int rsgpu_verify_dev_objs(rsgpu_ctx *ctx, const rsgpu_dev_obj *objs, int nobj, uint32_t *d_bad, void *stream) {
    if (!d_bad) return RSGPU_ERR_INVALID_ARG;
    int e = objs_prepare(ctx, objs, nobj);
    if (e) return e;
    DeviceGuard dg_;
    if ((e = ctx->use_device(dg_))) return e;
    if (nobj == 0) return RSGPU_OK;
    auto plan = ctx->plan_verify();
    HIP_TRY(hipMemsetAsync(d_bad, 0, (size_t)nobj * 4, (hipStream_t)stream));
    HIP_TRY(launch_plan_objs(*plan, (const DevObj *)objs, nobj, d_bad, (hipStream_t)stream, ctx->multi_ws));
    return RSGPU_OK;
}

static int recon_dev_objs(rsgpu_ctx *ctx, const rsgpu_dev_obj *objs, int nobj, const uint8_t *present,
                          bool data_only, bool check, uint32_t *d_bad, void *stream) {
    if (!present || (check && !d_bad)) return RSGPU_ERR_INVALID_ARG;
    int e = objs_prepare(ctx, objs, nobj);
    if (e) return e;
    int np = 0;
    for (int i = 0; i < ctx->n; ++i) np += present[i] != 0;
    if (np < ctx->k) return RSGPU_ERR_TOO_FEW_SHARDS;
    if (np == ctx->n) {
        if (!check) return RSGPU_OK;
        return rsgpu_verify_dev_objs(ctx, objs, nobj, d_bad, stream);
    }
    std::shared_ptr<Plan> plan;
    if ((e = ctx->plan_reconstruct(present, data_only, check, plan))) return e;
    DeviceGuard dg_;
    if ((e = ctx->use_device(dg_))) return e;
    if (nobj == 0) return RSGPU_OK;
    if (check && plan->nw < plan->R)  // check rows OR into the flags; else the pass clears them
        HIP_TRY(hipMemsetAsync(d_bad, 0, (size_t)nobj * 4, (hipStream_t)stream));
    HIP_TRY(launch_plan_objs(*plan, (const DevObj *)objs, nobj, check ? d_bad : nullptr, (hipStream_t)stream,
                             ctx->multi_ws));
    return RSGPU_OK;
}

int rsgpu_reconstruct_dev_objs(rsgpu_ctx *ctx, const rsgpu_dev_obj *objs, int nobj, const uint8_t *present,
                               int data_only, void *stream) {
    return recon_dev_objs(ctx, objs, nobj, present, data_only != 0, false, nullptr, stream);
}

int rsgpu_decode_dev_objs(rsgpu_ctx *ctx, const rsgpu_dev_obj *objs, int nobj, const uint8_t *present,
                          uint32_t *d_bad, void *stream) {
    return recon_dev_objs(ctx, objs, nobj, present, false, true, d_bad, stream);
}

int rsgpu_reconstruct_dev(rsgpu_ctx *ctx, void *d_base, const uint8_t *present, size_t shard_len,
                          size_t pitch, size_t obj_stride, int nobj, int data_only, void *stream) {
    RSGPU_FORWARD_DEV(rsgpu_reconstruct_dev, d_base, d_base, present, shard_len, pitch, obj_stride, nobj, data_only,
                      stream)
    return recon_dev(ctx, d_base, present, shard_len, pitch, obj_stride, nobj, data_only != 0, false,
                     nullptr, stream);
}

int rsgpu_decode_dev(rsgpu_ctx *ctx, void *d_base, const uint8_t *present, size_t shard_len,
                     size_t pitch, size_t obj_stride, int nobj, uint32_t *d_bad, void *stream) {
    RSGPU_FORWARD_DEV(rsgpu_decode_dev, d_base, d_base, present, shard_len, pitch, obj_stride, nobj, d_bad, stream)
    if (!d_bad) return RSGPU_ERR_INVALID_ARG;
    return recon_dev(ctx, d_base, present, shard_len, pitch, obj_stride, nobj, false, true, d_bad,
                     stream);
}

}  // extern "C"
