// gf_masked.h — device side of the device-resolved mixed-pattern passes
// (rsgpu_{decode,reconstruct}_dev_masks, include/rsgpu.h).
//
// A Get batch gives every object its own erasure pattern: the proxy answers
// each Get with the first d shards to arrive and "-1" for the rest
// (/root/reference/proxy/lambdastore/connection.go:274-306), and
// Client.decode reconstructs whatever is missing (client/ecRedis.go:404-427).
// Here the patterns arrive as present bitmasks in HBM (bit i: shard i
// present), and the pattern -> pass resolution happens on the device: the
// context keeps an ATLAS of every erasure pattern of the code (a direct
// table over all 2^n masks, built and uploaded once), so a call makes no host
// planning pass, no upload and no host synchronisation.
//
//   * gf_apply_masked (rows of > 128 vectors): one workgroup = 256 lanes x
//     16 B of one object chunk, as gf_apply_kernel.  The object's mask, its
//     atlas slot and the slot's record (input rows: the first kact present
//     rows in index order, upstream's survivor rule followed by the fused
//     decode's extra shards; written rows; coefficient tables) come through
//     scalar loads.
//   * gf_apply_lanes (rows of <= 128 vectors, small objects): one workgroup
//     codes opw = 256 / nvec whole objects in address order, lane -> (object,
//     vector), exactly as the uniform small-object launch, whatever their
//     patterns.  Each lane resolves its own object's pattern (input rows =
//     the set bits of its mask) and indexes a 256-entry coefficient table
//     staged in LDS by the coefficient bytes of its pattern (v_perm takes its
//     table words from VGPRs anyway).
//
// Inputs beyond an object's kact read through a zero-record buffer resource
// (or past every range): the load returns zero and touches no memory.
#pragma once
#include <cstddef>

#include "gf_device.h"

namespace rsgpu {

constexpr int kAtlasMaxN = 16;   // masks index a direct table of 2^n entries
constexpr int kCtabStride = 8;   // words per coefficient in the 256-entry table (kTabWords used)

// One sub-pass (<= 4 rows) of one erasure pattern.
struct alignas(16) PatRec {
    uint8_t kact;  // inputs: the first kact present rows in index order
    uint8_t nr;    // rows of the pattern in this sub-pass (0: none)
    uint8_t nw;    // rows [0, nw) written, [nw, nr) compared to zero
    uint8_t ki;    // trailing identity inputs: input kact-ki+j feeds row nr-ki+j
    uint8_t nchk;  // sub-passes of the pattern that hold check rows
    uint8_t pad0[3];
    uint8_t out_row[4];  // written rows (shard indices)
    uint8_t pad1[4];
    uint8_t coef[4][16];  // [r][c], zero for r >= nr or c >= kact
    uint8_t in_row[16];   // input rows: the first kact present rows, ascending (gf_apply_masked)
};
static_assert(sizeof(PatRec) == 96 && offsetof(PatRec, out_row) == 8 && offsetof(PatRec, coef) == 16 &&
                  offsetof(PatRec, in_row) == 80,
              "PatRec layout (host atlas builder, dword reads in both kernels)");

// pattern-table entries besides a record slot
constexpr int32_t kPatTooFew = -1;   // fewer than data shards present: ErrTooFewShards (status 2)
constexpr int32_t kPatNothing = -2;  // nothing to write or check (status 0)
constexpr int32_t kPatSingular = -3; // survivors' matrix not invertible: errSingular (status 3)

// status values (d_status, per object)
constexpr uint32_t kStatusOk = 0, kStatusMismatch = 1, kStatusTooFew = 2, kStatusSingular = 3;

// status of an object whose pattern needs no pass
__device__ __forceinline__ uint32_t pat_status(int32_t slot) {
    return slot == kPatTooFew ? kStatusTooFew : slot == kPatSingular ? kStatusSingular : kStatusOk;
}

struct MaskedArgs {
    const uint8_t *base;
    uint64_t obj_stride;
    const uint32_t *masks;  // [nobj] present bitmasks
    const int32_t *pat;     // [1 << n]: slot, kPatTooFew or kPatNothing
    const PatRec *recs;     // [slot][nsub]
    const uint32_t *tabs;   // [slot][nsub][KMAX][R][kTabWords] (gf_apply_masked)
    const uint32_t *ctab;   // [256][kCtabStride]              (gf_apply_lanes)
    uint32_t *status;       // [nobj] or nullptr: kStatus*
    uint32_t *acc, *cnt;    // [nobj] scratch for multi-reporter status; zero between calls
    uint32_t nmask;         // (1 << n) - 1
    uint32_t kfix;          // inputs per pattern when fixed (reconstruct: k); 0: popcount(mask)
    uint32_t nsub, sub;     // sub-pass of this launch
    uint32_t nvec, tail, pitch, span;
    uint32_t opw, nobj, gspan;  // gf_apply_lanes: objects per workgroup, batch size, group span
    Order ord;              // item = object (masked) or group of opw objects (lanes)
};

// Status of an object whose pattern has check rows in several workgroups
// (every chunk of every sub-pass holding checks): each reports its OR, the
// last one publishes the object's flag and resets the scratch for the next
// call.  Called by one lane of the reporting workgroup.
__device__ __forceinline__ void report_status(const MaskedArgs &a, uint32_t obj, bool any,
                                              uint32_t reporters) {
    if (any) atomicOr(&a.acc[obj], 1u);
    __threadfence();
    const uint32_t done = atomicAdd(&a.cnt[obj], 1u) + 1u;
    if (done == reporters) {
        __threadfence();
        const uint32_t f = atomicExch(&a.acc[obj], 0u);
        atomicExch(&a.cnt[obj], 0u);
        if (a.status) a.status[obj] = f ? kStatusMismatch : kStatusOk;
    }
}

// acc ^= c (x) w with c's table words in VGPRs
__device__ __forceinline__ uint32_t gf_mac_w(uint32_t acc, const u32x4 &t, uint32_t t4, const GfIdx &g) {
    acc = xor3(acc, lut8(t[0], t[1], g.i0), lut8(t[2], t[3], g.i1));
    return acc ^ lut8(t4, t4, g.i2);
}

template <int KMAX, int R, int LAUX, int SAUX>
__global__ __launch_bounds__(256) void gf_apply_masked(const MaskedArgs a) {
    uint32_t obj, chunk;
    if (!wg_item(a.ord, obj, chunk)) return;
    const uint32_t t = threadIdx.x;
    // constant address space: mask, slot and the slot's record are uniform
    // and invariant, fetched with s_load
    const uint32_t mask = ((constant_ptr<uint32_t>)a.masks)[obj] & a.nmask;
    const int32_t slot = ((constant_ptr<int32_t>)a.pat)[mask];
    if (slot < 0) {
        if (a.sub == 0 && chunk == 0 && t == 0 && a.status) a.status[obj] = pat_status(slot);
        return;
    }
    const uint32_t ri = (uint32_t)slot * a.nsub + a.sub;
    // the record as dwords (scalar loads are dword-granular; byte fields
    // would go through vector loads): [0] kact|nr|nw|ki, [1] nchk,
    // [2] out_row[0..3], [20..23] in_row[0..15]
    const constant_ptr<uint32_t> rw = (constant_ptr<uint32_t>)((constant_ptr<PatRec>)a.recs + ri);
    const uint32_t h0 = rw[0], h1 = rw[1], orow = rw[2];
    const uint32_t irow[4] = {rw[20], rw[21], rw[22], rw[23]};
    const uint32_t kact = h0 & 0xffu, nr = (h0 >> 8) & 0xffu, nw = (h0 >> 16) & 0xffu, ki = h0 >> 24;
    const uint32_t nchk = h1 & 0xffu;
    if (nchk == 0 && a.sub == 0 && chunk == 0 && t == 0 && a.status) a.status[obj] = kStatusOk;
    if (nr == 0) return;
    const constant_ptr<uint32_t> tb = (constant_ptr<uint32_t>)a.tabs + (size_t)ri * (KMAX * R * kTabWords);

    const uint32_t v = chunk * 256u + t;
    const bool lane_ok = v < a.nvec;
    // lanes past the row read nothing (offset past every range) and store nothing
    const uint32_t voff = lane_ok ? v * 16u : 0xfffffff0u;
    const uint8_t *ob = a.base + (uint64_t)obj * a.obj_stride;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)ob, (short)0, (int)a.span, 0x00020000);
    const __amdgpu_buffer_rsrc_t rsn = __builtin_amdgcn_make_buffer_rsrc((void *)ob, (short)0, 0, 0x00020000);

    // input rows (the record's, scalar): every load is issued, unused inputs
    // through the zero-record resource, so the wait counts stay static
    u32x4 x[KMAX];
#pragma unroll
    for (int c = 0; c < KMAX; ++c)
        x[c] = __builtin_amdgcn_raw_buffer_load_b128((uint32_t)c < kact ? rs : rsn, voff,
                                                     ((irow[c >> 2] >> (8 * (c & 3))) & 0xffu) * a.pitch, LAUX);
    // keep every load here, in input order: otherwise each one is sunk into
    // the `c < kact` block that uses it, and input 0 is fetched last
    asm volatile("" ::: "memory");

    uint32_t acc[R][4];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int d = 0; d < 4; ++d) acc[r][d] = 0;
#pragma unroll
    for (int c = 0; c < KMAX; ++c) {
        if ((uint32_t)c < kact) {
            if ((uint32_t)c + ki < kact) {
                // every row: rows past nr have zero tables (no per-row branches,
                // which would re-fetch the tables inside the dword loop)
#pragma unroll
                for (int d = 0; d < 4; ++d) {
                    const GfIdx g = gf_idx(x[c][d]);
#pragma unroll
                    for (int r = 0; r < R; ++r) acc[r][d] = gf_mac(acc[r][d], tb + (c * R + r) * kTabWords, g);
                }
            } else {
                // identity input (Verify's parity columns, the decode's extras):
                // feeds row c - kact + nr only, coefficient 1
#pragma unroll
                for (int r = 0; r < R; ++r)
                    if ((uint32_t)r + kact == (uint32_t)c + nr)
#pragma unroll
                        for (int d = 0; d < 4; ++d) acc[r][d] ^= x[c][d];
            }
        }
        // input-at-a-time order (see gf_apply_body)
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int d = 0; d < 4; ++d) asm volatile("" : "+v"(acc[r][d]));
        __builtin_amdgcn_sched_barrier(0);
    }

    bool mismatch = false;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        if ((uint32_t)r >= nr) continue;
        if ((uint32_t)r < nw) {
            if (lane_ok) {
                u32x4 o = {acc[r][0], acc[r][1], acc[r][2], acc[r][3]};
                __builtin_amdgcn_raw_buffer_store_b128(o, rs, voff, ((orow >> (8 * r)) & 0xffu) * a.pitch, SAUX);
            }
        } else if (lane_ok) {
            const uint32_t valid = (v == a.nvec - 1) ? a.tail : 16u;
#pragma unroll
            for (int d = 0; d < 4; ++d) mismatch |= (acc[r][d] & tail_mask(d, valid)) != 0;
        }
    }
    if (nw < nr) {  // this sub-pass checks: one report per workgroup
        const int any = __syncthreads_or(mismatch);
        if (t == 0) report_status(a, obj, any != 0, a.ord.nchunk * nchk);
    }
}

template <int KMAX, int R, int LAUX, int SAUX>
__global__ __launch_bounds__(256) void gf_apply_lanes(const MaskedArgs a) {
    __shared__ u32x4 lt[256][2];   // coefficient c: lt[c][0] = table words 0-3, lt[c][1].x = word 4
    __shared__ uint32_t lflag[256];  // mismatch per object of the group
    uint32_t grp, chunk;
    if (!wg_item(a.ord, grp, chunk)) return;
    const uint32_t t = threadIdx.x;
    // stage the 256-entry coefficient table (its loads overlap the lookups
    // and data loads below; written to LDS before the barrier)
    const u32x4 *ct = (const u32x4 *)(a.ctab + t * kCtabStride);
    const u32x4 ct0 = ct[0], ct1 = ct[1];

    const uint32_t j = t / a.nvec, v = t - j * a.nvec, o = grp * a.opw + j;
    const bool live = j < a.opw && o < a.nobj;
    const uint32_t mask = live ? a.masks[o] & a.nmask : 0u;
    const int32_t slot = live ? a.pat[mask] : kPatNothing;
    const bool act = slot >= 0;
    const uint32_t kact = act ? (a.kfix ? a.kfix : (uint32_t)__builtin_popcount(mask)) : 0u;

    // data loads: this lane's object, its first kact present rows
    const uint8_t *gb = a.base + (uint64_t)grp * a.opw * a.obj_stride;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)gb, (short)0, (int)a.gspan, 0x00020000);
    const uint32_t lane_off = j * (uint32_t)a.obj_stride + v * 16u;
    u32x4 x[KMAX];
    uint32_t m = mask;
#pragma unroll
    for (int c = 0; c < KMAX; ++c) {
        const uint32_t row = m ? (uint32_t)__builtin_ctz(m) : 0u;
        m &= m - 1u;
        x[c] = __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)c < kact ? lane_off + row * a.pitch : 0xfffffff0u,
                                                     0u, LAUX);
    }
    asm volatile("" ::: "memory");  // loads stay here, in input order (see gf_apply_masked)
    // the lane's record: header (kact, nr, nw, ki | nchk | out_row) and coefficient rows
    const u32x4 *rp = (const u32x4 *)(a.recs + (size_t)(act ? (uint32_t)slot : 0u) * a.nsub + a.sub);
    const u32x4 zero = {0u, 0u, 0u, 0u};
    const u32x4 hdr = act ? rp[0] : zero;
    u32x4 crow[R];
#pragma unroll
    for (int r = 0; r < R; ++r) crow[r] = act ? rp[1 + r] : zero;
    const uint32_t nr = (hdr[0] >> 8) & 0xffu, nw = (hdr[0] >> 16) & 0xffu, nchk = hdr[1] & 0xffu;

    lt[t][0] = ct0;
    lt[t][1] = ct1;
    lflag[t] = 0u;
    __syncthreads();

    uint32_t acc[R][4];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int d = 0; d < 4; ++d) acc[r][d] = 0;
#pragma unroll
    for (int c = 0; c < KMAX; ++c) {
        if (__builtin_amdgcn_ballot_w64((uint32_t)c < kact) != 0) {  // some lane of the wave uses input c
            GfIdx g[4];
#pragma unroll
            for (int d = 0; d < 4; ++d) g[d] = gf_idx(x[c][d]);
#pragma unroll
            for (int r = 0; r < R; ++r) {
                // coefficient (r, c) of this lane's pattern (zero where unused)
                const uint32_t cf = (crow[r][c >> 2] >> (8 * (c & 3))) & 0xffu;
                const u32x4 tw = lt[cf][0];
                const uint32_t t4 = lt[cf][1][0];
#pragma unroll
                for (int d = 0; d < 4; ++d) acc[r][d] = gf_mac_w(acc[r][d], tw, t4, g[d]);
            }
        }
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int d = 0; d < 4; ++d) asm volatile("" : "+v"(acc[r][d]));
        __builtin_amdgcn_sched_barrier(0);
    }

    bool mismatch = false;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        if (!act || (uint32_t)r >= nr) continue;
        if ((uint32_t)r < nw) {
            const uint32_t row = (hdr[2] >> (8 * r)) & 0xffu;
            u32x4 ov = {acc[r][0], acc[r][1], acc[r][2], acc[r][3]};
            __builtin_amdgcn_raw_buffer_store_b128(ov, rs, lane_off + row * a.pitch, 0u, SAUX);
        } else {
            const uint32_t valid = (v == a.nvec - 1) ? a.tail : 16u;
#pragma unroll
            for (int d = 0; d < 4; ++d) mismatch |= (acc[r][d] & tail_mask(d, valid)) != 0;
        }
    }
    if (mismatch) lflag[j] = 1u;
    __syncthreads();
    if (!live || v != 0) return;
    // one lane per object publishes its status
    if (!act) {
        if (a.sub == 0 && a.status) a.status[o] = pat_status(slot);
    } else if (nchk == 0) {
        if (a.sub == 0 && a.status) a.status[o] = kStatusOk;
    } else if (nw < nr) {
        if (nchk == 1) {
            if (a.status) a.status[o] = lflag[j] ? kStatusMismatch : kStatusOk;
        } else {
            report_status(a, o, lflag[j] != 0, nchk);
        }
    }
}

}  // namespace rsgpu
