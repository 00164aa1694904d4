// gf_kernels.hip — the hot path: GF(2^8) coding-matrix x object-shard kernels
// for CDNA4 (gfx950).  Replaces the upstream galMulSlice/galMulSliceXor SIMD
// loops and codeSomeShards(P) byte-range goroutine split that sit under
// reedsolomon.Encoder.Encode/Verify/Reconstruct (called from
// /root/reference/client/ecRedis.go:390,395,406,415,420).
//
// Design:
//   * one workgroup = 256 lanes x 16 B of one object, 1D grid over
//     (object, chunk) in XCD-contiguous order (Order, gf_device.h): each XCD
//     sweeps its own contiguous eighth of the launch;
//   * every input row is read once with buffer_load_dwordx4 (1 KiB per wave
//     instruction, the object base in a uniform SRD, the row offset in
//     soffset => no per-row VALU address math);
//   * all R outputs accumulate in VGPRs; GF multiply-by-constant is three
//     v_perm_b32 byte lookups on the 3/3/2-bit groups of the input (tables in
//     SGPRs, from the kernarg segment) merged with v_bitop3 (3-input XOR);
//   * rows [0, nw) are stored with buffer_store_dwordx4; rows [nw, R) are
//     compare-to-zero rows that raise a per-object flag (fused Verify);
//   * non-temporal loads and stores, and on passes that store rows an
//     occupancy cap through an LDS reservation (store_lds below);
//   * short rows (<= 128 vectors): one workgroup codes 256 / nvec whole
//     objects, lane -> (object, vector) (launch_fixed; the mixed-pattern
//     kernel groups same-pattern objects the same way, stage_class).
// No MFMA and no LDS data: the op is HBM-bound byte arithmetic.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <mutex>

#include "gf_apply.h"
#include "gf256.h"
#include "gf_device.h"
#include "gf_launch.h"

namespace rsgpu {

static_assert(kTabWords == kCoefWords, "host and device table formats differ");

void coef_tables(uint8_t c, uint32_t out[kCoefWords]) {
    const GF &g = gf();
    auto pack = [&](int shift, int j0) {
        uint32_t w = 0;
        for (int j = 0; j < 4; ++j) w |= (uint32_t)g.mul(c, (uint8_t)((j0 + j) << shift)) << (8 * j);
        return w;
    };
    out[0] = pack(0, 0);
    out[1] = pack(0, 4);
    out[2] = pack(3, 0);
    out[3] = pack(3, 4);
    out[4] = pack(6, 0);
}

void Plan::build_tables() {
    tab.assign((size_t)R * K * kTabWords, 0);
    for (int r = 0; r < R; ++r)
        for (int c = 0; c < K; ++c)
            coef_tables(coef[(size_t)r * K + c], &tab[((size_t)r * K + c) * kTabWords]);
    ki = identity_inputs();
}

// trailing identity inputs: input K-ki+j has coefficient 1 in row R-ki+j and
// 0 in every other row
int Plan::identity_inputs() const {
    int n = 0;
    for (int j = 1; j <= std::min(K, R); ++j) {
        const int c = K - j, row = R - j;
        bool unit = true;
        for (int r = 0; r < R && unit; ++r) unit = coef[(size_t)r * K + c] == (r == row ? 1 : 0);
        if (!unit) break;
        n = j;
    }
    return n;
}

Plan::~Plan() {
    retire(d_tab, false);
    retire(d_in_row, false);
    retire(d_tab3, false);
}

// Generic pass for K > 16 inputs (any shard count up to 256) and up to
// kMaxRG = 8 rows per pass: runtime input loop, tables and row indices read
// with scalar loads from device images (constant address space: s_load).
// The wide passes are VALU-bound, so the math is trimmed (tools/kbench
// lib:SHAPE, cold; profiles/r02_kbench_lib_generic_pair_ldst.txt,
// r02_kbench_generic_triples.txt):
//   * inputs go in triples: the 24 index bits of inputs a, b, c are eight
//     3-bit groups, bits [2:0] and [5:3] of each input plus {a[7:6], b[7]}
//     and {b[6], c[7:6]}, and each group is one v_perm lookup into an
//     8-entry table of its row (the two cross groups' tables mix two
//     coefficients).  Per row and dword: 8 v_perm + 4 xor3 for three inputs,
//     against 9 + 4.5 with three single inputs; selectors 17 ops per three
//     input dwords, shared by all rows;
//   * triples are pipelined through their selectors: once a triple's 32
//     selector words exist its inputs are dead, and the next triple's three
//     loads go out into those registers while this triple's rows are coded;
//   * the table words v_perm needs in VGPRs (GFX9's constant bus gives one
//     operand of each lookup its SGPR, the other must be a VGPR) are staged
//     in LDS once per workgroup and read as broadcast ds_read_b128;
//   * K mod 3 leftover inputs go as a pair (6 lookups, 3 xor3) or one input
//     through the 5-word single-coefficient tables;
//   * passes of <= 4 written rows use 8-B lane vectors (VW = 2: half the
//     accumulator and selector registers, 8 waves per SIMD), wider and
//     check-only passes 16 B (launch_generic).
constexpr int kMaxRG = 8;
constexpr int kRowPad = 8;  // row-index image padding past K (the pipelined loads' over-reach)
struct GenericArgs {
    const uint8_t *base;
    uint64_t obj_stride;
    uint32_t *bad;
    const uint32_t *tab;     // [K][rstride][kTabWords], pre-offset to this pass's first row
    const uint32_t *tab3;    // [K/3][rstride][16] triple tables, pre-offset the same way
    const uint32_t *in_row;  // [K + kRowPad] row indices; offset = row * pitch
    uint32_t nvec, tail, nw, span, K, rstride, pitch, clear, packed;
    Order ord;  // item = object
    uint32_t out_off[kMaxRG];
};

// 8-B vector store of the generic kernel's VW = 2 form; `part` (0..7) as in
// store_row: only the row's first `part` bytes of the last vector
template <int SAUX>
__device__ __forceinline__ void store_row8(const u32x2 &o, __amdgpu_buffer_rsrc_t rs, uint32_t voff, uint32_t soff,
                                           uint32_t part) {
    if (part == 0u) {
        __builtin_amdgcn_raw_buffer_store_b64(o, rs, voff, soff, SAUX);
        return;
    }
    uint32_t off = 0, rem = o[0];
    if (part & 4u) {
        __builtin_amdgcn_raw_buffer_store_b32(o[0], rs, voff, soff, SAUX);
        off = 4;
        rem = o[1];
    }
    if (part & 2u) {
        __builtin_amdgcn_raw_buffer_store_b16((unsigned short)rem, rs, voff + off, soff, SAUX);
        off += 2;
        rem >>= 16;
    }
    if (part & 1u) __builtin_amdgcn_raw_buffer_store_b8((unsigned char)rem, rs, voff + off, soff, SAUX);
}

// LDS: [K][R] u32x2 single-input table words 1 and 3, then [K/3][R][8] high
// words of the triple tables (generic_lds)
template <int R, int VW>
__global__ __launch_bounds__(kBlock) void gf_apply_generic(const GenericArgs a) {
    uint32_t obj, chunk;
    if (!wg_item(a.ord, obj, chunk)) return;
    extern __shared__ u32x4 lds_tab[];
    u32x2 *lvw = (u32x2 *)lds_tab;
    for (uint32_t i = threadIdx.x; i < a.K * R; i += kBlock) {
        const uint32_t c = i / R, r = i - c * R;
        const uint32_t *e = a.tab + ((size_t)c * a.rstride + r) * kTabWords;
        lvw[i] = u32x2{e[1], e[3]};
    }
    u32x4 *lv3 = lds_tab + (a.K * R + 1) / 2;
    for (uint32_t i = threadIdx.x; i < a.K / 3 * R * 2; i += kBlock) {
        const uint32_t tr = i >> 1, t = tr / R, r = tr - t * R;
        const uint32_t *e = a.tab3 + ((size_t)t * a.rstride + r) * 16 + 8 + (i & 1) * 4;
        lv3[i] = u32x4{e[0], e[1], e[2], e[3]};
    }
    __syncthreads();
    const uint32_t v = chunk * kBlock + threadIdx.x;
    if (v >= a.nvec) return;
    const uint8_t *ob = a.base + (uint64_t)obj * a.obj_stride;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void *)ob, (short)0, (int)a.span, 0x00020000);
    // loads past the last triple go through a zero-record resource: no memory
    // traffic, and the wait counts stay static
    const __amdgpu_buffer_rsrc_t rsn = __builtin_amdgcn_make_buffer_rsrc((void *)ob, (short)0, 0, 0x00020000);
    const uint32_t voff = v * (4u * VW);
    // one lane's vector of VW dwords (VW = 2: the upper half stays zero, unused)
    auto ldv = [](__amdgpu_buffer_rsrc_t r, uint32_t vo, uint32_t so, int) -> u32x4 {
        if (VW == 4) return __builtin_amdgcn_raw_buffer_load_b128(r, vo, so, kLoadAux);
        const u32x2 t = __builtin_amdgcn_raw_buffer_load_b64(r, vo, so, kLoadAux);
        return u32x4{t[0], t[1], 0u, 0u};
    };
    const constant_ptr<uint32_t> tab = (constant_ptr<uint32_t>)a.tab;
    const constant_ptr<uint32_t> rows = (constant_ptr<uint32_t>)a.in_row;
    uint32_t acc[R][VW];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int d = 0; d < VW; ++d) acc[r][d] = 0;
    // keep the input-at-a-time order: without these fences the scheduler
    // hoists every input's index math and splits the work row by row
    auto fence = [&] {
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int d = 0; d < VW; ++d) asm volatile("" : "+v"(acc[r][d]));
    };
    auto mac_input = [&](const u32x4 &x, uint32_t c) {
        const constant_ptr<uint32_t> t = tab + (size_t)c * a.rstride * kTabWords;
#pragma unroll
        for (int d = 0; d < VW; ++d) {
            const GfIdx g = gf_idx(x[d]);
#pragma unroll
            for (int r = 0; r < R; ++r) acc[r][d] = gf_mac(acc[r][d], t + r * kTabWords, g);
        }
        fence();
    };
    auto mac_pair = [&](const u32x4 &xa, const u32x4 &xb, uint32_t c) {
        const constant_ptr<uint32_t> ta = tab + (size_t)c * a.rstride * kTabWords;
        const constant_ptr<uint32_t> tb = ta + (size_t)a.rstride * kTabWords;
#pragma unroll
        for (int d = 0; d < VW; ++d) {
            const GfIdx ga = gf_idx(xa[d]), gb = gf_idx(xb[d]);
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const constant_ptr<uint32_t> A = ta + r * kTabWords, B = tb + r * kTabWords;
                const u32x2 wa = lvw[c * R + r], wb = lvw[(c + 1) * R + r];
                uint32_t s = xor3(acc[r][d], lut8(A[0], wa[0], ga.i0), lut8(A[2], wa[1], ga.i1));
                s = xor3(s, lut8(A[4], A[4], ga.i2), lut8(B[0], wb[0], gb.i0));
                acc[r][d] = xor3(s, lut8(B[2], wb[1], gb.i1), lut8(B[4], B[4], gb.i2));
            }
        }
        fence();
    };
    // selectors of one triple (the 8 groups above) for the lane's 4 dwords
    auto tri_sel = [&](const u32x4 &xa, const u32x4 &xb, const u32x4 &xc, uint32_t (&sel)[4][8]) {
#pragma unroll
        for (int d = 0; d < VW; ++d) {
            sel[d][0] = xa[d] & 0x07070707u;
            sel[d][1] = (xa[d] >> 3) & 0x07070707u;
            sel[d][2] = xb[d] & 0x07070707u;
            sel[d][3] = (xb[d] >> 3) & 0x07070707u;
            sel[d][4] = xc[d] & 0x07070707u;
            sel[d][5] = (xc[d] >> 3) & 0x07070707u;
            sel[d][6] = ((xa[d] >> 5) & 0x06060606u) | ((xb[d] >> 7) & 0x01010101u);
            sel[d][7] = ((xb[d] >> 6) & 0x01010101u) | ((xc[d] >> 5) & 0x06060606u);
        }
    };
    // triple t into every row: table word w of row r is the SGPR low half
    // T[r][w] and the LDS high half lv3[t][r][w]
    auto tri_rows = [&](const uint32_t (&sel)[4][8], uint32_t t) {
        const constant_ptr<uint32_t> T = (constant_ptr<uint32_t>)a.tab3 + (size_t)t * a.rstride * 16;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const constant_ptr<uint32_t> L = T + r * 16;
            const u32x4 h0 = lv3[(t * R + r) * 2], h1 = lv3[(t * R + r) * 2 + 1];
#pragma unroll
            for (int d = 0; d < VW; ++d) {
                uint32_t q = xor3(acc[r][d], lut8(L[0], h0[0], sel[d][0]), lut8(L[1], h0[1], sel[d][1]));
                q = xor3(q, lut8(L[2], h0[2], sel[d][2]), lut8(L[3], h0[3], sel[d][3]));
                q = xor3(q, lut8(L[4], h1[0], sel[d][4]), lut8(L[5], h1[1], sel[d][5]));
                acc[r][d] = xor3(q, lut8(L[6], h1[2], sel[d][6]), lut8(L[7], h1[3], sel[d][7]));
            }
        }
        fence();
    };
    const uint32_t nt = a.K / 3;
    u32x4 x0, x1, x2;
    auto load3 = [&](uint32_t c) {
        const __amdgpu_buffer_rsrc_t r3 = c < nt * 3 ? rs : rsn;
        x0 = ldv(r3, voff, rows[c] * a.pitch, kLoadAux);
        x1 = ldv(r3, voff, rows[c + 1] * a.pitch, kLoadAux);
        x2 = ldv(r3, voff, rows[c + 2] * a.pitch, kLoadAux);
        asm volatile("" ::: "memory");  // issue here, not sunk into the uses
    };
    load3(0);
    for (uint32_t t = 0; t < nt; ++t) {
        uint32_t sel[4][8];
        tri_sel(x0, x1, x2, sel);
        load3(3 * t + 3);
        tri_rows(sel, t);
    }
    const uint32_t c = nt * 3;
    if (c + 2 <= a.K) {
        const u32x4 y0 = ldv(rs, voff, rows[c] * a.pitch, kLoadAux);
        const u32x4 y1 = ldv(rs, voff, rows[c + 1] * a.pitch, kLoadAux);
        mac_pair(y0, y1, c);
    } else if (c < a.K) {
        mac_input(ldv(rs, voff, rows[c] * a.pitch, kLoadAux), c);
    }
    bool mismatch = false;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        if ((uint32_t)r < a.nw) {
            if (VW == 4) {
                u32x4 o = {acc[r][0], acc[r][1], acc[r][VW > 2 ? 2 : 0], acc[r][VW > 3 ? 3 : 0]};
                store_row<kStoreAux>(o, rs, voff, a.out_off[r], v == a.nvec - 1 ? a.packed : 0u);
            } else {
                store_row8<kStoreAux>(u32x2{acc[r][0], acc[r][1]}, rs, voff, a.out_off[r],
                                      v == a.nvec - 1 ? a.packed : 0u);
            }
        } else {
            const uint32_t valid = (v == a.nvec - 1) ? a.tail : 4u * VW;
#pragma unroll
            for (int d = 0; d < VW; ++d) mismatch |= (acc[r][d] & tail_mask(d, valid)) != 0;
        }
    }
    if (mismatch) a.bad[obj] = 1u;  // same value from every writer: no atomic needed
    if (a.clear && v == 0) a.bad[obj] = 0u;
}

inline unsigned generic_lds(int K, int R) { return (unsigned)((K * R + 1) / 2 * 16 + K / 3 * R * 32); }

// Specialised passes (K <= 16) of the VALU-heavy shapes tri_shape lists
// (rows written or checked): the generic kernel's input triples, with K, R
// and the trailing identity inputs KI known at compile time.  The fused Get
// of RS(10+4) with 2 extra parity shards (K = 12, R = 4: 2 rows written, 2
// checked, KI = 2) issued 1,197 VALU instructions per wave with single
// inputs, at 84 % VALUBusy and a 2.24 GHz held clock against the headline
// encode's 52 % and 2.40 GHz (profiles/r06_sq_dec4_get_single_inputs.json);
// this kernel issues 976 (r06_sq_dec4_get.json).
//   * the G = K - KI GF inputs go as NT = G / 3 triples (8 v_perm + 4 xor3
//     per row and dword for three inputs), the G mod 3 rest as one input or a
//     pair through the 5-word tables; identity inputs are one XOR each;
//   * the low halves of the triple tables are SGPRs (s_load from the plan's
//     device image), the high halves and the single inputs' words 1 and 3 are
//     staged in LDS once per workgroup (GFX9's constant bus: one SGPR per
//     lookup), so no lookup waits for a v_mov;
//   * every input row is loaded up front (K loads in flight per lane, as the
//     single-input kernel); VW = 4 (16-B lanes; 8-B lanes measured slower).
// Tables: the generic kernel's device image (upload_generic: [K][R] single
// words, [K/3][R][16] triples over inputs [0, 3 NT), which are the first
// NT triples of the GF inputs).
template <int K>
struct TriArgs {
    const uint8_t *base;
    uint64_t obj_stride;
    uint32_t *bad;
    const uint32_t *tab;   // [K][rstride][kTabWords]
    const uint32_t *tab3;  // [K/3][rstride][16]
    uint32_t nvec, tail, nw, span, rstride, clear, packed;
    Order ord;  // item = object
    uint32_t in_off[K];
    uint32_t out_off[kMaxR];
};

template <int K, int R, int KI>
struct TriShape {
    static constexpr int G = K - KI, NT = G / 3, NS = G - 3 * NT;
    // LDS: [NS][R] u32x2 words 1 and 3 of the rest inputs, then [NT][R][2]
    // u32x4 high halves of the triple tables
    static constexpr unsigned lds = (unsigned)((NS * R + 1) / 2 * 16 + NT * R * 32);
};

template <int K, int R, int KI, int VW>
__global__ __launch_bounds__(kBlock) void gf_apply_tri(const TriArgs<K> a) {
    using Sh = TriShape<K, R, KI>;
    constexpr int G = Sh::G, NT = Sh::NT, NS = Sh::NS;
    uint32_t obj, chunk;
    if (!wg_item(a.ord, obj, chunk)) return;
    extern __shared__ u32x4 lds_tab[];
    u32x2 *lvw = (u32x2 *)lds_tab;
    for (uint32_t i = threadIdx.x; i < (uint32_t)(NS * R); i += kBlock) {
        const uint32_t c = 3 * NT + i / R, r = i % R;
        const uint32_t *e = a.tab + ((size_t)c * a.rstride + r) * kTabWords;
        lvw[i] = u32x2{e[1], e[3]};
    }
    u32x4 *lv3 = lds_tab + (NS * R + 1) / 2;
    for (uint32_t i = threadIdx.x; i < (uint32_t)(NT * R * 2); i += kBlock) {
        const uint32_t tr = i >> 1, t = tr / R, r = tr - t * R;
        const uint32_t *e = a.tab3 + ((size_t)t * a.rstride + r) * 16 + 8 + (i & 1) * 4;
        lv3[i] = u32x4{e[0], e[1], e[2], e[3]};
    }
    __syncthreads();
    const uint32_t v = chunk * kBlock + threadIdx.x;
    if (v >= a.nvec) return;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(a.base + (uint64_t)obj * a.obj_stride), (short)0, (int)a.span, 0x00020000);
    const uint32_t voff = v * (4u * VW);
    u32x4 x[K];
#pragma unroll
    for (int c = 0; c < K; ++c) {
        if (VW == 4) {
            x[c] = __builtin_amdgcn_raw_buffer_load_b128(rs, voff, a.in_off[c], kLoadAux);
        } else {
            const u32x2 t = __builtin_amdgcn_raw_buffer_load_b64(rs, voff, a.in_off[c], kLoadAux);
            x[c] = u32x4{t[0], t[1], 0u, 0u};
        }
    }
    uint32_t acc[R][VW];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int d = 0; d < VW; ++d) acc[r][d] = 0;
    // one triple (or rest group) at a time: without the fences the scheduler
    // hoists every group's selector math and the registers run out
    auto fence = [&] {
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int d = 0; d < VW; ++d) asm volatile("" : "+v"(acc[r][d]));
        __builtin_amdgcn_sched_barrier(0);
    };
    const constant_ptr<uint32_t> tab = (constant_ptr<uint32_t>)a.tab;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        const u32x4 &xa = x[3 * t], &xb = x[3 * t + 1], &xc = x[3 * t + 2];
        uint32_t sel[VW][8];
#pragma unroll
        for (int d = 0; d < VW; ++d) {
            sel[d][0] = xa[d] & 0x07070707u;
            sel[d][1] = (xa[d] >> 3) & 0x07070707u;
            sel[d][2] = xb[d] & 0x07070707u;
            sel[d][3] = (xb[d] >> 3) & 0x07070707u;
            sel[d][4] = xc[d] & 0x07070707u;
            sel[d][5] = (xc[d] >> 3) & 0x07070707u;
            sel[d][6] = ((xa[d] >> 5) & 0x06060606u) | ((xb[d] >> 7) & 0x01010101u);
            sel[d][7] = ((xb[d] >> 6) & 0x01010101u) | ((xc[d] >> 5) & 0x06060606u);
        }
        const constant_ptr<uint32_t> T = (constant_ptr<uint32_t>)a.tab3 + (size_t)t * a.rstride * 16;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const constant_ptr<uint32_t> L = T + r * 16;
            const u32x4 h0 = lv3[(t * R + r) * 2], h1 = lv3[(t * R + r) * 2 + 1];
#pragma unroll
            for (int d = 0; d < VW; ++d) {
                uint32_t q = xor3(acc[r][d], lut8(L[0], h0[0], sel[d][0]), lut8(L[1], h0[1], sel[d][1]));
                q = xor3(q, lut8(L[2], h0[2], sel[d][2]), lut8(L[3], h0[3], sel[d][3]));
                q = xor3(q, lut8(L[4], h1[0], sel[d][4]), lut8(L[5], h1[1], sel[d][5]));
                acc[r][d] = xor3(q, lut8(L[6], h1[2], sel[d][6]), lut8(L[7], h1[3], sel[d][7]));
            }
        }
        fence();
    }
    if constexpr (NS == 2) {  // a pair: 6 lookups and 3 xor3 per row and dword
        constexpr int c = 3 * NT;
        const constant_ptr<uint32_t> ta = tab + (size_t)c * a.rstride * kTabWords;
        const constant_ptr<uint32_t> tb = ta + (size_t)a.rstride * kTabWords;
#pragma unroll
        for (int d = 0; d < VW; ++d) {
            const GfIdx ga = gf_idx(x[c][d]), gb = gf_idx(x[c + 1][d]);
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const constant_ptr<uint32_t> A = ta + r * kTabWords, B = tb + r * kTabWords;
                const u32x2 wa = lvw[r], wb = lvw[R + r];
                uint32_t s = xor3(acc[r][d], lut8(A[0], wa[0], ga.i0), lut8(A[2], wa[1], ga.i1));
                s = xor3(s, lut8(A[4], A[4], ga.i2), lut8(B[0], wb[0], gb.i0));
                acc[r][d] = xor3(s, lut8(B[2], wb[1], gb.i1), lut8(B[4], B[4], gb.i2));
            }
        }
        fence();
    } else if constexpr (NS == 1) {
        constexpr int c = 3 * NT;
        const constant_ptr<uint32_t> ta = tab + (size_t)c * a.rstride * kTabWords;
#pragma unroll
        for (int d = 0; d < VW; ++d) {
            const GfIdx g = gf_idx(x[c][d]);
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const constant_ptr<uint32_t> A = ta + r * kTabWords;
                const u32x2 w = lvw[r];
                const uint32_t s = xor3(acc[r][d], lut8(A[0], w[0], g.i0), lut8(A[2], w[1], g.i1));
                acc[r][d] = s ^ lut8(A[4], A[4], g.i2);
            }
        }
        fence();
    }
    // identity inputs: input G + j feeds row R - KI + j with coefficient 1
#pragma unroll
    for (int j = 0; j < KI; ++j)
#pragma unroll
        for (int d = 0; d < VW; ++d) acc[R - KI + j][d] ^= x[G + j][d];
    bool mismatch = false;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        if ((uint32_t)r < a.nw) {
            if (VW == 4) {
                const u32x4 o = {acc[r][0], acc[r][1], acc[r][VW > 2 ? 2 : 0], acc[r][VW > 3 ? 3 : 0]};
                store_row<kStoreAux>(o, rs, voff, a.out_off[r], v == a.nvec - 1 ? a.packed : 0u);
            } else {
                store_row8<kStoreAux>(u32x2{acc[r][0], acc[r][1]}, rs, voff, a.out_off[r],
                                      v == a.nvec - 1 ? a.packed : 0u);
            }
        } else {
            const uint32_t valid = (v == a.nvec - 1) ? a.tail : 4u * VW;
#pragma unroll
            for (int d = 0; d < VW; ++d) mismatch |= (acc[r][d] & tail_mask(d, valid)) != 0;
        }
    }
    if (mismatch) a.bad[obj] = 1u;  // same value from every writer: no atomic needed
    if (a.clear && v == 0) a.bad[obj] = 0u;
}

// ----------------------------------------------------------------- launchers

namespace {

struct Sub {  // one pass over <= kMaxR output rows of a plan
    int r0, R, nw;
};

// bytes an object's rows occupy for this plan (through its highest row)
size_t rows_extent(const Plan &p, size_t pitch) {
    int maxrow = 0;
    for (int r : p.in_rows) maxrow = std::max(maxrow, r);
    for (int r : p.out_rows) maxrow = std::max(maxrow, r);
    return (size_t)(maxrow + 1) * pitch;
}


template <int K, int R>
void fill_pass(const Plan &p, const Sub &s, size_t pitch, size_t space, uint32_t nvec, bool have_bad, Pass<K, R> &a) {
    a.nw = (uint32_t)s.nw;
    // identity inputs feed the plan's last ki rows; usable only when this
    // pass is the plan's last pass (it holds those rows at the same offsets)
    a.ki = (s.r0 + R == p.R) ? (uint32_t)std::min(p.ki, R) : 0u;
    a.clear = (have_bad && p.nw == p.R) ? 1u : 0u;
    a.packed = tail_part(space, nvec);
    a.sub_stride = a.sub_len = a.sub_n = 0;
    int maxrow = 0;
    for (int c = 0; c < K; ++c) {
        a.in_off[c] = (uint32_t)(p.in_rows[c] * pitch);
        maxrow = std::max(maxrow, p.in_rows[c]);
    }
    for (int r = 0; r < R; ++r) {
        const int row = p.out_rows[s.r0 + r];
        a.out_off[r] = (uint32_t)((row < 0 ? 0 : row) * pitch);
        maxrow = std::max(maxrow, row);
        for (int c = 0; c < K; ++c)
            for (int g = 0; g < kTabWords; ++g)
                a.tab[(c * R + r) * kTabWords + g] = p.tab[((size_t)(s.r0 + r) * K + c) * kTabWords + g];
    }
    a.span = (uint32_t)((size_t)maxrow * pitch + (size_t)nvec * 16);
}

// Input-triple tables of a sub-pass (Pass3): the GF inputs [0, K - ki) in
// triples, entries of the 8 tables per (triple, row) as gf_apply_body reads them
template <int K, int R>
void fill_triples(const Plan &p, const Sub &s, Pass3<K, R> &a) {
    const GF &g = gf();
    a.ntrip = (uint32_t)((K - (int)a.ki) / 3);
    std::memset(a.tab3, 0, sizeof(a.tab3));
    for (uint32_t t = 0; t < a.ntrip; ++t)
        for (int r = 0; r < R; ++r) {
            const size_t row = (size_t)(s.r0 + r) * K;
            const uint8_t ca = p.coef[row + 3 * t], cb = p.coef[row + 3 * t + 1], cc = p.coef[row + 3 * t + 2];
            uint32_t *w = &a.tab3[((size_t)t * R + r) * 16];
            for (int j = 0; j < 8; ++j) {
                const uint8_t ent[8] = {
                    g.mul(ca, (uint8_t)j), g.mul(ca, (uint8_t)(j << 3)), g.mul(cb, (uint8_t)j), g.mul(cb, (uint8_t)(j << 3)),
                    g.mul(cc, (uint8_t)j), g.mul(cc, (uint8_t)(j << 3)),
                    (uint8_t)(g.mul(ca, (uint8_t)((j >> 1) << 6)) ^ g.mul(cb, (uint8_t)((j & 1) << 7))),
                    (uint8_t)(g.mul(cb, (uint8_t)((j & 1) << 6)) ^ g.mul(cc, (uint8_t)((j >> 1) << 6)))};
                for (int q = 0; q < 8; ++q) w[q + (j >> 2) * 8] |= (uint32_t)ent[q] << (8 * (j & 3));
            }
        }
}

// Check-only passes of >= 3 rows are VALU-bound (Verify RS(10+4): 14 inputs
// x 4 check rows): their GF inputs go in triples (Pass3).  Verify RS(10+4)
// 75.4-76.3 -> 79.1-81.6 %; passes that store rows do not gain (encode
// RS(10+4) 72 % either way, the decode with checks loses 2-3 points;
// profiles/r03_kbench_tri_{off,on}.txt).  RSGPU_TRIPLES=0 / 2 (off / every
// pass of >= 3 rows) overrides, for measurement.
inline bool use_triples(int K, int R, int ki, int nw) {
    static const int env = [] {
        const char *e = std::getenv("RSGPU_TRIPLES");
        return e ? std::atoi(e) : -1;
    }();
    if (env == 0) return false;
    if (env == 2) return R >= 3 && K - ki >= 6;  // every pass of >= 3 rows
    return R >= 3 && K - ki >= 6 && nw == 0;
}

// LDS reservation (occupancy cap) of a pass: store_lds(K) for passes that
// store rows, none for check-only passes; RSGPU_MIXED_W=w overrides the cap
// of passes that both store and check rows (measurement)
inline unsigned pass_lds(int K, int nw, int R) {
    if (nw == 0) return 0u;
    static const int mixed_w = [] {
        const char *e = std::getenv("RSGPU_MIXED_W");
        return e ? std::atoi(e) : 0;
    }();
    if (nw < R && mixed_w > 0) return mixed_w >= 8 ? 0u : 160u * 1024u / (unsigned)mixed_w - 256u;
    // passes that store rows AND check rows (the fused decode with extra
    // parity shards) carry the check rows' VALU work: one workgroup more per
    // CU than store_lds gives them (RS(10+4) decode with 2 checks, K = 12:
    // W = 4 69.7-70.2 % vs W = 3 68.7-69.0 %, W = 6 / uncapped 68.5-68.9 %;
    // input triples on this pass lose 0.3-3 points at every W;
    // profiles/r03_kbench_dec10_4_sweep.txt)
    if (nw < R) return K <= 10 ? store_lds(K) : 160u * 1024u / 4u - 256u;
    return store_lds(K);
}

// The LDS-staged small-object form (gf_apply_staged) for rows of at most
// kStagedMaxVec whole vectors of an object-major batch; RSGPU_STAGED=0 turns
// it off (measurement)
template <int K, int R>
inline bool use_staged(uint32_t nvec, const Pass<K, R> &p) {
    static const bool on = [] {
        const char *e = std::getenv("RSGPU_STAGED");
        return !e || std::atoi(e) != 0;
    }();
    return on && nvec <= kStagedMaxVec && p.packed == 0 && p.sub_stride == 0;
}

template <int K, int R>
hipError_t launch_fixed(const Plan &p, const Sub &s, const Layout &L, uint32_t *d_bad,
                        hipStream_t st);

// The same launch with the pass's GF inputs in triples (chunk and small-object forms)
template <int K, int R>
hipError_t launch_fixed3(const Plan &p, const Sub &s, const Layout &L, uint32_t *d_bad, hipStream_t st);

// the triples kernel for this pass, when it has one (launch_tri, below);
// returns false when the pass takes the single-input kernel
template <int K, int R>
bool launch_tri(const Plan &p, const Sub &s, const Layout &L, uint32_t *d_bad, hipStream_t st, hipError_t &e);

template <int K, int R>
hipError_t launch_fixed(const Plan &p, const Sub &s, const Layout &L, uint32_t *d_bad,
                        hipStream_t st) {
    if constexpr (R >= 3 && K >= 6) {
        hipError_t e = hipSuccess;
        if (launch_tri<K, R>(p, s, L, d_bad, st, e)) return e;
        const int ki = (s.r0 + R == p.R) ? std::min(p.ki, R) : 0;
        if (!L.in_base && !L.out_base && use_triples(K, R, ki, s.nw)) return launch_fixed3<K, R>(p, s, L, d_bad, st);
    }
    ApplyArgs<K, R> a;
    a.obj_stride = L.obj_stride;
    a.nvec = (uint32_t)((L.shard_len + 15) / 16);
    a.tail = (uint32_t)(L.shard_len - (size_t)(a.nvec - 1) * 16);
    fill_pass<K, R>(p, s, L.pitch, row_space(L), a.nvec, d_bad != nullptr, a.p);
    a.p.sub_stride = L.sub_stride;
    a.p.sub_len = L.sub_len;
    a.p.sub_n = L.sub_n;
    const unsigned gx = (a.nvec + kBlock * kUnroll - 1) / (kBlock * kUnroll);
    // Small objects (a row of at most half a workgroup's vectors): one
    // workgroup codes opw whole objects, so its lanes stay busy (1 KiB
    // objects: 7 of 256 lanes otherwise).  The group's objects must lie in
    // one 32-bit buffer range.
    a.opw = 1;
    a.nobj = 0;
    a.gspan = 0;
    if (L.nobj > 1 && !L.in_base && !L.out_base && kUnroll == 1 && a.nvec * 2 <= kBlock) {
        uint32_t opw = kBlock / a.nvec;
        while (opw > 1 && (uint64_t)(opw - 1) * L.obj_stride + a.p.span >= 0xffffffffull) opw /= 2;
        if (opw > 1) {
            a.opw = opw;
            a.gspan = (uint32_t)((uint64_t)(opw - 1) * L.obj_stride + a.p.span);
            const int groups = (L.nobj + (int)opw - 1) / (int)opw;
            for (int g0 = 0; g0 < groups; g0 += max_items(1)) {
                const int ng = std::min(max_items(1), groups - g0);
                const size_t o0 = (size_t)g0 * opw;
                a.base = L.base + o0 * L.obj_stride;
                a.bad = d_bad ? d_bad + o0 : nullptr;
                a.nobj = (uint32_t)std::min<size_t>((size_t)ng * opw, (size_t)L.nobj - o0);
                unsigned grid;
                a.ord = make_order(1, (uint32_t)ng, (size_t)a.nobj * L.obj_stride, grid);
                // rows of <= 8 vectors (objects of ~1 KiB) staged through LDS
                // so that every wave load is ~1 KiB of consecutive rows
                // (gf_apply_staged); longer rows lose with it (kbench KB_SET=
                // small: -7 / -4 points at 4 / 16 KiB)
                if (use_staged(a.nvec, a.p)) {
                    const unsigned lds = opw * (unsigned)(K + R) * a.nvec * 16u;
                    hipLaunchKernelGGL((gf_apply_staged<K, R, kLoadAux, kStoreAux>), dim3(grid), dim3(kBlock),
                                       std::max(lds, pass_lds(K, (int)a.p.nw, R)), st, a);
                } else {
                    hipLaunchKernelGGL((gf_apply_kernel<K, R, kUnroll, kBlock, kLoadAux, kStoreAux, kFormSmall>),
                                       dim3(grid), dim3(kBlock), pass_lds(K, (int)a.p.nw, R), st, a);
                }
                hipError_t e = hipGetLastError();
                if (e != hipSuccess) return e;
            }
            return hipSuccess;
        }
    }
    const int step = max_items(gx);
    for (int o0 = 0; o0 < L.nobj; o0 += step) {
        const int no = std::min(step, L.nobj - o0);
        a.base = L.base + (size_t)o0 * L.obj_stride;
        a.out_base = L.out_base;  // redirection is single-object (nobj == 1, checked)
        a.out_dual = L.out_dual ? 1u : 0u;
        a.in_base = L.in_base;
        a.in_span = (uint32_t)std::min<size_t>(L.in_span, 0xffffffffu);
        a.copy_in = L.copy_in ? 1u : 0u;
        a.bad = d_bad ? d_bad + o0 : nullptr;
        unsigned grid;
        a.ord = make_order(gx, (uint32_t)no, objs_span(L, no, a.p.span), grid);
        if (L.in_base || L.out_base)
            hipLaunchKernelGGL((gf_apply_kernel<K, R, kUnroll, kBlock, kLoadAux, kStoreAux, kFormRedirect>),
                               dim3(grid), dim3(kBlock), pass_lds(K, (int)a.p.nw, R), st, a);
        else
            hipLaunchKernelGGL((gf_apply_kernel<K, R, kUnroll, kBlock, kLoadAux, kStoreAux, kFormChunks>),
                               dim3(grid), dim3(kBlock), pass_lds(K, (int)a.p.nw, R), st, a);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

template <int K, int R>
hipError_t launch_fixed3(const Plan &p, const Sub &s, const Layout &L, uint32_t *d_bad, hipStream_t st) {
    ApplyArgs<K, R, Pass3<K, R>> a;
    a.obj_stride = L.obj_stride;
    a.nvec = (uint32_t)((L.shard_len + 15) / 16);
    a.tail = (uint32_t)(L.shard_len - (size_t)(a.nvec - 1) * 16);
    fill_pass<K, R>(p, s, L.pitch, row_space(L), a.nvec, d_bad != nullptr, a.p);
    fill_triples<K, R>(p, s, a.p);
    a.p.sub_stride = L.sub_stride;
    a.p.sub_len = L.sub_len;
    a.p.sub_n = L.sub_n;
    a.in_base = a.out_base = nullptr;
    a.in_span = a.copy_in = a.out_dual = 0;
    const unsigned gx = (a.nvec + kBlock * kUnroll - 1) / (kBlock * kUnroll);
    a.opw = 1;
    a.nobj = 0;
    a.gspan = 0;
    if (L.nobj > 1 && kUnroll == 1 && a.nvec * 2 <= kBlock) {  // small objects: as launch_fixed
        uint32_t opw = kBlock / a.nvec;
        while (opw > 1 && (uint64_t)(opw - 1) * L.obj_stride + a.p.span >= 0xffffffffull) opw /= 2;
        if (opw > 1) {
            a.opw = opw;
            a.gspan = (uint32_t)((uint64_t)(opw - 1) * L.obj_stride + a.p.span);
            const int groups = (L.nobj + (int)opw - 1) / (int)opw;
            for (int g0 = 0; g0 < groups; g0 += max_items(1)) {
                const int ng = std::min(max_items(1), groups - g0);
                const size_t o0 = (size_t)g0 * opw;
                a.base = L.base + o0 * L.obj_stride;
                a.bad = d_bad ? d_bad + o0 : nullptr;
                a.nobj = (uint32_t)std::min<size_t>((size_t)ng * opw, (size_t)L.nobj - o0);
                unsigned grid;
                a.ord = make_order(1, (uint32_t)ng, (size_t)a.nobj * L.obj_stride, grid);
                hipLaunchKernelGGL((gf_apply_kernel<K, R, kUnroll, kBlock, kLoadAux, kStoreAux, kFormSmall, true>),
                                   dim3(grid), dim3(kBlock), pass_lds(K, (int)a.p.nw, R), st, a);
                hipError_t e = hipGetLastError();
                if (e != hipSuccess) return e;
            }
            return hipSuccess;
        }
    }
    const int step = max_items(gx);
    for (int o0 = 0; o0 < L.nobj; o0 += step) {
        const int no = std::min(step, L.nobj - o0);
        a.base = L.base + (size_t)o0 * L.obj_stride;
        a.bad = d_bad ? d_bad + o0 : nullptr;
        unsigned grid;
        a.ord = make_order(gx, (uint32_t)no, objs_span(L, no, a.p.span), grid);
        hipLaunchKernelGGL((gf_apply_kernel<K, R, kUnroll, kBlock, kLoadAux, kStoreAux, kFormChunks, true>),
                           dim3(grid), dim3(kBlock), pass_lds(K, (int)a.p.nw, R), st, a);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

// ---- mixed-pattern launch: one (K, R) class of (plan, sub-pass) entries

struct Entry {  // one sub-pass of one plan and the objects that use it
    const Plan *plan;
    Sub sub;
    std::vector<uint32_t> objs;
};

// Appends this class's device image — passes[], then objs[], obj_pass[] —
// to `img` (16-B aligned pieces) and returns the launch closure.
template <int K, int R>
std::function<hipError_t(const uint8_t *dimg, hipStream_t)> stage_class(
    const std::vector<const Entry *> &es, const Layout &L, uint32_t *d_bad, std::vector<uint8_t> &img) {
    const uint32_t nvec = (uint32_t)((L.shard_len + 15) / 16);
    auto align = [&]() { img.resize((img.size() + 15) & ~(size_t)15); };
    align();
    const size_t pass_off = img.size();
    img.resize(pass_off + es.size() * sizeof(Pass<K, R>));
    size_t nobj = 0;
    for (size_t i = 0; i < es.size(); ++i) {
        // the pass image depends on (plan, pitch, sub-pass, flags): cache it in the plan
        Plan &pl = const_cast<Plan &>(*es[i]->plan);
        const std::array<uint64_t, 3> key{L.pitch * 2 + (d_bad != nullptr), (uint64_t)es[i]->sub.r0,
                                          (uint64_t)row_space(L) << 32 | nvec};
        const std::vector<uint8_t> *cached = nullptr;
        {
            std::lock_guard<std::mutex> g(pl.img_mu);
            for (auto &kv : pl.pass_imgs)
                if (kv.first == key && kv.second.size() == sizeof(Pass<K, R>)) cached = &kv.second;
            if (!cached) {
                Pass<K, R> pp;
                fill_pass<K, R>(pl, es[i]->sub, L.pitch, row_space(L), nvec, d_bad != nullptr, pp);
                std::vector<uint8_t> b(sizeof(pp));
                std::memcpy(b.data(), &pp, sizeof(pp));
                if (pl.pass_imgs.size() > 16) pl.pass_imgs.clear();
                pl.pass_imgs.emplace_back(key, std::move(b));
                cached = &pl.pass_imgs.back().second;
            }
            std::memcpy(&img[pass_off + i * sizeof(Pass<K, R>)], cached->data(), sizeof(Pass<K, R>));
        }
        nobj += es[i]->objs.size();
    }
    bool stores = false;
    for (const Entry *e : es) stores |= e->sub.nw > 0;
    // Small objects (rows of <= half a workgroup's vectors): a workgroup codes
    // opw objects of ONE pattern (sorted by pattern, address order within),
    // lanes addressing object o at o * obj_stride from the batch base — so
    // the batch must lie in one 32-bit buffer range.
    uint32_t maxobj = 0;
    for (const Entry *e : es)
        for (uint32_t o : e->objs) maxobj = std::max(maxobj, o);
    const size_t gspan = (size_t)maxobj * L.obj_stride + (size_t)L.pitch * 256;  // >= any pass span
    if (kUnroll == 1 && nvec * 2 <= kBlock && gspan <= 0xffffffffull) {
        const uint32_t opw = kBlock / nvec;
        size_t ngroups = 0;
        for (const Entry *e : es) ngroups += (e->objs.size() + opw - 1) / opw;
        align();
        const size_t objs_off = img.size();
        img.resize(objs_off + ngroups * (opw + 1) * 4);
        uint32_t *gobjs = (uint32_t *)&img[objs_off], *gpass = gobjs + ngroups * opw;
        size_t g = 0;
        for (size_t i = 0; i < es.size(); ++i) {
            const std::vector<uint32_t> &os = es[i]->objs;  // ascending (launch_plans_multi)
            for (size_t a = 0; a < os.size(); a += opw, ++g) {
                for (uint32_t j = 0; j < opw; ++j) gobjs[g * opw + j] = a + j < os.size() ? os[a + j] : 0xffffffffu;
                gpass[g] = (uint32_t)i;
            }
        }
        return [=](const uint8_t *dimg, hipStream_t st) -> hipError_t {
            MultiArgs<K, R> m;
            m.base = L.base;
            m.obj_stride = L.obj_stride;
            m.bad = d_bad;
            m.nvec = nvec;
            m.tail = (uint32_t)(L.shard_len - (size_t)(nvec - 1) * 16);
            m.passes = (const Pass<K, R> *)(dimg + pass_off);
            m.objs = (const uint32_t *)(dimg + objs_off);
            m.obj_pass = m.objs + ngroups * opw;
            m.opw = opw;
            m.gspan = (uint32_t)gspan;
            unsigned grid;
            m.ord = make_order(1, (uint32_t)ngroups, gspan, grid);
            hipLaunchKernelGGL((gf_apply_multi<K, R, kUnroll, kBlock, kLoadAux, kStoreAux, kMultiChunks>),
                               dim3(grid), dim3(kBlock), stores ? store_lds(K) : 0u, st, m);
            return hipGetLastError();
        };
    }
    align();
    const size_t objs_off = img.size();
    img.resize(objs_off + nobj * 8);
    uint32_t *objs = (uint32_t *)&img[objs_off], *pidx = objs + nobj;
    // items in object (address) order, not grouped by pattern: each XCD then
    // sweeps its share of the batch in sequence (grouped order hopped across
    // the batch: 9 % slower cold, profiles/r01_kernel_stats_mixed.csv)
    std::vector<std::pair<uint32_t, uint32_t>> items;
    items.reserve(nobj);
    for (size_t i = 0; i < es.size(); ++i)
        for (uint32_t o : es[i]->objs) items.emplace_back(o, (uint32_t)i);
    std::sort(items.begin(), items.end());
    for (size_t j = 0; j < items.size(); ++j) {
        objs[j] = items[j].first;
        pidx[j] = items[j].second;
    }
    return [=](const uint8_t *dimg, hipStream_t st) -> hipError_t {
        MultiArgs<K, R> m;
        m.opw = 1;
        m.gspan = 0;
        m.base = L.base;
        m.obj_stride = L.obj_stride;
        m.bad = d_bad;
        m.nvec = nvec;
        m.tail = (uint32_t)(L.shard_len - (size_t)(nvec - 1) * 16);
        m.passes = (const Pass<K, R> *)(dimg + pass_off);
        const unsigned per = kBlock * kUnroll * kMultiChunks;
        const unsigned gx = (nvec + per - 1) / per;
        const size_t step = (size_t)max_items(gx);
        for (size_t o0 = 0; o0 < nobj; o0 += step) {
            const int no = (int)std::min(step, nobj - o0);
            m.objs = (const uint32_t *)(dimg + objs_off) + o0;
            m.obj_pass = (const uint32_t *)(dimg + objs_off) + nobj + o0;
            unsigned grid;
            m.ord = make_order(gx, (uint32_t)no, objs_span(L, no, L.pitch * 256), grid);
            hipLaunchKernelGGL((gf_apply_multi<K, R, kUnroll, kBlock, kLoadAux, kStoreAux, kMultiChunks>),
                               dim3(grid), dim3(kBlock), stores ? store_lds(K) : 0u, st, m);
            hipError_t e = hipGetLastError();
            if (e != hipSuccess) return e;
        }
        return hipSuccess;
    };
}

typedef std::function<hipError_t(const uint8_t *, hipStream_t)> (*stage_fn)(
    const std::vector<const Entry *> &, const Layout &, uint32_t *, std::vector<uint8_t> &);

template <int K>
stage_fn pick_stage_r(int R) {
    return R == 1 ? &stage_class<K, 1> : R == 2 ? &stage_class<K, 2> : R == 3 ? &stage_class<K, 3>
                                                                                : &stage_class<K, 4>;
}

stage_fn pick_stage(int K, int R) {
    switch (K) {
#define RSGPU_K(k) case k: return pick_stage_r<k>(R);
        RSGPU_K(1) RSGPU_K(2) RSGPU_K(3) RSGPU_K(4) RSGPU_K(5) RSGPU_K(6) RSGPU_K(7) RSGPU_K(8)
        RSGPU_K(9) RSGPU_K(10) RSGPU_K(11) RSGPU_K(12) RSGPU_K(13) RSGPU_K(14) RSGPU_K(15)
        RSGPU_K(16)
#undef RSGPU_K
        default: return nullptr;
    }
}

// Uploads the generic kernel's [K][R][kTabWords] table image, its triple
// tables and row indices (Plan::d_*); on failure frees what it allocated.
static hipError_t upload_generic(Plan &p) {
    const int K = p.K;
    // rows padded: the pipelined loads reach up to 3 rows past the last
    // triple (through a zero-record resource)
    std::vector<uint32_t> t((size_t)K * p.R * kTabWords), rows(K + kRowPad, 0);
    for (int c = 0; c < K; ++c) {
        rows[c] = (uint32_t)p.in_rows[c];
        for (int r = 0; r < p.R; ++r)
            for (int g = 0; g < kTabWords; ++g)
                t[((size_t)c * p.R + r) * kTabWords + g] = p.tab[((size_t)r * K + c) * kTabWords + g];
    }
    // input-triple tables [K/3][R][16]: words 0-7 the low halves (entries
    // 0-3) of the eight 8-entry tables, words 8-15 their high halves
    const GF &gf_ = gf();
    const int nt = K / 3;
    std::vector<uint32_t> t3((size_t)std::max(1, nt) * p.R * 16, 0);
    for (int tr = 0; tr < nt; ++tr)
        for (int r = 0; r < p.R; ++r) {
            const uint8_t ca = p.coef[(size_t)r * K + 3 * tr], cb = p.coef[(size_t)r * K + 3 * tr + 1],
                          cc = p.coef[(size_t)r * K + 3 * tr + 2];
            uint32_t *w = &t3[((size_t)tr * p.R + r) * 16];
            for (int j = 0; j < 8; ++j) {
                const uint8_t ent[8] = {
                    gf_.mul(ca, (uint8_t)j), gf_.mul(ca, (uint8_t)(j << 3)),
                    gf_.mul(cb, (uint8_t)j), gf_.mul(cb, (uint8_t)(j << 3)),
                    gf_.mul(cc, (uint8_t)j), gf_.mul(cc, (uint8_t)(j << 3)),
                    (uint8_t)(gf_.mul(ca, (uint8_t)((j >> 1) << 6)) ^ gf_.mul(cb, (uint8_t)((j & 1) << 7))),
                    (uint8_t)(gf_.mul(cb, (uint8_t)((j & 1) << 6)) ^ gf_.mul(cc, (uint8_t)((j >> 1) << 6)))};
                for (int g = 0; g < 8; ++g) w[g + (j >> 2) * 8] |= (uint32_t)ent[g] << (8 * (j & 3));
            }
        }
    hipError_t e = hipMalloc(&p.d_tab, t.size() * 4);
    if (e == hipSuccess) e = hipMalloc(&p.d_tab3, t3.size() * 4);
    if (e == hipSuccess) e = upload(p.d_tab3, t3.data(), t3.size() * 4);
    if (e == hipSuccess) e = hipMalloc(&p.d_in_row, rows.size() * 4);
    if (e == hipSuccess) e = upload(p.d_tab, t.data(), t.size() * 4);
    if (e == hipSuccess) e = upload(p.d_in_row, rows.data(), rows.size() * 4);
    if (e != hipSuccess) {
        for (uint32_t **d : {&p.d_tab, &p.d_tab3, &p.d_in_row}) {
            retire(*d, false);
            *d = nullptr;
        }
        return e;
    }
    return hipSuccess;
}

template <int R>
hipError_t launch_generic(Plan &p, const Sub &s, const Layout &L, uint32_t *d_bad,
                          hipStream_t st) {
    const int K = p.K;
    // upload once per plan (a failed upload is freed and retried by the next
    // launch: one transient hipMalloc failure must not disable the plan for
    // the context's life)
    if (!p.dev_done.load(std::memory_order_acquire)) {
        std::lock_guard<std::mutex> g(p.dev_mu);
        if (!p.dev_done.load(std::memory_order_relaxed)) {
            const hipError_t e = upload_generic(p);
            if (e != hipSuccess) return e;
            p.dev_done.store(true, std::memory_order_release);
        }
    }
    // 8-B lane vectors for narrow passes that write rows: 51 VGPRs at R = 4
    // (8 waves) against 81 (5 waves); RS(20+4) encode +2.5, RS(17+3) +3
    // points, the wide encode+decode workload +3 %.  Wider passes and
    // check-only passes keep 16 B (R = 8: -1 to -3 points; Verify -1.4)
    // (profiles/r02_kbench_generic_vw2*.txt)
    const int vw = (R <= 4 && s.nw > 0) ? 2 : 4;
    const uint32_t vb = vw == 2 ? 8u : 16u;  // bytes per lane vector
    GenericArgs a;
    a.obj_stride = L.obj_stride;
    a.nvec = (uint32_t)((L.shard_len + vb - 1) / vb);
    a.tail = (uint32_t)(L.shard_len - (size_t)(a.nvec - 1) * vb);
    a.nw = (uint32_t)s.nw;
    a.K = (uint32_t)K;
    a.rstride = (uint32_t)p.R;
    a.tab = p.d_tab + (size_t)s.r0 * kTabWords;
    a.tab3 = p.d_tab3 + (size_t)s.r0 * 16;
    a.in_row = p.d_in_row;
    a.pitch = (uint32_t)L.pitch;
    {
        const size_t w = row_space(L) - (size_t)(a.nvec - 1) * vb;
        a.packed = w < vb ? (uint32_t)w : 0u;
    }
    int maxrow = 0;
    for (int c = 0; c < K; ++c) maxrow = std::max(maxrow, p.in_rows[c]);
    for (int r = 0; r < R; ++r) {
        const int row = p.out_rows[s.r0 + r];
        a.out_off[r] = (uint32_t)((row < 0 ? 0 : row) * L.pitch);
        maxrow = std::max(maxrow, row);
    }
    a.span = (uint32_t)((size_t)maxrow * L.pitch + (size_t)a.nvec * vb);
    const unsigned gx = (a.nvec + kBlock - 1) / kBlock;
    const int step = max_items(gx);
    for (int o0 = 0; o0 < L.nobj; o0 += step) {
        const int no = std::min(step, L.nobj - o0);
        a.base = L.base + (size_t)o0 * L.obj_stride;
        a.bad = d_bad ? d_bad + o0 : nullptr;
        a.clear = (d_bad && p.nw == p.R) ? 1u : 0u;
        unsigned grid;
        a.ord = make_order(gx, (uint32_t)no, objs_span(L, no, a.span), grid);
        // full occupancy: the wide generic passes are VALU-bound (caps of 2-6
        // workgroups per CU lose 0.4-9 points, r02_kbench_generic_caps_pipelined.txt)
        if (vw == 2)
            hipLaunchKernelGGL((gf_apply_generic<R, 2>), dim3(grid), dim3(kBlock), generic_lds(K, R), st, a);
        else
            hipLaunchKernelGGL((gf_apply_generic<R, 4>), dim3(grid), dim3(kBlock), generic_lds(K, R), st, a);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

// Which passes take gf_apply_tri (set_tri_mode): 1 (default) every pass of
// an instantiated shape (tri_shape) over rows longer than 128 vectors; 0 none
// (the single-input kernel and, for check-only passes, its Pass3 triples).
// Cold, tools/kbench KB_SET=tri (profiles/r06_kbench_tri_*.txt), single
// inputs -> gf_apply_tri:
//   fused Get RS(10+4), 2 extra shards, 4 MiB: 72.7 -> 72.5 % (HBM-bound at
//     that size: VALUBusy 84 -> 68 %, WAIT_ANY 31 -> 55 % of wave cycles);
//     1 MiB 70.5 -> 72.6 %
//   encode RS(10+4) 4 MiB 73.5 -> 74.3 %;  Verify RS(10+4) 82.7 -> 87.9 %
//   (the XOR-only kernel on the same streams: 88.3 %)
// 8-B lanes lost 1.6-6.5 points on every shape (66.0 / 67.3 / 69.7 / 84.5 %).
// RSGPU_TRI sets the mode at load (measurement)
int env_int(const char *name, int dflt) {
    const char *e = std::getenv(name);
    return e ? std::atoi(e) : dflt;
}
std::atomic<int> g_tri_mode{env_int("RSGPU_TRI", 1)};

// (K, R, KI) shapes with a gf_apply_tri instantiation: the fused RS(10+4) Get
// with 2 extra shards (12, 4, 2) or 1 (11, 4, 1: 3 data shards lost), the
// RS(10+4) encode (10, 4, 0), and Verify of RS(10+4) (14, 4, 4), RS(10+3)
// (13, 3, 3) and RS(12+4) (16, 4, 4).  bench.py's kernel names follow this
// list (bench.py tri_shape).
constexpr bool tri_shape(int K, int R, int KI) {
    return (K == 12 && R == 4 && KI == 2) || (K == 11 && R == 4 && KI == 1) || (K == 10 && R == 4 && KI == 0) ||
           (K == 14 && R == 4 && KI == 4) || (K == 13 && R == 3 && KI == 3) || (K == 16 && R == 4 && KI == 4);
}

template <int K, int R, int KI, int VW>
hipError_t launch_tri_k(Plan &p, const Sub &s, const Layout &L, uint32_t *d_bad, hipStream_t st) {
    using Sh = TriShape<K, R, KI>;
    constexpr uint32_t vb = 4u * VW;  // bytes per lane vector
    TriArgs<K> a;
    a.obj_stride = L.obj_stride;
    a.nvec = (uint32_t)((L.shard_len + vb - 1) / vb);
    a.tail = (uint32_t)(L.shard_len - (size_t)(a.nvec - 1) * vb);
    a.nw = (uint32_t)s.nw;
    a.rstride = (uint32_t)p.R;
    a.tab = p.d_tab + (size_t)s.r0 * kTabWords;
    a.tab3 = p.d_tab3 + (size_t)s.r0 * 16;
    a.clear = (d_bad && p.nw == p.R) ? 1u : 0u;
    {
        const size_t w = row_space(L) - (size_t)(a.nvec - 1) * vb;
        a.packed = w < vb ? (uint32_t)w : 0u;
    }
    int maxrow = 0;
    for (int c = 0; c < K; ++c) {
        a.in_off[c] = (uint32_t)(p.in_rows[c] * L.pitch);
        maxrow = std::max(maxrow, p.in_rows[c]);
    }
    for (int r = 0; r < kMaxR; ++r) {
        const int row = r < R ? p.out_rows[s.r0 + r] : 0;
        a.out_off[r] = (uint32_t)((row < 0 ? 0 : row) * L.pitch);
        maxrow = std::max(maxrow, row);
    }
    a.span = (uint32_t)((size_t)maxrow * L.pitch + (size_t)a.nvec * vb);
    const unsigned gx = (a.nvec + kBlock - 1) / kBlock;
    const int step = max_items(gx);
    const unsigned lds = std::max(Sh::lds, pass_lds(K, s.nw, R));
    for (int o0 = 0; o0 < L.nobj; o0 += step) {
        const int no = std::min(step, L.nobj - o0);
        a.base = L.base + (size_t)o0 * L.obj_stride;
        a.bad = d_bad ? d_bad + o0 : nullptr;
        unsigned grid;
        a.ord = make_order(gx, (uint32_t)no, objs_span(L, no, a.span), grid);
        hipLaunchKernelGGL((gf_apply_tri<K, R, KI, VW>), dim3(grid), dim3(kBlock), lds, st, a);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

template <int K, int R>
bool launch_tri(const Plan &pc, const Sub &s, const Layout &L, uint32_t *d_bad, hipStream_t st, hipError_t &e) {
    if (g_tri_mode.load(std::memory_order_relaxed) == 0 || L.in_base || L.out_base || L.sub_stride ||
        s.r0 != 0 || s.R != pc.R)
        return false;
    if ((L.shard_len + 15) / 16 * 2 <= (size_t)kBlock) return false;  // small objects: the packed forms
    const int ki = std::min(pc.ki, R);
    Plan &p = const_cast<Plan &>(pc);
    auto ready = [&]() -> bool {  // the plan's table image (upload_generic), once
        if (p.dev_done.load(std::memory_order_acquire)) return true;
        std::lock_guard<std::mutex> g(p.dev_mu);
        if (!p.dev_done.load(std::memory_order_relaxed)) {
            if ((e = upload_generic(p)) != hipSuccess) return false;
            p.dev_done.store(true, std::memory_order_release);
        }
        return true;
    };
#define RSGPU_TRI(KI_)                                                \
    if constexpr (tri_shape(K, R, KI_)) {                             \
        if (ki == KI_) {                                              \
            if (!ready()) return e != hipSuccess;                     \
            e = launch_tri_k<K, R, KI_, 4>(p, s, L, d_bad, st);       \
            return true;                                              \
        }                                                             \
    }
    RSGPU_TRI(0) RSGPU_TRI(1) RSGPU_TRI(2) RSGPU_TRI(3) RSGPU_TRI(4)
#undef RSGPU_TRI
    return false;
}

typedef hipError_t (*fixed_fn)(const Plan &, const Sub &, const Layout &, uint32_t *, hipStream_t);

template <int K>
constexpr fixed_fn pick_r(int R) {
    return R == 1 ? &launch_fixed<K, 1>
         : R == 2 ? &launch_fixed<K, 2>
         : R == 3 ? &launch_fixed<K, 3>
                  : &launch_fixed<K, 4>;
}

fixed_fn pick_fixed(int K, int R) {
    switch (K) {
#define RSGPU_K(k) case k: return pick_r<k>(R);
        RSGPU_K(1) RSGPU_K(2) RSGPU_K(3) RSGPU_K(4) RSGPU_K(5) RSGPU_K(6) RSGPU_K(7) RSGPU_K(8)
        RSGPU_K(9) RSGPU_K(10) RSGPU_K(11) RSGPU_K(12) RSGPU_K(13) RSGPU_K(14) RSGPU_K(15)
        RSGPU_K(16)
#undef RSGPU_K
        default: return nullptr;
    }
}

}  // namespace

namespace {

// The batch's last object may read past the caller's buffer: a row's last
// 16-B vector reaches past the row, and nothing guarantees readable bytes
// after the batch (Layout::slack).  The caller's buffer spans every row's
// full pitch.  Object-major ([object][shard]): the last row of the last
// object ends at its pitch.  Shard-major ([shard][object], pitch >=
// (nobj-1)*obj_stride + S): the last object's piece of the last shard row
// ends where that row's pitch ends.
bool overhangs(const Layout &L) {
    if (L.slack || L.in_base || L.out_base) return false;
    const size_t vec_end = (L.shard_len + 15) / 16 * 16;
    const bool shard_major = L.nobj > 1 && L.pitch >= (size_t)(L.nobj - 1) * L.obj_stride + L.shard_len;
    return (shard_major ? (size_t)(L.nobj - 1) * L.obj_stride : 0) + vec_end > L.pitch;
}

hipError_t launch_plan_core(Plan &p, const Layout &L, uint32_t *d_bad, hipStream_t st);

// The batch's last object of an overhanging layout, coded in a stream-ordered
// scratch copy with slack: its rows copied in at a 16-B pitch (2D copy), the
// pass run there, the written rows' shard_len bytes copied back.
hipError_t launch_last_object(Plan &p, const Layout &L, uint32_t *d_bad, hipStream_t st) {
    uint8_t *obj = L.base + (size_t)(L.nobj - 1) * L.obj_stride;
    const size_t P = (L.shard_len + 15) / 16 * 16, rows = rows_extent(p, 1);
    uint8_t *tmp = nullptr;
    hipError_t e = hipMallocAsync((void **)&tmp, rows * P + 64, st);
    if (e != hipSuccess) return e;
    e = hipMemcpy2DAsync(tmp, P, obj, L.pitch, L.shard_len, rows, hipMemcpyDeviceToDevice, st);
    Layout one{tmp, 0, P, L.shard_len, 1};
    one.slack = true;
    if (e == hipSuccess) e = launch_plan_core(p, one, d_bad ? d_bad + (L.nobj - 1) : nullptr, st);
    for (int r = 0; r < p.nw && e == hipSuccess; ++r)
        e = hipMemcpyAsync(obj + (size_t)p.out_rows[r] * L.pitch, tmp + (size_t)p.out_rows[r] * P, L.shard_len,
                           hipMemcpyDeviceToDevice, st);
    const hipError_t f = hipFreeAsync(tmp, st);
    return e != hipSuccess ? e : f;
}

// Objects whose rows span 4 GiB or more (the 32-bit offsets of a pass's
// buffer resource cannot reach them): every operation is a byte-column map,
// so each object is coded in column slabs — the slab's rows gathered into a
// stream-ordered scratch image (one 2D copy, 16-B pitch, <= 1 GiB), the pass
// run there, the written rows' slab bytes copied back.  Check flags: the
// caller's memset precedes (check plans OR into d_bad[o]); plans without
// checks clear d_bad[o] in every slab alike.  Device-to-device copies move
// each slab twice, so these objects code at a fraction of the pass's rate.
hipError_t launch_huge(Plan &p, const Layout &L, uint32_t *d_bad, hipStream_t st) {
    const size_t nrows = rows_extent(p, 1);
    const size_t lim = (size_t)1 << 30;
    const size_t slab = std::max<size_t>(4096, (lim / nrows) & ~(size_t)4095);
    uint8_t *tmp = nullptr;
    hipError_t e = hipMallocAsync((void **)&tmp, nrows * slab + 64, st);
    if (e != hipSuccess) return e;
    for (int o = 0; o < L.nobj && e == hipSuccess; ++o) {
        uint8_t *obj = L.base + (size_t)o * L.obj_stride;
        for (size_t b0 = 0; b0 < L.shard_len && e == hipSuccess; b0 += slab) {
            const size_t len = std::min(slab, L.shard_len - b0), P = (len + 15) / 16 * 16;
            e = hipMemcpy2DAsync(tmp, P, obj + b0, L.pitch, len, nrows, hipMemcpyDeviceToDevice, st);
            Layout one{tmp, 0, P, len, 1};
            one.slack = true;
            if (e == hipSuccess) e = launch_plan_core(p, one, d_bad ? d_bad + o : nullptr, st);
            for (int r = 0; r < p.nw && e == hipSuccess; ++r)
                e = hipMemcpyAsync(obj + (size_t)p.out_rows[r] * L.pitch + b0, tmp + (size_t)p.out_rows[r] * P, len,
                                   hipMemcpyDeviceToDevice, st);
        }
    }
    const hipError_t f = hipFreeAsync(tmp, st);
    return e != hipSuccess ? e : f;
}

}  // namespace

void set_tri_mode(int mode) { g_tri_mode.store(mode, std::memory_order_relaxed); }

hipError_t launch_plan(Plan &p, const Layout &L, uint32_t *d_bad, hipStream_t st) {
    if (L.nobj <= 0 || p.R <= 0) return hipSuccess;
    if (!L.in_base && !L.out_base && L.sub_stride == 0 && rows_extent(p, L.pitch) + 16 >= ((size_t)1 << 32))
        return launch_huge(p, L, d_bad, st);
    // Shard-major batch ([shard][object]: shard i of object o at
    // base + i*pitch + o*obj_stride, the objects' pieces of one shard back to
    // back): coding is byte-position-wise, so the batch IS one object whose
    // shard is the whole row, streamed at the large-object rate however small
    // the objects are.  Gaps between pieces are pad bytes, coded along (and
    // overwritten in written rows): taken while a gap is at most
    // roundup16(S) - S or a quarter of S (1 KiB objects at a 128-B stride,
    // whole-line pieces); wider gaps go object by object.  Check flags stay
    // per object (Pass::sub_*); the generic kernel (K > 16) has no per-object
    // attribution, so it converts only without flags.
    const size_t row = (size_t)(L.nobj - 1) * L.obj_stride + L.shard_len;
    const bool narrow_gaps = L.obj_stride <= (L.shard_len + 15) / 16 * 16 || (L.obj_stride - L.shard_len) * 4 <= L.shard_len;
    if (L.nobj > 1 && !L.in_base && !L.out_base && L.sub_stride == 0 && L.obj_stride >= L.shard_len &&
        narrow_gaps && (row + 15) / 16 * 16 <= L.pitch &&
        (p.K <= kMaxK || !d_bad) && (size_t)L.nobj * L.obj_stride < ((size_t)1 << 32)) {
        Layout big{L.base, 0, L.pitch, row, 1};
        big.slack = L.slack;
        big.sub_stride = (uint32_t)L.obj_stride;
        big.sub_len = (uint32_t)L.shard_len;
        big.sub_n = (uint32_t)L.nobj;
        return launch_plan(p, big, d_bad, st);
    }
    if (overhangs(L)) {
        // every object's over-read lands in the next object, except the last one's
        Layout head = L;
        head.nobj = L.nobj - 1;
        head.slack = true;
        hipError_t e = launch_plan_core(p, head, d_bad, st);
        return e != hipSuccess ? e : launch_last_object(p, L, d_bad, st);
    }
    return launch_plan_core(p, L, d_bad, st);
}

namespace {

hipError_t launch_plan_core(Plan &p, const Layout &L, uint32_t *d_bad, hipStream_t st) {
    if (L.nobj <= 0 || p.R <= 0) return hipSuccess;
    static_assert(kRedirectMaxK == kMaxK, "redirect limit");
    if ((L.out_base || L.in_base) && (p.K > kMaxK || L.nobj != 1))
        return hipErrorInvalidValue;  // only the specialised single-object passes redirect
    if (p.K <= kMaxK) {
        // split R into passes of <= 4 rows; written rows first, then checks
        for (int r0 = 0; r0 < p.R; r0 += kMaxR) {
            Sub s{r0, std::min(kMaxR, p.R - r0), 0};
            s.nw = std::max(0, std::min(s.R, p.nw - r0));
            hipError_t e = pick_fixed(p.K, s.R)(p, s, L, d_bad, st);
            if (e != hipSuccess) return e;
        }
        return hipSuccess;
    }
    // K > 16: generic kernel, one pass per <= 8 rows over one table image
    for (int r0 = 0; r0 < p.R; r0 += kMaxRG) {
        Sub s{r0, std::min(kMaxRG, p.R - r0), 0};
        s.nw = std::max(0, std::min(s.R, p.nw - r0));
        hipError_t e;
        switch (s.R) {
            case 1: e = launch_generic<1>(p, s, L, d_bad, st); break;
            case 2: e = launch_generic<2>(p, s, L, d_bad, st); break;
            case 3: e = launch_generic<3>(p, s, L, d_bad, st); break;
            case 4: e = launch_generic<4>(p, s, L, d_bad, st); break;
            case 5: e = launch_generic<5>(p, s, L, d_bad, st); break;
            case 6: e = launch_generic<6>(p, s, L, d_bad, st); break;
            case 7: e = launch_generic<7>(p, s, L, d_bad, st); break;
            default: e = launch_generic<8>(p, s, L, d_bad, st); break;
        }
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace

MultiWorkspace::~MultiWorkspace() {
    for (auto &u : uploaded)
        if (u) (void)hipEventDestroy(u);
    if (upload) (void)hipStreamDestroy(upload);
    for (auto &s : slot) {
        if (s.done) (void)hipEventDestroy(s.done);
        retire(s.d, false, s.cap);
        retire(s.h, true, s.cap);
    }
}

hipError_t launch_plans_multi_core(const std::vector<Plan *> &plans, const std::vector<int> &plan_of,
                                   const Layout &L, uint32_t *d_bad, hipStream_t st, MultiWorkspace &ws);
hipError_t stage_image(MultiWorkspace &ws, const std::vector<uint8_t> &img, MultiWorkspace::Slot *&out);

hipError_t launch_plans_multi(const std::vector<Plan *> &plans, const std::vector<int> &plan_of,
                              const Layout &L, uint32_t *d_bad, hipStream_t st, MultiWorkspace &ws) {
    if (L.nobj > 0 && overhangs(L)) {  // the last object through launch_plan's scratch copy
        Layout head = L;
        head.nobj = L.nobj - 1;
        head.slack = true;
        std::vector<int> po(plan_of.begin(), plan_of.begin() + head.nobj);
        hipError_t e = launch_plans_multi_core(plans, po, head, d_bad, st, ws);
        const int last = plan_of[L.nobj - 1];
        if (e != hipSuccess || last < 0) return e;
        Layout one{L.base + (size_t)(L.nobj - 1) * L.obj_stride, L.obj_stride, L.pitch, L.shard_len, 1};
        return launch_plan(*plans[last], one, d_bad ? d_bad + (L.nobj - 1) : nullptr, st);
    }
    return launch_plans_multi_core(plans, plan_of, L, d_bad, st, ws);
}

hipError_t launch_plans_multi_core(const std::vector<Plan *> &plans, const std::vector<int> &plan_of,
                                   const Layout &L, uint32_t *d_bad, hipStream_t st, MultiWorkspace &ws) {
    // entries grouped into (K, R) classes; K > 16 plans run object by object
    std::vector<std::vector<Entry>> per_plan(plans.size());
    std::vector<std::vector<uint32_t>> objs_of(plans.size());
    // each plan's objects in ascending order (stage_class relies on it)
    for (size_t o = 0; o < plan_of.size(); ++o)
        if (plan_of[o] >= 0) objs_of[plan_of[o]].push_back((uint32_t)o);  // -1: skip object
    std::map<std::pair<int, int>, std::vector<const Entry *>> classes;
    std::vector<std::unique_ptr<Entry>> store;
    for (size_t i = 0; i < plans.size(); ++i) {
        Plan &p = *plans[i];
        if (objs_of[i].empty() || p.R <= 0) continue;
        if (p.K > kMaxK) {
            for (uint32_t o : objs_of[i]) {
                Layout one{L.base + (size_t)o * L.obj_stride, L.obj_stride, L.pitch, L.shard_len, 1};
                one.slack = L.slack || (int)o + 1 < L.nobj;  // the next object follows
                hipError_t e = launch_plan(p, one, d_bad ? d_bad + o : nullptr, st);
                if (e != hipSuccess) return e;
            }
            continue;
        }
        for (int r0 = 0; r0 < p.R; r0 += kMaxR) {
            Sub s{r0, std::min(kMaxR, p.R - r0), 0};
            s.nw = std::max(0, std::min(s.R, p.nw - r0));
            store.emplace_back(new Entry{&p, s, objs_of[i]});
            classes[{p.K, s.R}].push_back(store.back().get());
        }
    }
    if (classes.empty()) return hipSuccess;
    std::vector<uint8_t> img;
    std::vector<std::pair<size_t, std::function<hipError_t(const uint8_t *, hipStream_t)>>> launches;
    for (auto &kv : classes)
        launches.emplace_back(0, pick_stage(kv.first.first, kv.first.second)(kv.second, L, d_bad, img));
    std::lock_guard<std::mutex> g(ws.mu);
    MultiWorkspace::Slot *w = nullptr;
    hipError_t e = stage_image(ws, img, w);
    for (auto &l : launches)
        if (e == hipSuccess) e = l.second((const uint8_t *)w->d, st);
    if (e == hipSuccess) e = hipEventRecord(w->done, st);
    return e;
}

// The next ring slot of ws holding `img` in device memory (ws.mu held).
// The upload runs on its own stream and the HOST waits for it: the host is
// normally several calls ahead of the GPU (the slot ring throttles it), so
// the wait costs the GPU nothing.  Measured against a GPU-side
// hipStreamWaitEvent and against a copy in the caller's stream: 1 % and 3.5 %
// slower on the mixed bench (rocprof gaps).  The caller records
// w->done on its stream after the kernels that read the image.
hipError_t stage_image(MultiWorkspace &ws, const std::vector<uint8_t> &img, MultiWorkspace::Slot *&out) {
    MultiWorkspace::Slot &w = ws.slot[ws.next++ % MultiWorkspace::kRing];
    hipError_t e = hipSuccess;
    if (!ws.upload) {
        e = hipStreamCreateWithFlags(&ws.upload, hipStreamNonBlocking);
        if (e != hipSuccess) return e;
    }
    if (w.done) {  // the kernels that read this image kRing calls ago must be done
        e = hipEventSynchronize(w.done);
        if (e != hipSuccess) return e;
    } else {
        e = hipEventCreateWithFlags(&w.done, hipEventDisableTiming);
        if (e != hipSuccess) return e;
    }
    if (w.cap < img.size()) {
        retire(w.d, false, w.cap);  // (held while a worker kernel is resident: devmem.cpp)
        retire(w.h, true, w.cap);
        w.d = nullptr;
        w.h = nullptr;
        w.cap = 0;
        const size_t cap = std::max<size_t>(img.size() * 2, 1 << 16);
        e = hipMalloc(&w.d, cap);
        if (e == hipSuccess) e = hipHostMalloc(&w.h, cap, hipHostMallocDefault);
        if (e != hipSuccess) return e;
        w.cap = cap;
    }
    std::memcpy(w.h, img.data(), img.size());
    e = hipMemcpyAsync(w.d, w.h, img.size(), hipMemcpyHostToDevice, ws.upload);
    if (e == hipSuccess) e = hipStreamSynchronize(ws.upload);
    out = &w;
    return e;
}

// ---- variable-size batches (rsgpu_*_dev_objs): one launch per sub-pass over
// objects of any sizes and pitches, the object table uploaded once per call

namespace {

template <int K, int R>
hipError_t launch_var_t(const Plan &p, const Sub &s, const VarObj *d_objs, const uint32_t *d_chunk_obj,
                        uint32_t nobj, uint32_t total, uint32_t *d_bad, hipStream_t st) {
    VarArgs<K, R> a;
    a.objs = d_objs;
    a.chunk_obj = d_chunk_obj;
    a.nobj = nobj;
    a.bad = d_bad;
    // row indices, not offsets: pitch 1 (each object's pitch scales them in the kernel)
    fill_pass<K, R>(p, s, 1, 16, 1, d_bad != nullptr, a.p);
    unsigned grid;
    a.ord = make_order(1, total, (size_t)1 << 40, grid);
    hipLaunchKernelGGL((gf_apply_var<K, R, kBlock, kLoadAux, kStoreAux>), dim3(grid), dim3(kBlock),
                       pass_lds(K, (int)a.p.nw, R), st, a);
    return hipGetLastError();
}

typedef hipError_t (*var_fn)(const Plan &, const Sub &, const VarObj *, const uint32_t *, uint32_t, uint32_t,
                             uint32_t *, hipStream_t);
template <int K>
var_fn pick_var_r(int R) {
    return R == 1 ? &launch_var_t<K, 1> : R == 2 ? &launch_var_t<K, 2> : R == 3 ? &launch_var_t<K, 3>
                                                                            : &launch_var_t<K, 4>;
}
var_fn pick_var(int K, int R) {
    switch (K) {
#define RSGPU_K(k) case k: return pick_var_r<k>(R);
        RSGPU_K(1) RSGPU_K(2) RSGPU_K(3) RSGPU_K(4) RSGPU_K(5) RSGPU_K(6) RSGPU_K(7) RSGPU_K(8)
        RSGPU_K(9) RSGPU_K(10) RSGPU_K(11) RSGPU_K(12) RSGPU_K(13) RSGPU_K(14) RSGPU_K(15)
        RSGPU_K(16)
#undef RSGPU_K
        default: return nullptr;
    }
}

}  // namespace

hipError_t launch_plan_objs(Plan &p, const DevObj *objs, int nobj, uint32_t *d_bad, hipStream_t st,
                            MultiWorkspace &ws) {
    if (nobj <= 0 || p.R <= 0) return hipSuccess;
    if (p.K > kMaxK) {  // the generic kernel has no table form: object by object
        for (int o = 0; o < nobj; ++o) {
            Layout one{objs[o].base, 0, objs[o].pitch, objs[o].shard_len, 1};
            hipError_t e = launch_plan(p, one, d_bad ? d_bad + o : nullptr, st);
            if (e != hipSuccess) return e;
        }
        return hipSuccess;
    }
    int maxrow = 0;
    for (int r : p.in_rows) maxrow = std::max(maxrow, r);
    for (int r : p.out_rows) maxrow = std::max(maxrow, r);
    uint64_t total = 0;
    for (int o = 0; o < nobj; ++o) total += ((objs[o].shard_len + 15) / 16 + kBlock - 1) / kBlock;
    if (total >= 0x7ff00000ull) return hipErrorInvalidValue;  // > 2^31 workgroups: split the table
    // the image: the object table, then (up to 16 Mi chunks, a 64 MiB table)
    // each chunk's object index, so a workgroup finds its object with one
    // scalar load instead of a binary search (RSGPU_VAR_SEARCH=1: always search)
    static const bool force_search = std::getenv("RSGPU_VAR_SEARCH") != nullptr;
    const bool direct = !force_search && total <= ((uint64_t)1 << 24);
    const size_t tab_bytes = (size_t)nobj * sizeof(VarObj);
    std::vector<uint8_t> img(tab_bytes + (direct ? (size_t)total * 4 : 0));
    VarObj *t = (VarObj *)img.data();
    uint32_t *cobj = (uint32_t *)(img.data() + tab_bytes);
    uint64_t c = 0;
    for (int o = 0; o < nobj; ++o) {
        const DevObj &d = objs[o];
        VarObj &v = t[o];
        v.base = (uint64_t)d.base;
        v.nvec = (uint32_t)((d.shard_len + 15) / 16);
        v.tail = (uint32_t)(d.shard_len - (size_t)(v.nvec - 1) * 16);
        v.pitch = (uint32_t)d.pitch;
        v.span = (uint32_t)((size_t)maxrow * d.pitch + (size_t)v.nvec * 16);
        v.packed = tail_part(d.pitch, v.nvec);
        v.chunk0 = (uint32_t)c;
        const uint32_t nch = (v.nvec + kBlock - 1) / kBlock;
        if (direct)
            for (uint32_t j = 0; j < nch; ++j) cobj[c + j] = (uint32_t)o;
        c += nch;
    }
    std::lock_guard<std::mutex> g(ws.mu);
    MultiWorkspace::Slot *w = nullptr;
    hipError_t e = stage_image(ws, img, w);
    for (int r0 = 0; r0 < p.R && e == hipSuccess; r0 += kMaxR) {
        Sub s{r0, std::min(kMaxR, p.R - r0), 0};
        s.nw = std::max(0, std::min(s.R, p.nw - r0));
        const uint8_t *d = (const uint8_t *)w->d;
        e = pick_var(p.K, s.R)(p, s, (const VarObj *)d, direct ? (const uint32_t *)(d + tab_bytes) : nullptr,
                               (uint32_t)nobj, (uint32_t)total, d_bad, st);
    }
    if (e == hipSuccess) e = hipEventRecord(w->done, st);
    return e;
}

}  // namespace rsgpu
