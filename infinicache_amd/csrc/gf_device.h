// gf_device.h — device side of the GF(2^8) apply pass (gfx950).  Shared by
// the product (gf_kernels.hip) and the variant micro-benchmark
// (tools/kbench.hip); see gf_kernels.hip for the design notes.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <type_traits>

namespace rsgpu {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// GF(2^8) multiply-by-constant c as three byte lookups on the bit groups
// [2:0], [5:3] and [7:6] of every byte: v_perm_b32 selects any of 8 bytes
// from its two source dwords, so one perm is a 3-bit table lookup.  A
// coefficient's table is kTabWords dwords:
//   t[0], t[1]: c*j, j = 0..7 (bytes 0-3, 4-7)   group [2:0]
//   t[2], t[3]: c*(j<<3), j = 0..7               group [5:3]
//   t[4]:       c*(j<<6), j = 0..3               group [7:6]
// 5 VALU ops per (coefficient, dword) plus 5 per input dword for the indices,
// vs 6 + 7 with four 2-bit groups (tools/kbench.hip).
constexpr int kTabWords = 5;

struct GfIdx {
    uint32_t i0, i1, i2;
};
__device__ __forceinline__ GfIdx gf_idx(uint32_t w) {
    return {w & 0x07070707u, (w >> 3) & 0x07070707u, (w >> 6) & 0x03030303u};
}

// v_perm_b32 byte select: 0-3 pick bytes of the second operand, 4-7 of the first
__device__ __forceinline__ uint32_t lut8(uint32_t lo, uint32_t hi, uint32_t sel) {
    return __builtin_amdgcn_perm(hi, lo, sel);
}

// acc ^= c (x) w, for one dword w with group indices g
template <typename T>  // T: uint32_t in any address space (kernarg / constant image)
__device__ __forceinline__ uint32_t gf_mac(uint32_t acc, T *t, const GfIdx &g) {
    acc = xor3(acc, lut8(t[0], t[1], g.i0), lut8(t[2], t[3], g.i1));
    return acc ^ lut8(t[4], t[4], g.i2);
}

// Store one 16-B output vector.  `part` (0..15) is non-zero only for the last
// vector of a row whose pitch is not a multiple of 16 and leaves fewer than
// 16 bytes to the next row (the host API's byte-packed staging image, pitch =
// S; device batches with pitch = S rounded to 4): only the row's first `part`
// bytes of that vector may be written, as one 8/4/2/1-byte store each.
// Rows need no 16-B alignment: gfx950 buffer loads/stores honour unaligned
// offsets (the driver's SH_MEM_CONFIG unaligned mode; tools/unaligned_probe.hip).
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
template <int SAUX>
__device__ __forceinline__ void store_row(const u32x4 &o, __amdgpu_buffer_rsrc_t rs, uint32_t voff,
                                          uint32_t soff, uint32_t part) {
    if (part == 0u) {
        __builtin_amdgcn_raw_buffer_store_b128(o, rs, voff, soff, SAUX);
        return;
    }
    // select dwords with compares, never by indexing the vector with a
    // runtime value (that puts `o` in private memory: a scratch frame per lane)
    uint32_t off = 0;
    if (part & 8u) {
        const u32x2 lo = {o[0], o[1]};
        __builtin_amdgcn_raw_buffer_store_b64(lo, rs, voff, soff, SAUX);
        off = 8;
    }
    if (part & 4u) {
        __builtin_amdgcn_raw_buffer_store_b32(off ? o[2] : o[0], rs, voff + off, soff, SAUX);
        off += 4;
    }
    uint32_t rem = off == 12 ? o[3] : off == 8 ? o[2] : off == 4 ? o[1] : o[0];
    if (part & 2u) {
        __builtin_amdgcn_raw_buffer_store_b16((unsigned short)rem, rs, voff + off, soff, SAUX);
        off += 2;
        rem >>= 16;
    }
    if (part & 1u) __builtin_amdgcn_raw_buffer_store_b8((unsigned char)rem, rs, voff + off, soff, SAUX);
}

// mask of the valid bytes of dword d in a 16-B vector holding `valid` bytes
__device__ __forceinline__ uint32_t tail_mask(int d, uint32_t valid) {
    int v = (int)valid - 4 * d;
    if (v >= 4) return 0xffffffffu;
    if (v <= 0) return 0u;
    return (1u << (8 * v)) - 1u;
}

// Everything of one pass that depends on the operation / erasure pattern.
template <int K, int R>
struct Pass {
    uint32_t nw;     // rows [0, nw) stored, [nw, R) compared to zero
    uint32_t ki;     // trailing identity inputs (see gf_apply_body)
    uint32_t clear;  // the plan has no check rows: this pass zeroes bad[obj]
    uint32_t span;   // bytes addressable from an object base
    uint32_t packed; // bytes of a row's last vector that may be written when < 16, else 0 (store_row)
    // shard-major batch coded as one object (launch_plan): the row holds
    // sub_n objects' shards of sub_len bytes every sub_stride bytes; check
    // flags and clears are per object, attributed by byte position
    uint32_t sub_stride, sub_len, sub_n;
    uint32_t in_off[K];
    uint32_t out_off[R];
    uint32_t tab[K * R * kTabWords];  // input-major [K][R][kTabWords]: scalar loads per input
};

// A pass whose GF inputs go in triples (gf_apply_body<..., TRI = true>): the
// 24 index bits of inputs a, b, c are eight 3-bit groups, bits [2:0] and
// [5:3] of each input plus {a[7:6], b[7]} and {b[6], c[7:6]}; each group is
// one v_perm lookup into an 8-entry table of its row (the two cross groups'
// tables mix two coefficients, as the generic kernel's, gf_kernels.hip).
// Per row and dword 8 v_perm + 4 xor3 for three inputs instead of 9 + 6.
template <int K, int R>
struct Pass3 : Pass<K, R> {
    uint32_t ntrip;  // inputs [0, 3 * ntrip) go in triples, the rest one at a time
    uint32_t tab3[(K / 3 > 0 ? K / 3 : 1) * R * 16];  // [t][r]: words 0-7 entries 0-3, 8-15 entries 4-7
};

// Workgroup -> (item, chunk) order of a 1D launch over `total` = nitem x
// nchunk workgroups.  The hardware deals workgroup ids round-robin to the 8
// XCDs (id % 8), and each XCD translates through its own TLB.
//   xper == 0: linear order (an item's chunks on consecutive ids);
//   xper  > 0: XCD x walks the contiguous items [x*xper, (x+1)*xper), so each
//              XCD's TLB sees 1/8 of the launch's pages.
// The host uses xper > 0 (on cold batches the XCD-contiguous
// order runs 2-4 points of HBM peak above the linear one).
struct Order {
    uint32_t nchunk, total, xper;
};
__device__ __forceinline__ bool wg_item(const Order &o, uint32_t &item, uint32_t &chunk) {
    const uint32_t b = blockIdx.x;
    const uint32_t w = o.xper ? (b & 7u) * o.xper + (b >> 3) : b;
    if (w >= o.total) return false;
    item = w / o.nchunk;
    chunk = w - item * o.nchunk;
    return true;
}

template <int K, int R, typename PT = Pass<K, R>>
struct ApplyArgs {  // one pass for every object of the launch (kernarg)
    const uint8_t *base;
    // per-object host API (one object, rsgpu.cpp run_host): the rows may be
    // read from / written to a caller's pinned host buffer over PCIe
    const uint8_t *in_base;   // input rows read here (same offsets); nullptr: base
    const uint8_t *out_base;  // written rows go here (same offsets); nullptr: base
    uint32_t in_span;         // bytes readable from in_base (clips the tail vector)
    uint32_t copy_in;         // with in_base: copy the input rows into base too
    uint32_t out_dual;        // with out_base: store the written rows to base too
    uint64_t obj_stride;
    uint32_t *bad;
    uint32_t nvec;   // 16-B vectors per row
    uint32_t tail;   // valid bytes in the last vector (1..16)
    uint32_t opw;    // objects per workgroup (> 1: small objects, item = group of opw)
    uint32_t nobj;   // objects in the launch (bounds the last group when opw > 1)
    uint32_t gspan;  // opw > 1: bytes a group's objects cover from the first one's base
    Order ord;       // item = object, or group of opw objects
    PT p;
};

template <int K, int R>
struct MultiArgs {  // per-object passes (a Get batch with mixed erasure patterns)
    const uint8_t *base;
    uint64_t obj_stride;
    uint32_t *bad;
    uint32_t nvec, tail;
    Order ord;                 // item i codes object objs[i] ...
    const Pass<K, R> *passes;  // device array, one per distinct pattern
    const uint32_t *objs;
    const uint32_t *obj_pass;  // ... with passes[obj_pass[i]]
    // opw > 1 (small objects): item i is a group of opw objects sharing one
    // pass, objs[i*opw + j] (~0u: empty slot), passes[obj_pass[i]]; lanes
    // address object o at o * obj_stride from base, within gspan bytes
    uint32_t opw, gspan;
};

// One workgroup = BS lanes x U vectors of 16 B of one object (grid.y).
// Lane t handles vectors blockIdx.x*BS*U + t + u*BS, so every wave-wide
// load/store is 1 KiB contiguous.  LAUX/SAUX are the buffer-op cache-policy
// bits (gfx950: 1 = sc0, 2 = nt, 16 = sc1).
// Trailing identity inputs: the last `ki` inputs (runtime, <= R) each enter
// exactly one row with coefficient 1 — input K-ki+j feeds row R-ki+j — and no
// other row.  That is Verify's parity columns (check row = M[j] x data XOR
// parity_j) and the fused decode's extra shards; the host detects it
// (Plan::ki).  Those inputs cost one XOR instead of four v_perm + two XOR per
// row, and one uniform branch per input (no per-coefficient branches).
// P: Pass<K, R> (kernarg) or its constant-address-space alias (device image)
// Zero-copy redirection of one object's rows (the per-object host API,
// rsgpu.cpp run_host): inputs read from / outputs written to a caller's
// pinned host buffer over PCIe, at the image's own row offsets.
struct Redirect {
    const uint8_t *in = nullptr;   // input rows read here; nullptr: the object base
    uint32_t in_span = 0;          // bytes readable from `in` (the tail vector's over-read is clipped)
    bool copy_in = false;          // also copy the input rows into the object base (image)
    const uint8_t *out = nullptr;  // written rows go here; nullptr: the object base
    bool dual = false;             // also store the written rows to the object base
};

// Small objects (ApplyArgs::opw > 1): a workgroup codes several whole
// objects, lane -> (object, vector); `ob` is then the first object's base
// (uniform), `lane_off` the lane's object offset from it and `span` the bytes
// the group's objects cover.
// Variable-size batches (VAR = true, gf_apply_var): the pass's in_off /
// out_off hold row INDICES, scaled by the object's own pitch `vp`; `span` is
// the object's own span and `vpacked` its store_row part.
template <int K, int R, int U, int BS, int LAUX, int SAUX, typename P, bool VAR = false, bool TRI = false>
__device__ __forceinline__ void gf_apply_body(const uint8_t *ob, uint32_t obj, P &a,
                                              uint32_t nvec, uint32_t tail, uint32_t *bad,
                                              uint32_t v0, const Redirect &rd = Redirect(),
                                              uint32_t lane_off = 0, uint32_t span = 0,
                                              uint32_t vp = 0, uint32_t vpacked = 0) {
    if (v0 >= nvec) return;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void *)ob, (short)0, (int)(span ? span : a.span), 0x00020000);
    const __amdgpu_buffer_rsrc_t rsi =
        rd.in ? __builtin_amdgcn_make_buffer_rsrc((void *)rd.in, (short)0, (int)rd.in_span, 0x00020000) : rs;
    const __amdgpu_buffer_rsrc_t rso =
        rd.out ? __builtin_amdgcn_make_buffer_rsrc((void *)rd.out, (short)0, (int)a.span, 0x00020000) : rs;

    auto in_off = [&](int c) -> uint32_t { return VAR ? a.in_off[c] * vp : a.in_off[c]; };
    auto out_off = [&](int r) -> uint32_t { return VAR ? a.out_off[r] * vp : a.out_off[r]; };
    const uint32_t packed = VAR ? vpacked : a.packed;
    u32x4 x[U][K];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint32_t v = v0 + u * BS;
        if (U == 1 || v < nvec) {
#pragma unroll
            for (int c = 0; c < K; ++c)
                x[u][c] = __builtin_amdgcn_raw_buffer_load_b128(rsi, lane_off + v * 16u, in_off(c), LAUX);
            if (rd.copy_in) {
#pragma unroll
                for (int c = 0; c < K; ++c)
                    store_row<SAUX>(x[u][c], rs, lane_off + v * 16u, in_off(c), v == nvec - 1 ? packed : 0u);
            }
        }
    }

    bool mismatch = false;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint32_t v = v0 + u * BS;
        if (U > 1 && v >= nvec) break;
        uint32_t acc[R][4];
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int d = 0; d < 4; ++d) acc[r][d] = 0;
        uint32_t ntr = 0;
        if constexpr (TRI) {  // GF inputs in triples (Pass3)
            ntr = a.ntrip;
#pragma unroll
            for (int tt = 0; tt < K / 3; ++tt) {
                if ((uint32_t)tt < ntr) {
                    uint32_t sel[4][8];
#pragma unroll
                    for (int d = 0; d < 4; ++d) {
                        const uint32_t xa = x[u][3 * tt][d], xb = x[u][3 * tt + 1][d], xc = x[u][3 * tt + 2][d];
                        sel[d][0] = xa & 0x07070707u;
                        sel[d][1] = (xa >> 3) & 0x07070707u;
                        sel[d][2] = xb & 0x07070707u;
                        sel[d][3] = (xb >> 3) & 0x07070707u;
                        sel[d][4] = xc & 0x07070707u;
                        sel[d][5] = (xc >> 3) & 0x07070707u;
                        sel[d][6] = ((xa >> 5) & 0x06060606u) | ((xb >> 7) & 0x01010101u);
                        sel[d][7] = ((xb >> 6) & 0x01010101u) | ((xc >> 5) & 0x06060606u);
                    }
#pragma unroll
                    for (int r = 0; r < R; ++r) {
                        const auto *T = &a.tab3[(tt * R + r) * 16];
#pragma unroll
                        for (int d = 0; d < 4; ++d) {
                            uint32_t q = xor3(acc[r][d], lut8(T[0], T[8], sel[d][0]), lut8(T[1], T[9], sel[d][1]));
                            q = xor3(q, lut8(T[2], T[10], sel[d][2]), lut8(T[3], T[11], sel[d][3]));
                            q = xor3(q, lut8(T[4], T[12], sel[d][4]), lut8(T[5], T[13], sel[d][5]));
                            acc[r][d] = xor3(q, lut8(T[6], T[14], sel[d][6]), lut8(T[7], T[15], sel[d][7]));
                        }
                    }
                }
#pragma unroll
                for (int r = 0; r < R; ++r)
#pragma unroll
                    for (int d = 0; d < 4; ++d) asm volatile("" : "+v"(acc[r][d]));
                __builtin_amdgcn_sched_barrier(0);
            }
        }
#pragma unroll
        for (int c = 0; c < K; ++c) {
            if (TRI && (uint32_t)c < 3 * ntr) continue;  // coded in its triple
            if (c >= K - R && c >= K - (int)a.ki) {
                // identity input: row R-K+c (compile-time index) ^= input
#pragma unroll
                for (int d = 0; d < 4; ++d) acc[(R - K + c) < 0 ? 0 : (R - K + c)][d] ^= x[u][c][d];
            } else {
#pragma unroll
                for (int d = 0; d < 4; ++d) {
                    const GfIdx g = gf_idx(x[u][c][d]);
#pragma unroll
                    for (int r = 0; r < R; ++r)
                        acc[r][d] = gf_mac(acc[r][d], &a.tab[(c * R + r) * kTabWords], g);
                }
            }
            // keep the input-at-a-time order: without these fences the IR
            // passes and the scheduler hoist every input's index math and
            // split the work row by row (160+ VGPRs, 2 waves/SIMD)
#pragma unroll
            for (int r = 0; r < R; ++r)
#pragma unroll
                for (int d = 0; d < 4; ++d) asm volatile("" : "+v"(acc[r][d]));
            __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int r = 0; r < R; ++r) {
            if ((uint32_t)r < a.nw) {
                u32x4 o = {acc[r][0], acc[r][1], acc[r][2], acc[r][3]};
                store_row<SAUX>(o, rso, lane_off + v * 16u, out_off(r), v == nvec - 1 ? packed : 0u);
                if (rd.dual) store_row<SAUX>(o, rs, lane_off + v * 16u, out_off(r), v == nvec - 1 ? packed : 0u);
            } else {
                const uint32_t valid = (v == nvec - 1) ? tail : 16u;
#pragma unroll
                for (int d = 0; d < 4; ++d) {
                    uint32_t m = acc[r][d] & tail_mask(d, valid);
                    if (a.sub_stride) {  // shard-major: flag the object each nonzero byte belongs to
                        while (m) {
                            const uint32_t b = (uint32_t)__builtin_ctz(m) >> 3, x = v * 16u + d * 4u + b;
                            const uint32_t o = x / a.sub_stride;
                            if (x - o * a.sub_stride < a.sub_len) bad[o] = 1u;  // gap bytes are pads
                            m &= ~(0xffu << (8 * b));
                        }
                    } else {
                        mismatch |= m != 0;
                    }
                }
            }
        }
    }
    // every writer stores the same 1 (no atomic needed, and the flag may
    // live in mapped host memory); zeroing happens before the launch
    if (mismatch) bad[obj] = 1u;
    // the plan has no check rows: the pass itself clears the object's flag
    // (saves the caller's memset launch on the decode hot path); shard-major:
    // the flags of the objects whose first byte is in this lane's vector
    if (a.clear) {
        if (a.sub_stride) {
            const uint32_t x0 = v0 * 16u;
            for (uint32_t o = (x0 + a.sub_stride - 1) / a.sub_stride; o < a.sub_n && o * a.sub_stride < x0 + 16u; ++o)
                bad[o] = 0u;
        } else if (v0 == 0) {
            bad[obj] = 0u;
        }
    }
}

// FORM: which launch shapes one instantiation serves.  Each form is its own
// kernel so that its register allocation is its own: with every form in one
// kernel the 100 table words no longer fit the SGPR file beside the other
// forms' uniforms, and the compiler parks them in VGPR lanes (80 v_writelane
// per wave, plus 92 v_readlane per wave in the small-object form).
constexpr int kFormAny = 0;       // runtime: small objects if a.opw > 1, else chunks (+ redirection)
constexpr int kFormChunks = 1;    // one object per workgroup chunk, no redirection
constexpr int kFormSmall = 2;     // a.opw > 1 objects per workgroup
constexpr int kFormRedirect = 3;  // one object, zero-copy redirection (per-object host API)
template <int K, int R, int U, int BS, int LAUX, int SAUX, int FORM = kFormAny, bool TRI = false>
__global__ __launch_bounds__(BS) void gf_apply_kernel(
    const ApplyArgs<K, R, std::conditional_t<TRI, Pass3<K, R>, Pass<K, R>>> a) {
    uint32_t obj, chunk;
    if (!wg_item(a.ord, obj, chunk)) return;
    if (FORM == kFormSmall || (FORM == kFormAny && a.opw > 1)) {  // small objects: lane -> (object j of the group, vector v)
        const uint32_t j = threadIdx.x / a.nvec, o0 = obj * a.opw;
        if (j >= a.opw || o0 + j >= a.nobj) return;
        gf_apply_body<K, R, U, BS, LAUX, SAUX, const decltype(a.p), false, TRI>(
            a.base + (uint64_t)o0 * a.obj_stride, o0 + j, a.p, a.nvec, a.tail, a.bad, threadIdx.x - j * a.nvec,
            Redirect(), j * (uint32_t)a.obj_stride, a.gspan);
        return;
    }
    Redirect rd;
    if (FORM == kFormAny || FORM == kFormRedirect) {
        rd.in = a.in_base;
        rd.in_span = a.in_span;
        rd.copy_in = a.copy_in != 0;
        rd.out = a.out_base;
        rd.dual = a.out_dual != 0;
    }
    gf_apply_body<K, R, U, BS, LAUX, SAUX, const decltype(a.p), false, TRI>(a.base + (uint64_t)obj * a.obj_stride, obj, a.p,
                                                                       a.nvec, a.tail, a.bad,
                                                                       chunk * (BS * U) + threadIdx.x, rd);
}

// Short rows (<= kStagedMaxVec vectors: objects of about 1 KiB), opw objects
// per workgroup, staged through LDS.  Lane (object, vector) loads straight
// from HBM (gf_apply_kernel's small form) make every wave load a gather of
// ~9 row pieces of 112 B; here the workgroup
//   1. loads its objects' input rows with lanes walking (object, input,
//      vector) in address order, so each wave load is ~1 KiB of consecutive
//      rows (as on large objects), into LDS;
//   2. codes lane (object, vector) from LDS, written rows back into LDS;
//   3. stores the written rows the same address-ordered way.
// LDS: opw * (K + R) * nvec * 16 B (<= 64 KiB).  Rows must hold whole
// vectors (no packed tail) and the batch must not be shard-major.
constexpr uint32_t kStagedMaxVec = 8;
__device__ __forceinline__ uint32_t udiv_small(uint32_t x, uint32_t d, float rcp) {
    uint32_t q = (uint32_t)((float)x * rcp);  // x < 2^16: off by at most one
    if (q * d > x) --q;
    else if ((q + 1) * d <= x) ++q;
    return q;
}

template <int K, int R, int LAUX, int SAUX>
__global__ __launch_bounds__(256) void gf_apply_staged(const ApplyArgs<K, R> a) {
    extern __shared__ u32x4 lds[];  // [opw][K][nvec] inputs, then [opw][R][nvec] written rows
    uint32_t grp, chunk;
    if (!wg_item(a.ord, grp, chunk)) return;
    const uint32_t t = threadIdx.x, nvec = a.nvec, o0 = grp * a.opw;
    const uint32_t nob = min(a.opw, a.nobj - o0);
    const uint32_t stride = (uint32_t)a.obj_stride;  // the group spans < 4 GiB (host)
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(a.base + (uint64_t)o0 * a.obj_stride), (short)0, (int)a.gspan, 0x00020000);
    const float rn = 1.0f / (float)nvec, rkn = 1.0f / (float)(K * nvec);
    u32x4 *in = lds, *out = lds + a.opw * K * nvec;

    // 1. inputs in address order; every load of a lane issued before its LDS stores
    const uint32_t nin = nob * K * nvec;
    u32x4 x[K];
#pragma unroll
    for (int i = 0; i < K; ++i) {
        const uint32_t e = t + i * 256u;
        if (e < nin) {
            const uint32_t j = udiv_small(e, K * nvec, rkn), rem = e - j * K * nvec;
            const uint32_t c = udiv_small(rem, nvec, rn), v = rem - c * nvec;
            // row offsets of the pass: select with compares (a runtime index
            // into the kernarg array would go through scratch)
            uint32_t off = a.p.in_off[0];
#pragma unroll
            for (int q = 1; q < K; ++q) off = c == (uint32_t)q ? a.p.in_off[q] : off;
            x[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, j * stride + off + v * 16u, 0, LAUX);
        }
    }
#pragma unroll
    for (int i = 0; i < K; ++i)
        if (t + i * 256u < nin) in[t + i * 256u] = x[i];
    __syncthreads();

    // 2. lane (object j, vector v) codes from LDS
    const uint32_t j = udiv_small(t, nvec, rn), v = t - j * nvec;
    if (j < nob) {
        uint32_t acc[R][4];
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int d = 0; d < 4; ++d) acc[r][d] = 0;
#pragma unroll
        for (int c = 0; c < K; ++c) {
            const u32x4 y = in[(j * K + c) * nvec + v];
            if (c >= K - R && c >= K - (int)a.p.ki) {
#pragma unroll
                for (int d = 0; d < 4; ++d) acc[(R - K + c) < 0 ? 0 : (R - K + c)][d] ^= y[d];
            } else {
#pragma unroll
                for (int d = 0; d < 4; ++d) {
                    const GfIdx g = gf_idx(y[d]);
#pragma unroll
                    for (int r = 0; r < R; ++r) acc[r][d] = gf_mac(acc[r][d], &a.p.tab[(c * R + r) * kTabWords], g);
                }
            }
        }
        bool mismatch = false;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            if ((uint32_t)r < a.p.nw) {
                out[(j * R + r) * nvec + v] = u32x4{acc[r][0], acc[r][1], acc[r][2], acc[r][3]};
            } else {
                const uint32_t valid = (v == nvec - 1) ? a.tail : 16u;
#pragma unroll
                for (int d = 0; d < 4; ++d) mismatch |= (acc[r][d] & tail_mask(d, valid)) != 0;
            }
        }
        if (mismatch) a.bad[o0 + j] = 1u;
        if (a.p.clear && v == 0) a.bad[o0 + j] = 0u;
    }
    if (a.p.nw == 0) return;  // uniform: no barrier skipped by part of the group
    __syncthreads();

    // 3. written rows in address order
    const uint32_t nwv = a.p.nw * nvec, nout = nob * nwv;
    const float rnw = 1.0f / (float)nwv;
    for (uint32_t e = t; e < nout; e += 256u) {
        const uint32_t jj = udiv_small(e, nwv, rnw), rem = e - jj * nwv;
        const uint32_t r = udiv_small(rem, nvec, rn), vv = rem - r * nvec;
        uint32_t off = a.p.out_off[0];
#pragma unroll
        for (int q = 1; q < R; ++q) off = r == (uint32_t)q ? a.p.out_off[q] : off;
        __builtin_amdgcn_raw_buffer_store_b128(out[(jj * R + r) * nvec + vv], rs, jj * stride + off + vv * 16u, 0,
                                               SAUX);
    }
}

// constant address space: uniform invariant data the compiler may (and does)
// fetch with scalar loads
template <typename T>
using constant_ptr = const __attribute__((address_space(4))) T *;

// One object of a variable-size batch (rsgpu_*_dev_objs): a device table
// entry, read by scalar loads.  chunk0 = the object's first workgroup in the
// launch's flattened (object, chunk) space; the entries are in chunk0 order.
struct VarObj {
    uint64_t base;
    uint32_t nvec, tail, pitch, span, packed, chunk0;
};
static_assert(sizeof(VarObj) == 32, "VarObj: one 32-B table entry");

template <int K, int R>
struct VarArgs {  // one pass over objects of different sizes and pitches (kernarg)
    const VarObj *objs;
    const uint32_t *chunk_obj;  // [total]: the object of each flattened chunk, or nullptr
    uint32_t nobj;
    uint32_t *bad;   // per object (index into objs), or nullptr
    Order ord;       // item = flattened chunk (nchunk = 1)
    Pass<K, R> p;    // in_off / out_off: row indices (scaled by each object's pitch)
};

// Workgroup w codes chunk w - chunk0 of the object whose chunk range holds w:
// one scalar load from the host's chunk -> object table, or (tables too large
// to build) a binary search over the entries' chunk0, whose dependent scalar
// loads a workgroup waits out before its first data load.
template <int K, int R, int BS, int LAUX, int SAUX>
__global__ __launch_bounds__(BS) void gf_apply_var(const VarArgs<K, R> a) {
    uint32_t w, unused;
    if (!wg_item(a.ord, w, unused)) return;
    const constant_ptr<VarObj> objs = (constant_ptr<VarObj>)a.objs;
    uint32_t lo = 0;
    if (a.chunk_obj) {
        lo = ((constant_ptr<uint32_t>)a.chunk_obj)[w];
    } else {
        uint32_t hi = a.nobj;  // objs[lo].chunk0 <= w < objs[hi].chunk0
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (objs[mid].chunk0 <= w) lo = mid;
            else hi = mid;
        }
    }
    const uint64_t base = objs[lo].base;
    const uint32_t nvec = objs[lo].nvec, tail = objs[lo].tail, pitch = objs[lo].pitch;
    const uint32_t span = objs[lo].span, packed = objs[lo].packed, c0 = objs[lo].chunk0;
    gf_apply_body<K, R, 1, BS, LAUX, SAUX, const Pass<K, R>, true>(
        (const uint8_t *)base, lo, a.p, nvec, tail, a.bad, (w - c0) * BS + threadIdx.x, Redirect(), 0u, span,
        pitch, packed);
}

// Mixed erasure patterns in one launch: each workgroup reads its object's
// pass index (uniform) and then the pass itself through scalar loads.  CH > 1
// walks several chunks of the object per workgroup with the pass kept in
// SGPRs; the product uses CH = 1 (the lookups cost nothing measurable,
// tools/kbench KB_SET=multi, and longer walks were slower).

template <int K, int R, int U, int BS, int LAUX, int SAUX, int CH>
__global__ __launch_bounds__(BS) void gf_apply_multi(const MultiArgs<K, R> m) {
    // constant address space: the compiler may (and does) fetch the object
    // index, pass index and the pass itself with s_load (invariant, uniform)
    uint32_t item, chunk;
    if (!wg_item(m.ord, item, chunk)) return;
    if (m.opw > 1) {  // small objects: lane -> (object j of the group, vector v)
        const __attribute__((address_space(4))) Pass<K, R> &p =
            ((constant_ptr<Pass<K, R>>)m.passes)[((constant_ptr<uint32_t>)m.obj_pass)[item]];
        const uint32_t j = threadIdx.x / m.nvec;
        if (j >= m.opw) return;
        const uint32_t obj = m.objs[item * m.opw + j];
        if (obj == 0xffffffffu) return;
        gf_apply_body<K, R, U, BS, LAUX, SAUX>(m.base, obj, p, m.nvec, m.tail, m.bad, threadIdx.x - j * m.nvec,
                                               Redirect(), obj * (uint32_t)m.obj_stride, m.gspan);
        return;
    }
    const uint32_t obj = ((constant_ptr<uint32_t>)m.objs)[item];
    const uint32_t pi = ((constant_ptr<uint32_t>)m.obj_pass)[item];
    const __attribute__((address_space(4))) Pass<K, R> &p = ((constant_ptr<Pass<K, R>>)m.passes)[pi];
    const uint8_t *ob = m.base + (uint64_t)obj * m.obj_stride;
    for (int ch = 0; ch < CH; ++ch)
        gf_apply_body<K, R, U, BS, LAUX, SAUX>(ob, obj, p, m.nvec, m.tail, m.bad,
                                               (chunk * CH + ch) * (BS * U) + threadIdx.x);
}

}  // namespace rsgpu
