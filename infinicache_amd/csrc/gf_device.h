// gf_device.h — device side of the GF(2^8) apply pass (gfx950).  Shared by
// the product (gf_kernels.hip) and the variant micro-benchmark
// (tools/kbench.hip); see gf_kernels.hip for the design notes.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace rsgpu {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
__device__ __forceinline__ uint32_t lut(uint32_t t, uint32_t sel) {
    return __builtin_amdgcn_perm(t, t, sel);
}

// acc ^= c (x) w, for one dword w whose 2-bit group indices are i0..i3.
template <typename T>  // T: uint32_t in any address space (kernarg / constant image)
__device__ __forceinline__ uint32_t gf_mac(uint32_t acc, T *t, uint32_t i0, uint32_t i1,
                                           uint32_t i2, uint32_t i3) {
    acc = xor3(acc, lut(t[0], i0), lut(t[1], i1));
    return xor3(acc, lut(t[2], i2), lut(t[3], i3));
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
    uint32_t in_off[K];
    uint32_t out_off[R];
    uint32_t tab[K * R * 4];  // input-major [K][R][4]: one s_load_dwordx(4R) per input
};

template <int K, int R>
struct ApplyArgs {  // one pass for every object of the launch (kernarg)
    const uint8_t *base;
    uint64_t obj_stride;
    uint32_t *bad;
    uint32_t nvec;   // 16-B vectors per row
    uint32_t tail;   // valid bytes in the last vector (1..16)
    Pass<K, R> p;
};

template <int K, int R>
struct MultiArgs {  // per-object passes (a Get batch with mixed erasure patterns)
    const uint8_t *base;
    uint64_t obj_stride;
    uint32_t *bad;
    uint32_t nvec, tail;
    const Pass<K, R> *passes;  // device array, one per distinct pattern
    const uint32_t *objs;      // block y codes object objs[y] ...
    const uint32_t *obj_pass;  // ... with passes[obj_pass[y]]
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
template <int K, int R, int U, int BS, int LAUX, int SAUX, typename P>
__device__ __forceinline__ void gf_apply_body(const uint8_t *ob, uint32_t obj, P &a,
                                              uint32_t nvec, uint32_t tail, uint32_t *bad,
                                              uint32_t v0) {
    if (v0 >= nvec) return;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void *)ob, (short)0, (int)a.span, 0x00020000);

    u32x4 x[U][K];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint32_t v = v0 + u * BS;
        if (U == 1 || v < nvec) {
#pragma unroll
            for (int c = 0; c < K; ++c)
                x[u][c] = __builtin_amdgcn_raw_buffer_load_b128(rs, v * 16u, a.in_off[c], LAUX);
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
#pragma unroll
        for (int c = 0; c < K; ++c) {
            if (c >= K - R && c >= K - (int)a.ki) {
                // identity input: row R-K+c (compile-time index) ^= input
#pragma unroll
                for (int d = 0; d < 4; ++d) acc[(R - K + c) < 0 ? 0 : (R - K + c)][d] ^= x[u][c][d];
            } else {
#pragma unroll
                for (int d = 0; d < 4; ++d) {
                    const uint32_t w = x[u][c][d];
                    const uint32_t i0 = w & 0x03030303u;
                    const uint32_t i1 = (w >> 2) & 0x03030303u;
                    const uint32_t i2 = (w >> 4) & 0x03030303u;
                    const uint32_t i3 = (w >> 6) & 0x03030303u;
#pragma unroll
                    for (int r = 0; r < R; ++r)
                        acc[r][d] = gf_mac(acc[r][d], &a.tab[(c * R + r) * 4], i0, i1, i2, i3);
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
                __builtin_amdgcn_raw_buffer_store_b128(o, rs, v * 16u, a.out_off[r], SAUX);
            } else {
                const uint32_t valid = (v == nvec - 1) ? tail : 16u;
#pragma unroll
                for (int d = 0; d < 4; ++d) mismatch |= (acc[r][d] & tail_mask(d, valid)) != 0;
            }
        }
    }
    if (mismatch) atomicOr(bad + obj, 1u);
    // the plan has no check rows: the pass itself clears the object's flag
    // (saves the caller's memset launch on the decode hot path)
    if (a.clear && v0 == 0) bad[obj] = 0u;
}

template <int K, int R, int U, int BS, int LAUX, int SAUX>
__global__ __launch_bounds__(BS) void gf_apply_kernel(const ApplyArgs<K, R> a) {
    gf_apply_body<K, R, U, BS, LAUX, SAUX>(a.base + (uint64_t)blockIdx.y * a.obj_stride, blockIdx.y,
                                           a.p, a.nvec, a.tail, a.bad,
                                           blockIdx.x * (BS * U) + threadIdx.x);
}

// Mixed erasure patterns in one launch: each workgroup reads its object's
// pass index (uniform) and then the pass itself through scalar loads — two
// dependent loads before its first data load, so a workgroup walks CH chunks
// of its object with the pass kept in SGPRs to amortise them.
template <typename T>
using constant_ptr = const __attribute__((address_space(4))) T *;

template <int K, int R, int U, int BS, int LAUX, int SAUX, int CH>
__global__ __launch_bounds__(BS) void gf_apply_multi(const MultiArgs<K, R> m) {
    // constant address space: the compiler may (and does) fetch the object
    // index, pass index and the pass itself with s_load (invariant, uniform)
    const uint32_t obj = ((constant_ptr<uint32_t>)m.objs)[blockIdx.y];
    const uint32_t pi = ((constant_ptr<uint32_t>)m.obj_pass)[blockIdx.y];
    const __attribute__((address_space(4))) Pass<K, R> &p = ((constant_ptr<Pass<K, R>>)m.passes)[pi];
    const uint8_t *ob = m.base + (uint64_t)obj * m.obj_stride;
    for (int ch = 0; ch < CH; ++ch)
        gf_apply_body<K, R, U, BS, LAUX, SAUX>(ob, obj, p, m.nvec, m.tail, m.bad,
                                               (blockIdx.x * CH + ch) * (BS * U) + threadIdx.x);
}

}  // namespace rsgpu
