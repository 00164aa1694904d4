// kbench.hip — interleaved A/B timing of gf_apply_kernel launch variants on
// real codec plans (built by the library itself, so check-row plans run on
// consistent data), layout [obj][row][pitch] in HBM.
//
//   make -C tools kbench          (links ../infinicache_amd/librsgpu.so)
//   ./tools/kbench SHAPE [rounds]
//   SHAPE: enc10_2 | enc10_4 | dec10_2 | rdata10_4 | decx10_4 | ver10_2 | ver10_4
//          optionally @M: M-MiB objects (e.g. enc10_2@4), xN: N objects (enc10_2x2048@1)
//
// Every variant's output rows are checked bit-exact against the library's own
// launch (which the product tests pin to the oracle); check-row plans must
// report no mismatch.  An xor-only kernel with the same streams gives the
// memory-pattern ceiling.  Timing: one HIP-event pair per launch, variants
// interleaved round-robin in one process (methodology rule 24).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "ctx.h"
#include "gf_device.h"

using namespace rsgpu;

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(1);                                                                          \
        }                                                                                          \
    } while (0)

__global__ void fill(uint8_t *p, size_t n, uint64_t seed) {
    size_t i = (blockIdx.x * (size_t)blockDim.x + threadIdx.x);
    for (; i * 8 < n; i += (size_t)gridDim.x * blockDim.x) {
        uint64_t z = seed + i * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        *(uint64_t *)(p + i * 8) = z;
    }
}

// memory-pattern ceiling: same loads/stores as the plan, XOR instead of GF math
template <int K, int R>
__global__ __launch_bounds__(256) void xor_only(const ApplyArgs<K, R> a) {
    const uint32_t v = blockIdx.x * 256 + threadIdx.x;
    if (v >= a.nvec) return;
    const uint8_t *ob = a.base + (uint64_t)blockIdx.y * a.obj_stride;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void *)ob, (short)0, (int)a.p.span, 0x00020000);
    u32x4 x[K];
#pragma unroll
    for (int c = 0; c < K; ++c) x[c] = __builtin_amdgcn_raw_buffer_load_b128(rs, v * 16u, a.p.in_off[c], 2);
    u32x4 acc = x[0];
#pragma unroll
    for (int c = 1; c < K; ++c) acc ^= x[c];
    for (uint32_t r = 0; r < a.p.nw; ++r)
        __builtin_amdgcn_raw_buffer_store_b128(acc, rs, v * 16u, a.p.out_off[r], 16);
    if (a.p.nw == 0 && acc[0] == 0x12345678u && acc[1] == 0x9abcdef0u) a.bad[0] = 1;  // keep live
}

// Ablation: the north star's "LDS-staged log/exp tables" formulation.  The
// 256-entry log table and the 510-entry exp table of GF(2^8)/0x11D are staged
// in LDS once per workgroup; each byte of each input is multiplied by each
// coefficient as exp[log[x] + log[c]] (x == 0 -> 0), i.e. one LDS byte
// lookup for log[x] per input byte (shared by all rows) and one for exp per
// (byte, row), then the bytes are re-packed into dwords.  Same loads/stores
// and launch shape as the shipped kernel.
__constant__ uint8_t c_logexp[256 + 512];
template <int K, int R>
__global__ __launch_bounds__(256) void lds_logexp(const ApplyArgs<K, R> a, const uint8_t *logc) {
    __shared__ uint8_t s_log[256];
    __shared__ uint8_t s_exp[512];
    for (int i = threadIdx.x; i < 256; i += 256) s_log[i] = c_logexp[i];
    for (int i = threadIdx.x; i < 512; i += 256) s_exp[i] = c_logexp[256 + i];
    __syncthreads();
    const uint32_t v = blockIdx.x * 256 + threadIdx.x;
    if (v >= a.nvec) return;
    const uint8_t *ob = a.base + (uint64_t)blockIdx.y * a.obj_stride;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void *)ob, (short)0, (int)a.p.span, 0x00020000);
    uint32_t acc[R][4] = {};
    for (int c = 0; c < K; ++c) {
        const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(rs, v * 16u, a.p.in_off[c], 2);
#pragma unroll
        for (int d = 0; d < 4; ++d) {
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const uint32_t byte = (x[d] >> (8 * b)) & 0xffu;
                const uint32_t lx = s_log[byte];
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const uint32_t lc = logc[c * R + r];  // 255 encodes coefficient 0
                    const uint32_t prod = (byte == 0 || lc == 255u) ? 0u : s_exp[lx + lc];
                    acc[r][d] ^= prod << (8 * b);
                }
            }
        }
    }
    bool mismatch = false;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        if ((uint32_t)r < a.p.nw) {
            u32x4 o = {acc[r][0], acc[r][1], acc[r][2], acc[r][3]};
            __builtin_amdgcn_raw_buffer_store_b128(o, rs, v * 16u, a.p.out_off[r], 16);
        } else {
            const uint32_t valid = (v == a.nvec - 1) ? a.tail : 16u;
#pragma unroll
            for (int d = 0; d < 4; ++d) mismatch |= (acc[r][d] & tail_mask(d, valid)) != 0;
        }
    }
    if (mismatch) atomicOr(a.bad + blockIdx.y, 1u);
    if (a.p.clear && v == 0) a.bad[blockIdx.y] = 0u;
}
static const uint8_t *g_logc = nullptr;
template <int K, int R>
void launch_lds(const void *args, dim3 grid, hipStream_t st) {
    hipLaunchKernelGGL((lds_logexp<K, R>), grid, dim3(256), 0, st, *(const ApplyArgs<K, R> *)args, g_logc);
}

// grid-order ablation: blockIdx.x = object, blockIdx.y = chunk (resident
// workgroups spread over many objects instead of walking one object)
template <int K, int R>
__global__ __launch_bounds__(256) void apply_objmajor(const ApplyArgs<K, R> a) {
    gf_apply_body<K, R, 1, 256, 2, 2>(a.base + (uint64_t)blockIdx.x * a.obj_stride, blockIdx.x, a.p,
                                       a.nvec, a.tail, a.bad, blockIdx.y * 256 + threadIdx.x);
}
template <int K, int R>
void launch_om(const void *args, dim3 grid, hipStream_t st) {
    hipLaunchKernelGGL((apply_objmajor<K, R>), dim3(grid.y, grid.x), dim3(256), 0, st,
                       *(const ApplyArgs<K, R> *)args);
}
typedef void (*launch_fn)(const void *, dim3, hipStream_t);
// 1D order for a (chunks, objects) grid: ORD 0 = the library's policy
// (XCD-contiguous for every launch of >= 8 workgroups), 1 = linear,
// 2 = XCD-contiguous.  (Profiles before the cold-batch retune used ORD 0 =
// XCD-contiguous only past 1.5 GiB of objects.)
template <int ORD>
Order order_for(dim3 grid, size_t span, unsigned &nb) {
    (void)span;
    Order o{grid.x, grid.x * grid.y, 0};
    const bool xcd = ORD == 2 || (ORD == 0 && o.total >= 8);
    if (xcd) o.xper = (o.total + 7) / 8;
    nb = o.xper ? o.xper * 8 : o.total;
    return o;
}
template <int K, int R, int U, int BS, int LA, int SA, bool NOKI = false, int ORD = 0>
void launch_v(const void *args, dim3 grid, hipStream_t st) {
    ApplyArgs<K, R> a = *(const ApplyArgs<K, R> *)args;
    if (NOKI) a.p.ki = 0;  // every input through the dense GF path
    unsigned nb;
    a.ord = order_for<ORD>(grid, (size_t)grid.y * a.obj_stride, nb);
    hipLaunchKernelGGL((gf_apply_kernel<K, R, U, BS, LA, SA, kFormChunks>), dim3(nb), dim3(BS), 0, st, a);
}
// the library's launch exactly: the chunk-form instantiation (kFormChunks,
// as launch_fixed runs it), nt loads/stores, XCD-contiguous order, and the
// LDS occupancy cap of gf_kernels.hip pass_lds (store_lds(K) workgroups per
// CU on passes that store rows; 4 on passes that store and check rows with
// K > 10).  Before round 4 this launched the kFormAny instantiation, whose
// extra forms cost registers: 1-1.5 % on RS(10+2), 11 points on the RS(10+4)
// decode with checks (profiles/r04_kbench_store_order.txt).
template <int K, int R>
void launch_ship(const void *args, dim3 grid, hipStream_t st) {
    ApplyArgs<K, R> a = *(const ApplyArgs<K, R> *)args;
    unsigned nb;
    a.ord = order_for<0>(grid, 0, nb);
    int w = K <= 5 ? 8 : (40 / K < 2 ? 2 : 40 / K);  // gf_kernels.hip store_lds
    if (a.p.nw < (uint32_t)R && K > 10) w = 4;
    hipLaunchKernelGGL((gf_apply_kernel<K, R, 1, 256, 2, 2, kFormChunks>), dim3(nb), dim3(256),
                       a.p.nw ? 160u * 1024u / (unsigned)w - 256u : 0u, st, a);
}
template <int K, int R>
void launch_x(const void *args, dim3 grid, hipStream_t st) {
    hipLaunchKernelGGL((xor_only<K, R>), grid, dim3(256), 0, st, *(const ApplyArgs<K, R> *)args);
}

// multi-pass variant: the same plan fetched per workgroup from device memory
static const void *g_multi_args = nullptr;
// the uniform kernel with its pass read from a device image through a
// constant-address-space pointer (scalar loads) instead of the kernarg
template <int K, int R>
__global__ __launch_bounds__(256) void apply_cpass(const MultiArgs<K, R> m) {
    uint32_t obj, chunk;
    if (!wg_item(m.ord, obj, chunk)) return;
    const __attribute__((address_space(4))) Pass<K, R> &p = *((constant_ptr<Pass<K, R>>)m.passes);
    gf_apply_body<K, R, 1, 256, 2, 2>(m.base + (uint64_t)obj * m.obj_stride, obj, p, m.nvec, m.tail,
                                       m.bad, chunk * 256 + threadIdx.x);
}
template <int K, int R>
void launch_cp(const void *, dim3 grid, hipStream_t st) {
    MultiArgs<K, R> m = *(const MultiArgs<K, R> *)g_multi_args;
    unsigned nb;
    m.ord = order_for<0>(grid, (size_t)grid.y * m.obj_stride, nb);
    hipLaunchKernelGGL((apply_cpass<K, R>), dim3(nb), dim3(256), 0, st, m);
}

template <int K, int R, int CH>
void launch_m(const void *, dim3 grid, hipStream_t st) {
    grid.x = (grid.x + CH - 1) / CH;
    MultiArgs<K, R> m = *(const MultiArgs<K, R> *)g_multi_args;
    unsigned nb;
    m.ord = order_for<0>(grid, (size_t)grid.y * m.obj_stride, nb);
    hipLaunchKernelGGL((gf_apply_multi<K, R, 1, 256, 2, 2, CH>), dim3(nb), dim3(256), 0, st, m);
}

// the mixed-pattern kernel under an occupancy cap of W workgroups per CU
// (W = 0: the library's store_lds(K) cap)
template <int K, int R, int W>
void launch_mc(const void *, dim3 grid, hipStream_t st) {
    MultiArgs<K, R> m = *(const MultiArgs<K, R> *)g_multi_args;
    unsigned nb;
    m.ord = order_for<0>(grid, (size_t)grid.y * m.obj_stride, nb);
    const int w = W ? W : (K <= 5 ? 8 : (40 / K < 2 ? 2 : 40 / K));
    hipLaunchKernelGGL((gf_apply_multi<K, R, 1, 256, 2, 2, 1>), dim3(nb), dim3(256),
                       160u * 1024u / (unsigned)w - 256u, st, m);
}
// the same with the pass read through the kernarg-fetched pointer but the
// object / pass index of the item computed, not loaded (isolates the first
// scalar load of the chain)
template <int K, int R, int W>
__global__ __launch_bounds__(256) void apply_cpass_cap(const MultiArgs<K, R> m) {
    uint32_t obj, chunk;
    if (!wg_item(m.ord, obj, chunk)) return;
    const __attribute__((address_space(4))) Pass<K, R> &p = *((constant_ptr<Pass<K, R>>)m.passes);
    gf_apply_body<K, R, 1, 256, 2, 2>(m.base + (uint64_t)obj * m.obj_stride, obj, p, m.nvec, m.tail,
                                       m.bad, chunk * 256 + threadIdx.x);
}
template <int K, int R, int W>
void launch_cpc(const void *, dim3 grid, hipStream_t st) {
    MultiArgs<K, R> m = *(const MultiArgs<K, R> *)g_multi_args;
    unsigned nb;
    m.ord = order_for<0>(grid, (size_t)grid.y * m.obj_stride, nb);
    const int w = W ? W : (K <= 5 ? 8 : (40 / K < 2 ? 2 : 40 / K));
    hipLaunchKernelGGL((apply_cpass_cap<K, R, W>), dim3(nb), dim3(256), 160u * 1024u / (unsigned)w - 256u,
                       st, m);
}

// one workgroup walks CH consecutive chunks of its object (longer
// sequential runs per DRAM page for each of the K+R row streams)
template <int K, int R, int CH>
__global__ __launch_bounds__(256) void apply_walk(const ApplyArgs<K, R> a) {
    uint32_t obj, chunk;
    if (!wg_item(a.ord, obj, chunk)) return;
    const uint8_t *ob = a.base + (uint64_t)obj * a.obj_stride;
    for (int ch = 0; ch < CH; ++ch)
        gf_apply_body<K, R, 1, 256, 2, 2>(ob, obj, a.p, a.nvec, a.tail, a.bad,
                                          (chunk * CH + ch) * 256 + threadIdx.x);
}
template <int K, int R, int CH>
void launch_w(const void *args, dim3 grid, hipStream_t st) {
    grid.x = (grid.x + CH - 1) / CH;
    ApplyArgs<K, R> a = *(const ApplyArgs<K, R> *)args;
    unsigned nb;
    a.ord = order_for<0>(grid, (size_t)grid.y * a.obj_stride, nb);
    hipLaunchKernelGGL((apply_walk<K, R, CH>), dim3(nb), dim3(256), 0, st, a);
}

struct Variant {
    std::string name;
    launch_fn fn;
    int U, BS;
    bool ceiling;
    int rd = -1, wr = -1;  // rows read / written per object (-1: the plan's K / nw)
};

// stream probes for KB_SET=stream: the plan's K input rows read and nothing
// written, or W rows written (rows 0..W-1 of the object) and nothing read
template <int K, int R>
__global__ __launch_bounds__(256) void stream_read(const ApplyArgs<K, R> a) {
    uint32_t obj, chunk;
    if (!wg_item(a.ord, obj, chunk)) return;
    const uint32_t v = chunk * 256 + threadIdx.x;
    if (v >= a.nvec) return;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(a.base + (uint64_t)obj * a.obj_stride), (short)0, (int)a.p.span, 0x00020000);
    u32x4 acc = {0, 0, 0, 0};
#pragma unroll
    for (int c = 0; c < K; ++c) acc ^= __builtin_amdgcn_raw_buffer_load_b128(rs, v * 16u, a.p.in_off[c], 2);
    if (acc[0] == 0x12345678u && acc[1] == 0x9abcdef0u && acc[2] == 7u) a.bad[0] = 1;  // keep live
}
template <int K, int R, int W>
__global__ __launch_bounds__(256) void stream_write(const ApplyArgs<K, R> a, uint32_t pitch) {
    uint32_t obj, chunk;
    if (!wg_item(a.ord, obj, chunk)) return;
    const uint32_t v = chunk * 256 + threadIdx.x;
    if (v >= a.nvec) return;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(a.base + (uint64_t)obj * a.obj_stride), (short)0, (int)a.p.span, 0x00020000);
    const u32x4 o = {v, obj, v ^ obj, 0x5a5a5a5au};
#pragma unroll
    for (int r = 0; r < W; ++r) __builtin_amdgcn_raw_buffer_store_b128(o, rs, v * 16u, r * pitch, 2);
}
static uint32_t g_pitch = 0;
// the library's own launch_plan on the same buffers (sanity: must equal "shipped")
static Plan *g_plan = nullptr;
static size_t g_S = 0;
template <int K, int R>
void launch_lib(const void *args, dim3 grid, hipStream_t st) {
    const ApplyArgs<K, R> &a = *(const ApplyArgs<K, R> *)args;
    (void)launch_plan(*g_plan, Layout{(uint8_t *)a.base, a.obj_stride, g_pitch, g_S, (int)grid.y}, a.bad, st);
}
template <int K, int R>
void launch_sr(const void *args, dim3 grid, hipStream_t st) {
    ApplyArgs<K, R> a = *(const ApplyArgs<K, R> *)args;
    unsigned nb;
    a.ord = order_for<0>(grid, 0, nb);
    hipLaunchKernelGGL((stream_read<K, R>), dim3(nb), dim3(256), 0, st, a);
}
template <int K, int R, int W>
void launch_sw(const void *args, dim3 grid, hipStream_t st) {
    ApplyArgs<K, R> a = *(const ApplyArgs<K, R> *)args;
    unsigned nb;
    a.ord = order_for<0>(grid, 0, nb);
    hipLaunchKernelGGL((stream_write<K, R, W>), dim3(nb), dim3(256), 0, st, a, g_pitch);
}

// memory-pattern ceiling with a chosen store policy
template <int K, int R, int SA>
__global__ __launch_bounds__(256) void xor_only_sa(const ApplyArgs<K, R> a) {
    const uint32_t v = blockIdx.x * 256 + threadIdx.x;
    if (v >= a.nvec) return;
    const uint8_t *ob = a.base + (uint64_t)blockIdx.y * a.obj_stride;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void *)ob, (short)0, (int)a.p.span, 0x00020000);
    u32x4 x[K];
#pragma unroll
    for (int c = 0; c < K; ++c) x[c] = __builtin_amdgcn_raw_buffer_load_b128(rs, v * 16u, a.p.in_off[c], 2);
    u32x4 acc = x[0];
#pragma unroll
    for (int c = 1; c < K; ++c) acc ^= x[c];
    for (uint32_t r = 0; r < a.p.nw; ++r)
        __builtin_amdgcn_raw_buffer_store_b128(acc, rs, v * 16u, a.p.out_off[r], SA);
    if (a.p.nw == 0 && acc[0] == 0x12345678u && acc[1] == 0x9abcdef0u) a.bad[0] = 1;  // keep live
}
template <int K, int R, int SA>
void launch_xs(const void *args, dim3 grid, hipStream_t st) {
    hipLaunchKernelGGL((xor_only_sa<K, R, SA>), grid, dim3(256), 0, st, *(const ApplyArgs<K, R> *)args);
}

// M sub-streams per XCD: workgroup b runs on XCD x = b % 8; its t-th turn
// (t = b / 8) goes to region x + 8 * (t % M) at position t / M, so the launch
// is swept as 8*M contiguous regions at once (M = 1: XCD-contiguous order)
template <int K, int R, int M, int BS, int LA, int SA>
__global__ __launch_bounds__(BS) void apply_regions(const ApplyArgs<K, R> a, uint32_t per) {
    const uint32_t b = blockIdx.x, x = b & 7u, t = b >> 3;
    const uint32_t w = (x + 8u * (t % M)) * per + t / M;
    if (w >= a.ord.total) return;
    const uint32_t obj = w / a.ord.nchunk, chunk = w - obj * a.ord.nchunk;
    gf_apply_body<K, R, 1, BS, LA, SA>(a.base + (uint64_t)obj * a.obj_stride, obj, a.p, a.nvec, a.tail,
                                       a.bad, chunk * BS + threadIdx.x);
}
template <int K, int R, int M, int BS = 256>
void launch_rg(const void *args, dim3 grid, hipStream_t st) {
    ApplyArgs<K, R> a = *(const ApplyArgs<K, R> *)args;
    a.ord.nchunk = grid.x;
    a.ord.total = grid.x * grid.y;
    const uint32_t per = (a.ord.total + 8 * M - 1) / (8 * M);
    hipLaunchKernelGGL((apply_regions<K, R, M, BS, 2, 2>), dim3(per * 8 * M), dim3(BS), 0, st, a, per);
}

// occupancy cap: a dynamic LDS reservation of 160 KiB / W per workgroup
// leaves room for at most W workgroups (4 waves each) per CU
template <int K, int R, int W, int U = 1, int BS = 256>
void launch_occ(const void *args, dim3 grid, hipStream_t st) {
    ApplyArgs<K, R> a = *(const ApplyArgs<K, R> *)args;
    unsigned nb;
    a.ord = order_for<0>(grid, 0, nb);
    hipLaunchKernelGGL((gf_apply_kernel<K, R, U, BS, 2, 2, kFormChunks>), dim3(nb), dim3(BS), (160 * 1024) / W - 256, st, a);
}

// persistent form: W workgroups per CU (256 CUs), each walking the items of
// its XCD's contiguous share with stride = workgroups per XCD
template <int K, int R>
__global__ __launch_bounds__(256) void apply_persist(const ApplyArgs<K, R> a, uint32_t per_xcd) {
    const uint32_t b = blockIdx.x, x = b & 7u, t = b >> 3, T = gridDim.x >> 3;
    const uint32_t xper = (a.ord.total + 7) / 8;
    (void)per_xcd;
    for (uint32_t i = t; i < xper; i += T) {
        const uint32_t w = x * xper + i;
        if (w >= a.ord.total) break;
        const uint32_t obj = w / a.ord.nchunk, chunk = w - obj * a.ord.nchunk;
        gf_apply_body<K, R, 1, 256, 2, 2>(a.base + (uint64_t)obj * a.obj_stride, obj, a.p, a.nvec, a.tail,
                                          a.bad, chunk * 256 + threadIdx.x);
    }
}
template <int K, int R, int W>
void launch_pers(const void *args, dim3 grid, hipStream_t st) {
    ApplyArgs<K, R> a = *(const ApplyArgs<K, R> *)args;
    a.ord.nchunk = grid.x;
    a.ord.total = grid.x * grid.y;
    hipLaunchKernelGGL((apply_persist<K, R>), dim3(256 * W), dim3(256), 0, st, a, 0u);
}

// KB_SET=rows: the same pass on another row assignment (timing only): inputs
// on rows 0..K-1 and outputs on K..K+R-1 (encode's layout), or inputs on
// {1-4, 6-11} and outputs on {0, 5} (the healthy-Get decode's layout)
template <int K, int R, int LAYOUT>
void launch_rows(const void *args, dim3 grid, hipStream_t st) {
    ApplyArgs<K, R> a = *(const ApplyArgs<K, R> *)args;
    if (LAYOUT == 0) {
        for (int c = 0; c < K; ++c) a.p.in_off[c] = c * g_pitch;
        for (int r = 0; r < R; ++r) a.p.out_off[r] = (K + r) * g_pitch;
    } else {
        static const int in[12] = {1, 2, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13};
        static const int out[4] = {0, 5, 12, 13};
        for (int c = 0; c < K; ++c) a.p.in_off[c] = in[c] * g_pitch;
        for (int r = 0; r < R; ++r) a.p.out_off[r] = out[r] * g_pitch;
    }
    unsigned nb;
    a.ord = order_for<0>(grid, 0, nb);
    hipLaunchKernelGGL((gf_apply_kernel<K, R, 1, 256, 2, 2, kFormChunks>), dim3(nb), dim3(256),
                       a.p.nw ? 160u * 1024u / 4u - 256u : 0u, st, a);
}
template <int K, int R>
std::vector<Variant> rows_variants() {
    return {
        {"shipped", launch_ship<K, R>, 1, 256, false},
        {"encode's row layout", launch_rows<K, R, 0>, 1, 256, true},
        {"decode's row layout", launch_rows<K, R, 1>, 1, 256, true},
    };
}

// KB_SET=small: the LDS-staged small-object kernel is the library's
// gf_apply_staged (gf_device.h; shipped for rows of <= 8 vectors since round
// 3), timed here at every row length against the register form.

// KB_SET=small: the packed small-object launch (opw objects per workgroup,
// gf_kernels.hip launch_fixed) under other load/store policies and caps.
// W: workgroups per CU (0: the library's store_lds(K) cap, -1: no cap)
template <int K, int R, int LAUX, int SAUX, int W>
void launch_small(const void *args, dim3 grid, hipStream_t st) {
    ApplyArgs<K, R> a = *(const ApplyArgs<K, R> *)args;
    const uint32_t nobj = grid.y, opw = std::max(1u, 256u / a.nvec);
    a.opw = opw;
    a.nobj = nobj;
    a.gspan = (uint32_t)((uint64_t)(opw - 1) * a.obj_stride + a.p.span);
    unsigned nb;
    a.ord = order_for<0>(dim3(1, (nobj + opw - 1) / opw), 0, nb);
    const int w = W > 0 ? W : (K <= 5 ? 8 : (40 / K < 2 ? 2 : 40 / K));
    hipLaunchKernelGGL((gf_apply_kernel<K, R, 1, 256, LAUX, SAUX, kFormChunks>), dim3(nb), dim3(256),
                       W < 0 ? 0u : 160u * 1024u / (unsigned)w - 256u, st, a);
}
// the LDS-staged small-object kernel (gf_apply_staged); W > 0: at most W
// workgroups per CU through a larger LDS reservation
template <int K, int R, int LAUX, int SAUX, int W>
void launch_small_lds(const void *args, dim3 grid, hipStream_t st) {
    ApplyArgs<K, R> a = *(const ApplyArgs<K, R> *)args;
    const uint32_t nobj = grid.y, opw = std::max(1u, 256u / a.nvec);
    a.opw = opw;
    a.nobj = nobj;
    a.gspan = (uint32_t)((uint64_t)(opw - 1) * a.obj_stride + a.p.span);
    unsigned nb;
    a.ord = order_for<0>(dim3(1, (nobj + opw - 1) / opw), 0, nb);
    unsigned lds = opw * (K + R) * a.nvec * 16u;
    if (W > 0) lds = std::max(lds, 160u * 1024u / (unsigned)W - 256u);
    hipLaunchKernelGGL((gf_apply_staged<K, R, LAUX, SAUX>), dim3(nb), dim3(256), lds, st, a);
}
template <int K, int R>
std::vector<Variant> small_variants() {
    return {
        {"one object per workgroup", launch_ship<K, R>, 1, 256, false},
        {"library", launch_lib<K, R>, 1, 256, false},
        {"LDS-staged", launch_small_lds<K, R, 2, 2, 0>, 1, 256, false},
        {"LDS-staged default loads", launch_small_lds<K, R, 0, 2, 0>, 1, 256, false},
        {"LDS-staged default/default", launch_small_lds<K, R, 0, 0, 0>, 1, 256, false},
        {"LDS-staged cap 2", launch_small_lds<K, R, 2, 2, 2>, 1, 256, false},
        {"LDS-staged cap 4", launch_small_lds<K, R, 2, 2, 4>, 1, 256, false},
        {"registers (packed, no LDS)", launch_small<K, R, 2, 2, 0>, 1, 256, false},
        {"registers, default loads", launch_small<K, R, 0, 2, 0>, 1, 256, false},
        {"registers, full occupancy", launch_small<K, R, 2, 2, -1>, 1, 256, false},
    };
}

// KB_SET=burst: store bursts.  A workgroup codes CH consecutive 4 KiB chunks
// of one object, holding all outputs in VGPRs, then stores them: each output
// row gets CH*4 KiB in one burst per workgroup (the write stream arrives in
// larger runs).  Shapes with nw == R only (encode, decode without checks).
template <int K, int R, int CH>
__global__ __launch_bounds__(256) void apply_burst(const ApplyArgs<K, R> a) {
    uint32_t obj, chunk;
    if (!wg_item(a.ord, obj, chunk)) return;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(a.base + (uint64_t)obj * a.obj_stride), (short)0, (int)a.p.span, 0x00020000);
    u32x4 out[CH][R];
#pragma unroll
    for (int ch = 0; ch < CH; ++ch) {
        const uint32_t v = (chunk * CH + ch) * 256u + threadIdx.x;
        u32x4 x[K];
#pragma unroll
        for (int c = 0; c < K; ++c) x[c] = __builtin_amdgcn_raw_buffer_load_b128(rs, v * 16u, a.p.in_off[c], 2);
        uint32_t acc[R][4];
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int d = 0; d < 4; ++d) acc[r][d] = 0;
#pragma unroll
        for (int c = 0; c < K; ++c) {
#pragma unroll
            for (int d = 0; d < 4; ++d) {
                const GfIdx g = gf_idx(x[c][d]);
#pragma unroll
                for (int r = 0; r < R; ++r) acc[r][d] = gf_mac(acc[r][d], &a.p.tab[(c * R + r) * kTabWords], g);
            }
#pragma unroll
            for (int r = 0; r < R; ++r)
#pragma unroll
                for (int d = 0; d < 4; ++d) asm volatile("" : "+v"(acc[r][d]));
            __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int r = 0; r < R; ++r) out[ch][r] = u32x4{acc[r][0], acc[r][1], acc[r][2], acc[r][3]};
    }
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int ch = 0; ch < CH; ++ch) {
            const uint32_t v = (chunk * CH + ch) * 256u + threadIdx.x;
            if (v < a.nvec) __builtin_amdgcn_raw_buffer_store_b128(out[ch][r], rs, v * 16u, a.p.out_off[r], 2);
        }
    if (a.p.clear && chunk == 0 && threadIdx.x == 0) a.bad[obj] = 0u;
}
template <int K, int R, int CH, int W>
void launch_burst(const void *args, dim3 grid, hipStream_t st) {
    ApplyArgs<K, R> a = *(const ApplyArgs<K, R> *)args;
    grid.x = (grid.x + CH - 1) / CH;
    unsigned nb;
    a.ord = order_for<0>(grid, 0, nb);
    const int w = W > 0 ? W : (K <= 5 ? 8 : (40 / K < 2 ? 2 : 40 / K));
    hipLaunchKernelGGL((apply_burst<K, R, CH>), dim3(nb), dim3(256), W < 0 ? 0u : 160u * 1024u / (unsigned)w - 256u,
                       st, a);
}
template <int K, int R>
std::vector<Variant> burst_variants() {
    return {
        {"shipped", launch_ship<K, R>, 1, 256, false},
        {"burst CH1, lib cap", launch_burst<K, R, 1, 0>, 1, 256, false},
        {"burst CH2, lib cap", launch_burst<K, R, 2, 0>, 1, 256, false},
        {"burst CH4, lib cap", launch_burst<K, R, 4, 0>, 1, 256, false},
        {"burst CH2, cap 8", launch_burst<K, R, 2, 8>, 1, 256, false},
        {"burst CH4, cap 8", launch_burst<K, R, 4, 8>, 1, 256, false},
        {"burst CH4, full occupancy", launch_burst<K, R, 4, -1>, 1, 256, false},
        {"burst CH8, full occupancy", launch_burst<K, R, 8, -1>, 1, 256, false},
    };
}

// KB_SET=multi: cost of the mixed-pattern kernel's per-workgroup lookups
// (object index, pass index, then the pass) on a uniform pattern, and its
// occupancy cap
template <int K, int R>
std::vector<Variant> multi_variants() {
    return {
        {"shipped", launch_ship<K, R>, 1, 256, false},
        {"device pass, library cap", launch_cpc<K, R, 0>, 1, 256, false},
        {"multi, library cap", launch_mc<K, R, 0>, 1, 256, false},
        {"multi, cap 2", launch_mc<K, R, 2>, 1, 256, false},
        {"multi, cap 6", launch_mc<K, R, 6>, 1, 256, false},
        {"multi, cap 8", launch_mc<K, R, 8>, 1, 256, false},
        {"multi, cap 12", launch_mc<K, R, 12>, 1, 256, false},
        {"multi, full occupancy", launch_m<K, R, 1>, 1, 256, false},
    };
}

// KB_SET=occ: occupancy sweep
template <int K, int R>
std::vector<Variant> occ_variants() {
    return {
        {"shipped", launch_ship<K, R>, 1, 256, false},
        {"nt/nt, full occupancy", launch_v<K, R, 1, 256, 2, 2>, 1, 256, false},
        {"library launch_plan", launch_lib<K, R>, 1, 256, false},
        {"occ<=1 U1", launch_occ<K, R, 1>, 1, 256, false},
        {"occ<=2 U1", launch_occ<K, R, 2>, 1, 256, false},
        {"occ<=3 U1", launch_occ<K, R, 3>, 1, 256, false},
        {"occ<=4 U1", launch_occ<K, R, 4>, 1, 256, false},
        {"occ<=5 U1", launch_occ<K, R, 5>, 1, 256, false},
        {"occ<=1 U2", launch_occ<K, R, 1, 2>, 2, 256, false},
        {"occ<=2 U2", launch_occ<K, R, 2, 2>, 2, 256, false},
        {"occ<=1 B512", launch_occ<K, R, 1, 1, 512>, 1, 512, false},
        {"occ<=2 B512", launch_occ<K, R, 2, 1, 512>, 1, 512, false},
        {"occ<=1 B1024", launch_occ<K, R, 1, 1, 1024>, 1, 1024, false},
        {"persistent W=2", launch_pers<K, R, 2>, 1, 256, false},
        {"persistent W=4", launch_pers<K, R, 4>, 1, 256, false},
        {"persistent W=8", launch_pers<K, R, 8>, 1, 256, false},
    };
}

// KB_SET=order: cold-HBM sweep of the launch order with nt/nt policy
template <int K, int R>
std::vector<Variant> order_variants() {
    return {
        {"shipped", launch_ship<K, R>, 1, 256, false},
        {"nt/nt, full occupancy", launch_v<K, R, 1, 256, 2, 2>, 1, 256, false},
        {"nt/sc1 (pre-retune)", launch_v<K, R, 1, 256, 2, 16>, 1, 256, false},
        {"nt/nt linear", launch_v<K, R, 1, 256, 2, 2, false, 1>, 1, 256, false},
        {"nt/nt XCD-contiguous", launch_v<K, R, 1, 256, 2, 2, false, 2>, 1, 256, false},
        {"nt/nt regions M=1", launch_rg<K, R, 1>, 1, 256, false},
        {"nt/nt regions M=2", launch_rg<K, R, 2>, 1, 256, false},
        {"nt/nt regions M=4", launch_rg<K, R, 4>, 1, 256, false},
        {"nt/nt regions M=8", launch_rg<K, R, 8>, 1, 256, false},
        {"nt/nt regions M=32", launch_rg<K, R, 32>, 1, 256, false},
        {"B128 nt/nt regions M=1", launch_rg<K, R, 1, 128>, 1, 128, false},
        {"B128 nt/nt regions M=2", launch_rg<K, R, 2, 128>, 1, 128, false},
        {"B512 nt/nt regions M=1", launch_rg<K, R, 1, 512>, 1, 512, false},
        {"occupancy <= 2 WG/CU", launch_occ<K, R, 2>, 1, 256, false},
        {"occupancy <= 3 WG/CU", launch_occ<K, R, 3>, 1, 256, false},
        {"occupancy <= 4 WG/CU", launch_occ<K, R, 4>, 1, 256, false},
        {"occupancy <= 6 WG/CU", launch_occ<K, R, 6>, 1, 256, false},
        {"xor-only, SA nt", launch_xs<K, R, 2>, 1, 256, true},
    };
}

// the shipped launch (XCD order, occupancy cap) with other cache-policy bits
template <int K, int R, int LA, int SA>
void launch_capp(const void *args, dim3 grid, hipStream_t st) {
    ApplyArgs<K, R> a = *(const ApplyArgs<K, R> *)args;
    unsigned nb;
    a.ord = order_for<0>(grid, 0, nb);
    const int w = K <= 5 ? 8 : (40 / K < 2 ? 2 : 40 / K);
    hipLaunchKernelGGL((gf_apply_kernel<K, R, 1, 256, LA, SA, kFormChunks>), dim3(nb), dim3(256),
                       a.p.nw ? 160u * 1024u / (unsigned)w - 256u : 0u, st, a);
}
template <int K, int R>
std::vector<Variant> capp_variants() {
    return {
        {"shipped (nt / nt)", launch_ship<K, R>, 1, 256, false},
        {"cap, nt / sc1 nt", launch_capp<K, R, 2, 18>, 1, 256, false},
        {"cap, nt / sc0 sc1 nt", launch_capp<K, R, 2, 19>, 1, 256, false},
        {"cap, nt / sc0 nt", launch_capp<K, R, 2, 3>, 1, 256, false},
        {"cap, nt / sc1", launch_capp<K, R, 2, 16>, 1, 256, false},
        {"cap, sc1 nt / nt", launch_capp<K, R, 18, 2>, 1, 256, false},
        {"cap, sc0 sc1 nt / nt", launch_capp<K, R, 19, 2>, 1, 256, false},
        {"cap, default / nt", launch_capp<K, R, 0, 2>, 1, 256, false},
    };
}

// KB_SET=policy: cache-policy bits of loads (LA) and stores (SA); gfx950
// buffer-op aux: 1 = sc0, 2 = nt, 16 = sc1
template <int K, int R>
std::vector<Variant> policy_variants() {
    return {
        {"shipped", launch_ship<K, R>, 1, 256, false},
        {"nt/nt, full occupancy", launch_v<K, R, 1, 256, 2, 2>, 1, 256, false},
        {"LA nt / SA sc1 (pre-retune)", launch_v<K, R, 1, 256, 2, 16>, 1, 256, false},
        {"LA nt / SA 0", launch_v<K, R, 1, 256, 2, 0>, 1, 256, false},
        {"LA nt / SA sc0", launch_v<K, R, 1, 256, 2, 1>, 1, 256, false},
        {"LA nt / SA nt", launch_v<K, R, 1, 256, 2, 2>, 1, 256, false},
        {"LA nt / SA sc0 nt", launch_v<K, R, 1, 256, 2, 3>, 1, 256, false},
        {"LA nt / SA sc1 nt", launch_v<K, R, 1, 256, 2, 18>, 1, 256, false},
        {"LA nt / SA sc0 sc1 nt", launch_v<K, R, 1, 256, 2, 19>, 1, 256, false},
        {"LA sc0 nt / SA nt", launch_v<K, R, 1, 256, 3, 2>, 1, 256, false},
        {"LA sc1 nt / SA nt", launch_v<K, R, 1, 256, 18, 2>, 1, 256, false},
        {"LA sc0 sc1 nt / SA nt", launch_v<K, R, 1, 256, 19, 2>, 1, 256, false},
        {"LA sc0 sc1 / SA nt", launch_v<K, R, 1, 256, 17, 2>, 1, 256, false},
        {"B128 nt/nt", launch_v<K, R, 1, 128, 2, 2>, 1, 128, false},
        {"B512 nt/nt", launch_v<K, R, 1, 512, 2, 2>, 1, 512, false},
        {"U2 nt/nt", launch_v<K, R, 2, 256, 2, 2>, 2, 256, false},
        {"nt/nt XCD order", launch_v<K, R, 1, 256, 2, 2, false, 2>, 1, 256, false},
        {"nt/nt linear order", launch_v<K, R, 1, 256, 2, 2, false, 1>, 1, 256, false},
        {"xor-only, SA sc1", launch_xs<K, R, 16>, 1, 256, true},
        {"xor-only, SA nt", launch_xs<K, R, 2>, 1, 256, true},
        {"xor-only, SA sc0 sc1 nt", launch_xs<K, R, 19>, 1, 256, true},
    };
}

// Two-phase coding (KB_SET=twophase): the write stream costs ~13 % more mixed
// with the read stream than the two cost separately (KB_SET=stream).  Phase A
// reads a sub-batch's input rows from HBM and writes its outputs into a small
// scratch ring (SB objects x nw rows, kept in the 256 MiB Infinity Cache by
// sc1 stores, re-dirtied every sub-batch); phase B copies the ring to the real
// output rows (Infinity-Cache reads, nt HBM writes).  DRAM then sees a
// read-only stream and a write-only stream in turn.
static uint8_t *g_scr = nullptr;
template <int K, int R, int SA>
__global__ __launch_bounds__(256) void phase_a(const ApplyArgs<K, R> a, uint8_t *scr, uint32_t pitch) {
    uint32_t obj, chunk;
    if (!wg_item(a.ord, obj, chunk)) return;
    const uint32_t v = chunk * 256 + threadIdx.x;
    if (v >= a.nvec) return;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(a.base + (uint64_t)obj * a.obj_stride), (short)0, (int)a.p.span, 0x00020000);
    const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(scr + (uint64_t)obj * R * pitch), (short)0, (int)(R * pitch), 0x00020000);
    u32x4 x[K];
#pragma unroll
    for (int c = 0; c < K; ++c) x[c] = __builtin_amdgcn_raw_buffer_load_b128(rs, v * 16u, a.p.in_off[c], 2);
    uint32_t acc[R][4];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int d = 0; d < 4; ++d) acc[r][d] = 0;
#pragma unroll
    for (int c = 0; c < K; ++c) {
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            const GfIdx g = gf_idx(x[c][d]);
#pragma unroll
            for (int r = 0; r < R; ++r) acc[r][d] = gf_mac(acc[r][d], &a.p.tab[(c * R + r) * kTabWords], g);
        }
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int d = 0; d < 4; ++d) asm volatile("" : "+v"(acc[r][d]));
        __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        u32x4 o = {acc[r][0], acc[r][1], acc[r][2], acc[r][3]};
        __builtin_amdgcn_raw_buffer_store_b128(o, ro, v * 16u, r * pitch, SA);
    }
}
template <int K, int R, int LA>
__global__ __launch_bounds__(256) void phase_b(const ApplyArgs<K, R> a, const uint8_t *scr, uint32_t pitch) {
    uint32_t obj, chunk;
    if (!wg_item(a.ord, obj, chunk)) return;
    const uint32_t v = chunk * 256 + threadIdx.x;
    if (v >= a.nvec) return;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(a.base + (uint64_t)obj * a.obj_stride), (short)0, (int)a.p.span, 0x00020000);
    const __amdgpu_buffer_rsrc_t ri = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(scr + (uint64_t)obj * R * pitch), (short)0, (int)(R * pitch), 0x00020000);
    u32x4 o[R];
#pragma unroll
    for (int r = 0; r < R; ++r) o[r] = __builtin_amdgcn_raw_buffer_load_b128(ri, v * 16u, r * pitch, LA);
#pragma unroll
    for (int r = 0; r < R; ++r) __builtin_amdgcn_raw_buffer_store_b128(o[r], rs, v * 16u, a.p.out_off[r], 2);
    if (a.p.clear && v == 0) a.bad[obj] = 0u;
}
template <int K, int R, int SB, int SA, int LA>
void launch_2p(const void *args, dim3 grid, hipStream_t st) {
    const int nobj = (int)grid.y;
    for (int o0 = 0; o0 < nobj; o0 += SB) {
        ApplyArgs<K, R> a = *(const ApplyArgs<K, R> *)args;
        a.base += (size_t)o0 * a.obj_stride;
        a.bad += o0;
        const dim3 g(grid.x, std::min(SB, nobj - o0));
        unsigned nb;
        a.ord = order_for<0>(g, 0, nb);
        hipLaunchKernelGGL((phase_a<K, R, SA>), dim3(nb), dim3(256), 0, st, a, g_scr, g_pitch);
        hipLaunchKernelGGL((phase_b<K, R, LA>), dim3(nb), dim3(256), 0, st, a, (const uint8_t *)g_scr, g_pitch);
    }
}
template <int K, int R>
std::vector<Variant> twophase_variants() {
    return {
        {"shipped", launch_ship<K, R>, 1, 256, false},
        {"nt/nt, full occupancy", launch_v<K, R, 1, 256, 2, 2>, 1, 256, false},
        {"2-phase SB=64 sc1", launch_2p<K, R, 64, 16, 16>, 1, 256, false},
        {"2-phase SB=128 sc1", launch_2p<K, R, 128, 16, 16>, 1, 256, false},
        {"2-phase SB=256 sc1", launch_2p<K, R, 256, 16, 16>, 1, 256, false},
        {"2-phase SB=512 sc1", launch_2p<K, R, 512, 16, 16>, 1, 256, false},
        {"2-phase SB=256 default", launch_2p<K, R, 256, 0, 0>, 1, 256, false},
        {"2-phase SB=256 sc0sc1", launch_2p<K, R, 256, 17, 17>, 1, 256, false},
        {"read-only, K rows", launch_sr<K, R>, 1, 256, true, K, 0},
        {"write-only, nw rows", launch_sw<K, R, R>, 1, 256, true, 0, R},
    };
}

// memory-pattern ceiling under the product's launch policy: the same loads and
// stores as the pass, XOR instead of GF math, XCD-contiguous workgroup order
// and the occupancy cap of passes that store and check rows (W = 4
// workgroups per CU through an LDS reservation), nt loads and stores
template <int K, int R>
__global__ __launch_bounds__(256) void xor_policy(const ApplyArgs<K, R> a) {
    uint32_t obj, chunk;
    if (!wg_item(a.ord, obj, chunk)) return;
    const uint32_t v = chunk * 256 + threadIdx.x;
    if (v >= a.nvec) return;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(a.base + (uint64_t)obj * a.obj_stride), (short)0, (int)a.p.span, 0x00020000);
    u32x4 x[K];
#pragma unroll
    for (int c = 0; c < K; ++c) x[c] = __builtin_amdgcn_raw_buffer_load_b128(rs, v * 16u, a.p.in_off[c], 2);
    u32x4 acc = x[0];
#pragma unroll
    for (int c = 1; c < K; ++c) acc ^= x[c];
    for (uint32_t r = 0; r < a.p.nw; ++r)
        __builtin_amdgcn_raw_buffer_store_b128(acc, rs, v * 16u, a.p.out_off[r], 2);
    if (a.p.nw == 0 && acc[0] == 0x12345678u && acc[1] == 0x9abcdef0u) a.bad[0] = 1;  // keep live
}
template <int K, int R, int W>
void launch_xp(const void *args, dim3 grid, hipStream_t st) {
    ApplyArgs<K, R> a = *(const ApplyArgs<K, R> *)args;
    unsigned nb;
    a.ord = order_for<0>(grid, 0, nb);
    hipLaunchKernelGGL((xor_policy<K, R>), dim3(nb), dim3(256), W ? (160u * 1024u) / W - 256u : 0u, st, a);
}

// KB_SET=tri: the library's own launch (launch_plan) with the input-triples
// kernel off / on (set_tri_mode), 16-B and 8-B lanes; the reference output
// is the single-input kernel's (mode 0)
template <int K, int R, int MODE>
void launch_lib_tri(const void *args, dim3 grid, hipStream_t st) {
    set_tri_mode(MODE);
    launch_lib<K, R>(args, grid, st);
    set_tri_mode(0);
}
template <int K, int R>
std::vector<Variant> tri_variants() {
    return {
        {"lib, single inputs", launch_lib_tri<K, R, 0>, 1, 256, false},
        {"lib, gf_apply_tri", launch_lib_tri<K, R, 1>, 1, 256, false},
        {"xor-only ceiling", launch_x<K, R>, 1, 256, true},
        {"xor-only, product policy W4", launch_xp<K, R, 4>, 1, 256, true},
        {"xor-only, XCD order, no cap", launch_xp<K, R, 0>, 1, 256, true},
    };
}

template <int K, int R>
std::vector<Variant> stream_variants() {
    return {
        {"shipped", launch_ship<K, R>, 1, 256, false},
        {"nt/nt, full occupancy", launch_v<K, R, 1, 256, 2, 2>, 1, 256, false},
        {"read-only, K rows", launch_sr<K, R>, 1, 256, true, K, 0},
        {"write-only, 2 rows", launch_sw<K, R, 2>, 1, 256, true, 0, 2},
        {"write-only, 12 rows", launch_sw<K, R, 12>, 1, 256, true, 0, 12},
        {"xor-only (same streams)", launch_xs<K, R, 2>, 1, 256, true},
    };
}

template <int K, int R>
std::vector<Variant> variants() {
    if (std::getenv("KB_SET") && std::string(std::getenv("KB_SET")) == "tri") return tri_variants<K, R>();
    if (std::getenv("KB_SET") && std::string(std::getenv("KB_SET")) == "stream") return stream_variants<K, R>();
    if (std::getenv("KB_SET") && std::string(std::getenv("KB_SET")) == "rows") return rows_variants<K, R>();
    if (std::getenv("KB_SET") && std::string(std::getenv("KB_SET")) == "multi") return multi_variants<K, R>();
    if (std::getenv("KB_SET") && std::string(std::getenv("KB_SET")) == "burst") return burst_variants<K, R>();
    if (std::getenv("KB_SET") && std::string(std::getenv("KB_SET")) == "small") return small_variants<K, R>();
    if (std::getenv("KB_SET") && std::string(std::getenv("KB_SET")) == "occ") return occ_variants<K, R>();
    if (std::getenv("KB_SET") && std::string(std::getenv("KB_SET")) == "capp") return capp_variants<K, R>();
    if (std::getenv("KB_SET") && std::string(std::getenv("KB_SET")) == "twophase") return twophase_variants<K, R>();
    if (std::getenv("KB_SET") && std::string(std::getenv("KB_SET")) == "policy") return policy_variants<K, R>();
    if (std::getenv("KB_SET") && std::string(std::getenv("KB_SET")) == "order") return order_variants<K, R>();
    return {
        {"shipped", launch_ship<K, R>, 1, 256, false},
        {"nt/nt, full occupancy", launch_v<K, R, 1, 256, 2, 2>, 1, 256, false},
        {"nt/sc1 (pre-retune)", launch_v<K, R, 1, 256, 2, 16>, 1, 256, false},
        {"no identity inputs", launch_v<K, R, 1, 256, 2, 2, true>, 1, 256, false},
        {"nt/sc01", launch_v<K, R, 1, 256, 2, 17>, 1, 256, false},
        {"default-policy", launch_v<K, R, 1, 256, 0, 0>, 1, 256, false},
        {"B128 nt/nt", launch_v<K, R, 1, 128, 2, 2>, 1, 128, false},
        {"B512 nt/nt", launch_v<K, R, 1, 512, 2, 2>, 1, 512, false},
        {"U2 nt/nt", launch_v<K, R, 2, 256, 2, 2>, 2, 256, false},
        {"U4 nt/nt", launch_v<K, R, 4, 256, 2, 2>, 4, 256, false},
        {"B1024 nt/nt", launch_v<K, R, 1, 1024, 2, 2>, 1, 1024, false},
        {"walk CH2", launch_w<K, R, 2>, 1, 256, false},
        {"walk CH4", launch_w<K, R, 4>, 1, 256, false},
        {"walk CH8", launch_w<K, R, 8>, 1, 256, false},
        {"default loads / sc1", launch_v<K, R, 1, 256, 0, 16>, 1, 256, false},
        {"nt / default stores", launch_v<K, R, 1, 256, 2, 0>, 1, 256, false},
        {"object-major grid", launch_om<K, R>, 1, 256, false},
        {"order: linear", launch_v<K, R, 1, 256, 2, 2, false, 1>, 1, 256, false},
        {"order: XCD-contiguous", launch_v<K, R, 1, 256, 2, 2, false, 2>, 1, 256, false},
        {"LDS log/exp tables (ablation)", launch_lds<K, R>, 1, 256, false},
        {"device pass (uniform)", launch_cp<K, R>, 1, 256, false},
        {"multi CH1", launch_m<K, R, 1>, 1, 256, false},
        {"multi CH2", launch_m<K, R, 2>, 1, 256, false},
        {"multi CH4", launch_m<K, R, 4>, 1, 256, false},
        {"multi CH8", launch_m<K, R, 8>, 1, 256, false},
        {"xor-only ceiling", launch_x<K, R>, 1, 256, true},
    };
}

template <int K, int R>
int run(rsgpu_ctx *ctx, Plan &plan, size_t S, int nobj, int rounds, const char *shape) {
    const int n = ctx->n;
    // KB_PALIGN: row pitch alignment (default 256; 16 packs small rows tight)
    const size_t pal = std::getenv("KB_PALIGN") ? (size_t)std::atoi(std::getenv("KB_PALIGN")) : 256;
    const size_t pitch = (S + pal - 1) / pal * pal, stride = n * pitch, total = stride * nobj;
    // KB_ROT=NB: NB copies of the batch; every timed launch moves on to the
    // next copy, so with NB*total >> 256 MiB no byte of a launch is still in
    // the Infinity Cache from the launch before (cold-HBM rate; NB=1 repeats
    // one batch, which a 1.3 GB sweep partly re-reads from that cache)
    const int NB = std::max(1, std::getenv("KB_ROT") ? std::atoi(std::getenv("KB_ROT")) : 1);
    g_pitch = (uint32_t)pitch;
    g_plan = &plan;
    g_S = S;
    CK(hipMalloc(&g_scr, (size_t)512 * R * pitch));  // two-phase scratch ring (<= 512 objects)
    // KB_ALLOC=1: physically contiguous allocation (hipDeviceMallocContiguous),
    // which lets the driver map the batch with the largest page fragments
    const int alloc = std::getenv("KB_ALLOC") ? std::atoi(std::getenv("KB_ALLOC")) : 0;
    uint8_t *d;
    if (alloc == 1) CK(hipExtMallocWithFlags((void **)&d, total * NB, hipDeviceMallocContiguous));
    else CK(hipMalloc(&d, total * NB));
    std::printf("allocation: %s\n", alloc == 1 ? "hipExtMallocWithFlags(contiguous)" : "hipMalloc");
    uint32_t *bad;
    CK(hipMalloc(&bad, nobj * 4));
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, d, total * NB, 12345ull);
    CK(hipDeviceSynchronize());
    // consistent parity for check-row plans
    if (rsgpu_encode_dev(ctx, d, S, pitch, stride, nobj * NB, nullptr)) return 1;
    CK(hipDeviceSynchronize());

    ApplyArgs<K, R> a;
    std::memset(&a, 0, sizeof(a));
    a.base = d;
    a.obj_stride = stride;
    a.bad = bad;
    a.nvec = (uint32_t)((S + 15) / 16);
    a.tail = (uint32_t)(S - (a.nvec - 1) * 16);
    a.p.nw = (uint32_t)plan.nw;
    a.p.clear = plan.nw == plan.R;
    a.p.ki = (uint32_t)plan.ki;
    int maxrow = 0;
    for (int c = 0; c < K; ++c) {
        a.p.in_off[c] = (uint32_t)(plan.in_rows[c] * pitch);
        maxrow = std::max(maxrow, plan.in_rows[c]);
    }
    for (int r = 0; r < R; ++r) {
        const int row = plan.out_rows[r];
        a.p.out_off[r] = (uint32_t)((row < 0 ? 0 : row) * pitch);
        maxrow = std::max(maxrow, row);
        for (int c = 0; c < K; ++c)
            for (int g = 0; g < kTabWords; ++g) a.p.tab[(c * R + r) * kTabWords + g] = plan.tab[((size_t)r * K + c) * kTabWords + g];
    }
    a.p.span = (uint32_t)((size_t)maxrow * pitch + (size_t)a.nvec * 16);

    // device pass image for the multi variant: one pass, identity object list
    Pass<K, R> *d_pass;
    uint32_t *d_objs;
    CK(hipMalloc(&d_pass, sizeof(Pass<K, R>)));
    CK(hipMalloc(&d_objs, nobj * 8));
    CK(hipMemcpy(d_pass, &a.p, sizeof(Pass<K, R>), hipMemcpyHostToDevice));
    {
        std::vector<uint32_t> h(nobj * 2, 0);
        for (int o = 0; o < nobj; ++o) h[o] = o;
        CK(hipMemcpy(d_objs, h.data(), nobj * 8, hipMemcpyHostToDevice));
    }
    MultiArgs<K, R> ma;
    ma.base = d;
    ma.obj_stride = stride;
    ma.bad = bad;
    ma.nvec = a.nvec;
    ma.tail = a.tail;
    ma.passes = d_pass;
    ma.objs = d_objs;
    ma.obj_pass = d_objs + nobj;
    g_multi_args = &ma;

    {   // log/exp tables + per-(input,row) coefficient logs for the LDS ablation
        const GF &g = gf();
        uint8_t le[256 + 512];
        for (int i = 0; i < 256; ++i) le[i] = g.log[i];
        for (int i = 0; i < 512; ++i) le[256 + i] = g.exp[i];
        CK(hipMemcpyToSymbol(HIP_SYMBOL(c_logexp), le, sizeof(le)));
        std::vector<uint8_t> lc(K * R);
        for (int c = 0; c < K; ++c)
            for (int r = 0; r < R; ++r) {
                const uint8_t cf = plan.coef[(size_t)r * K + c];
                lc[c * R + r] = cf == 0 ? 255 : g.log[cf];
            }
        uint8_t *d_lc;
        CK(hipMalloc(&d_lc, lc.size()));
        CK(hipMemcpy(d_lc, lc.data(), lc.size(), hipMemcpyHostToDevice));
        g_logc = d_lc;
    }
    hipStream_t st;
    CK(hipStreamCreate(&st));
    std::vector<Variant> vs = variants<K, R>();
    const int nv = (int)vs.size();
    auto grid = [&](const Variant &v) {
        return dim3((a.nvec + v.BS * v.U - 1) / (v.BS * v.U), nobj);
    };
    // reference output from the library's own pass (single-input kernel)
    set_tri_mode(0);
    CK(hipMemset(bad, 0, nobj * 4));
    CK(launch_plan(plan, Layout{d, stride, pitch, S, nobj}, bad, st));
    CK(hipStreamSynchronize(st));
    std::vector<uint8_t> ref(total), got(total);
    std::vector<uint32_t> hb(nobj);
    CK(hipMemcpy(ref.data(), d, total, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hb.data(), bad, nobj * 4, hipMemcpyDeviceToHost));
    for (int o = 0; o < nobj; ++o)
        if (hb[o]) { std::printf("library pass flagged object %d\n", o); return 1; }
    std::vector<std::string> status(nv);
    for (int v = 0; v < nv; ++v) {
        if (vs[v].ceiling) { status[v] = "(pattern ceiling)"; continue; }
        for (int r = 0; r < plan.nw; ++r)
            for (int o = 0; o < nobj; o += 61)
                CK(hipMemset(d + o * stride + plan.out_rows[r] * pitch, 0x5A, S));
        CK(hipMemset(bad, 0xFF, nobj * 4));
        vs[v].fn(&a, grid(vs[v]), st);
        CK(hipStreamSynchronize(st));
        CK(hipMemcpy(got.data(), d, total, hipMemcpyDeviceToHost));
        CK(hipMemcpy(hb.data(), bad, nobj * 4, hipMemcpyDeviceToHost));
        bool ok = true;
        for (int o = 0; o < nobj && ok; ++o) {
            if (plan.nw < plan.R && hb[o] != 0xFFFFFFFFu) ok = false;  // no spurious flags
            if (plan.nw == plan.R && hb[o] != 0) ok = false;          // cleared by the pass
            for (int r = 0; r < plan.nw; ++r) {
                const size_t off = o * stride + plan.out_rows[r] * pitch;
                if (std::memcmp(&got[off], &ref[off], S)) ok = false;
            }
        }
        status[v] = ok ? "bit-exact" : "MISMATCH";
    }
    std::vector<std::vector<float>> ms(nv);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int it = 0; it < rounds + 3; ++it)
        for (int v = 0; v < nv; ++v)
            for (int j = 0; j < NB; ++j) {
                a.base = d + (size_t)j * total;
                ma.base = a.base;
                CK(hipEventRecord(e0, st));
                vs[v].fn(&a, grid(vs[v]), st);
                CK(hipEventRecord(e1, st));
                CK(hipEventSynchronize(e1));
                float t;
                CK(hipEventElapsedTime(&t, e0, e1));
                if (it >= 3) ms[v].push_back(t);
            }
    const double alg = (double)nobj * (plan.K + plan.nw) * S;
    std::printf("shape %s: K=%d R=%d (nw=%d, ki=%d) S=%zu nobj=%d, algorithmic bytes/launch %.0f, "
                "%d rotating batch cop%s (%s)\n",
                shape, K, R, plan.nw, plan.ki, S, nobj, alg, NB, NB > 1 ? "ies" : "y",
                NB > 1 ? "cold Infinity Cache" : "repeat: warm Infinity Cache");
    for (int v = 0; v < nv; ++v) {
        std::vector<float> x = ms[v];
        std::sort(x.begin(), x.end());
        const double med = x[x.size() / 2];
        const double vb = (vs[v].rd < 0 && vs[v].wr < 0)
                              ? alg
                              : (double)nobj * (vs[v].rd + vs[v].wr) * S;  // this variant's own bytes
        std::printf("  %-26s med %8.1f us  best %8.1f us  %7.1f GB/s  %5.1f%% of 8 TB/s  %s\n",
                    vs[v].name.c_str(), med * 1e3, x[0] * 1e3, vb / (med * 1e-3) / 1e9,
                    100.0 * vb / (med * 1e-3) / 8e12, status[v].c_str());
    }
    CK(hipFree(d));
    CK(hipFree(bad));
    return 0;
}

// Pitch sweep: the shipped variant of one plan on layouts whose row pitch is
// roundup(S, 256) + pad, interleaved in one process (HBM channel effects).
// One encoded buffer per pad (row pitch = roundup(S, 256) + pad) and its kernarg.
template <int K, int R>
int setup_bufs(rsgpu_ctx *ctx, Plan &plan, size_t S, int nobj, const std::vector<size_t> &pads,
               std::vector<uint8_t *> &bufs, std::vector<ApplyArgs<K, R>> &args, uint32_t *&bad) {
    const int n = ctx->n;
    const int np = (int)pads.size();
    bufs.assign(np, nullptr);
    args.assign(np, ApplyArgs<K, R>());
    CK(hipMalloc(&bad, nobj * 4));
    for (int i = 0; i < np; ++i) {
        const size_t pitch = (S + 255) / 256 * 256 + pads[i], stride = n * pitch;
        CK(hipMalloc(&bufs[i], stride * nobj));
        hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, bufs[i], stride * nobj, 777ull);
        CK(hipDeviceSynchronize());
        if (rsgpu_encode_dev(ctx, bufs[i], S, pitch, stride, nobj, nullptr)) return 1;
        ApplyArgs<K, R> &a = args[i];
        std::memset(&a, 0, sizeof(a));
        a.base = bufs[i];
        a.obj_stride = stride;
        a.bad = bad;
        a.nvec = (uint32_t)((S + 15) / 16);
        a.tail = (uint32_t)(S - (a.nvec - 1) * 16);
        a.p.nw = (uint32_t)plan.nw;
        a.p.clear = plan.nw == plan.R;
        a.p.ki = (uint32_t)plan.ki;
        int maxrow = 0;
        for (int c = 0; c < K; ++c) {
            a.p.in_off[c] = (uint32_t)(plan.in_rows[c] * pitch);
            maxrow = std::max(maxrow, plan.in_rows[c]);
        }
        for (int r = 0; r < R; ++r) {
            const int row = plan.out_rows[r];
            a.p.out_off[r] = (uint32_t)((row < 0 ? 0 : row) * pitch);
            maxrow = std::max(maxrow, row);
            for (int c = 0; c < K; ++c)
                for (int g = 0; g < kTabWords; ++g) a.p.tab[(c * R + r) * kTabWords + g] = plan.tab[((size_t)r * K + c) * kTabWords + g];
        }
        a.p.span = (uint32_t)((size_t)maxrow * pitch + (size_t)a.nvec * 16);
    }
    CK(hipDeviceSynchronize());
    return 0;
}

template <int K, int R>
int pitch_sweep(rsgpu_ctx *ctx, Plan &plan, size_t S, int nobj, int rounds, const char *shape) {
    // every buffer is revisited only after the other pads' buffers (>= 9 GB of
    // traffic), so this sweep is cold
    const std::vector<size_t> pads = {0, 16, 64, 128, 256, 512, 1024, 2048, 3072, 4096, 4352, 8192, 65792};
    const int np = (int)pads.size();
    std::vector<uint8_t *> bufs;
    std::vector<ApplyArgs<K, R>> args;
    uint32_t *bad;
    if (setup_bufs<K, R>(ctx, plan, S, nobj, pads, bufs, args, bad)) return 1;
    CK(hipDeviceSynchronize());
    hipStream_t st;
    CK(hipStreamCreate(&st));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<std::vector<float>> ms(np);
    const dim3 grid((args[0].nvec + 255) / 256, nobj);
    for (int it = 0; it < rounds + 3; ++it)
        for (int i = 0; i < np; ++i) {
            CK(hipEventRecord(e0, st));
            launch_ship<K, R>(&args[i], grid, st);
            CK(hipEventRecord(e1, st));
            CK(hipEventSynchronize(e1));
            float t;
            CK(hipEventElapsedTime(&t, e0, e1));
            if (it >= 3) ms[i].push_back(t);
        }
    const double alg = (double)nobj * (plan.K + plan.nw) * S;
    std::printf("pitch sweep %s: K=%d R=%d S=%zu nobj=%d\n", shape, K, R, S, nobj);
    for (int i = 0; i < np; ++i) {
        std::vector<float> x = ms[i];
        std::sort(x.begin(), x.end());
        const double med = x[x.size() / 2];
        const size_t pitch = (S + 255) / 256 * 256 + pads[i];
        std::printf("  pitch %8zu (+%5zu)  med %8.1f us  %7.1f GB/s  %5.1f%% of 8 TB/s\n", pitch, pads[i],
                    med * 1e3, alg / (med * 1e-3) / 1e9, 100.0 * alg / (med * 1e-3) / 8e12);
    }
    for (auto b : bufs) CK(hipFree(b));
    CK(hipFree(bad));
    return 0;
}

// Translation warmth: NB same-pitch buffers, each launch timed either
// repeating one buffer (its pages' translations stay warm) or rotating
// through all NB (every launch sweeps pages untouched for NB-1 launches),
// in linear and XCD-contiguous workgroup order.
template <int K, int R>
int rot_sweep(rsgpu_ctx *ctx, Plan &plan, size_t S, int nobj, int rounds, const char *shape) {
    const int NB = 4;
    std::vector<uint8_t *> bufs;
    std::vector<ApplyArgs<K, R>> args;
    uint32_t *bad;
    if (setup_bufs<K, R>(ctx, plan, S, nobj, std::vector<size_t>(NB, 0), bufs, args, bad)) return 1;
    hipStream_t st;
    CK(hipStreamCreate(&st));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const dim3 grid((args[0].nvec + 255) / 256, nobj);
    const double alg = (double)nobj * (plan.K + plan.nw) * S;
    std::printf("buffer rotation %s: K=%d R=%d S=%zu nobj=%d, %d buffers of %.2f GB\n", shape, K, R, S,
                nobj, NB, (double)args[0].obj_stride * nobj / 1e9);
    // modes 4/5: repeat one buffer, but sweep 512 MiB of scratch writes
    // through the Infinity Cache (256 MiB) before each timed launch, so no
    // byte of the launch can hit in it (cold-MALL rate)
    const char *names[6] = {"repeat, linear order", "repeat, XCD-contiguous", "rotate, linear order",
                            "rotate, XCD-contiguous", "repeat+MALL flush, linear", "repeat+MALL flush, XCD"};
    const size_t nflush = (size_t)512 << 20;
    uint8_t *flush;
    CK(hipMalloc(&flush, nflush));
    const int NM = 6;
    std::vector<std::vector<float>> ms(NM);
    for (int it = 0; it < rounds + 2; ++it)
        for (int m = 0; m < NM; ++m)
            for (int j = 0; j < NB; ++j) {
                const int i = (m == 2 || m == 3) ? j : 0;
                if (m >= 4) hipLaunchKernelGGL(fill, dim3(8192), dim3(256), 0, st, flush, nflush, 99ull + j);
                CK(hipEventRecord(e0, st));
                if (m % 2 == 0) launch_v<K, R, 1, 256, 2, 2, false, 1>(&args[i], grid, st);
                else launch_v<K, R, 1, 256, 2, 2, false, 2>(&args[i], grid, st);
                CK(hipEventRecord(e1, st));
                CK(hipEventSynchronize(e1));
                float t;
                CK(hipEventElapsedTime(&t, e0, e1));
                if (it >= 2) ms[m].push_back(t);
            }
    CK(hipFree(flush));
    for (int m = 0; m < NM; ++m) {
        std::sort(ms[m].begin(), ms[m].end());
        const double med = ms[m][ms[m].size() / 2];
        std::printf("  %-24s med %8.1f us  %7.1f GB/s  %5.1f%% of 8 TB/s\n", names[m], med * 1e3,
                    alg / (med * 1e-3) / 1e9, 100.0 * alg / (med * 1e-3) / 8e12);
    }
    for (auto b : bufs) CK(hipFree(b));
    CK(hipFree(bad));
    return 0;
}

// lib:OPk_p (OP = enc | dec | ver): times the library's own launch_plan for
// any shape, including K > 16 (the generic kernel), cold (4 rotating copies),
// 1 MiB objects, ~1.3 GB per launch.  dec = fused decode, data {0, 1} lost.
int lib_time(std::string spec, int rounds) {
    double obj_mib = 1;  // lib:OPk_p@M: object size M MiB (fractions allowed)
    if (spec.find('@') != std::string::npos) {
        obj_mib = std::atof(spec.substr(spec.find('@') + 1).c_str());
        spec = spec.substr(0, spec.find('@'));
    }
    const std::string op = spec.substr(0, 3);
    const size_t us = spec.find('_');
    const int k = std::atoi(spec.substr(3, us - 3).c_str()), p = std::atoi(spec.substr(us + 1).c_str());
    const int n = k + p;
    rsgpu_ctx *ctx;
    if (rsgpu_create(k, p, 0, 0, &ctx)) return 1;
    DeviceGuard dg_;
    if (ctx->use_device(dg_)) { std::printf("no device\n"); return 1; }
    std::shared_ptr<Plan> plan;
    std::vector<uint8_t> present(n, 1);
    if (op == "enc") plan = ctx->plan_encode();
    else if (op == "ver") plan = ctx->plan_verify();
    else {
        // KB_LOST="a,b": the lost data rows (default 0,1)
        int l0 = 0, l1 = 1;
        if (const char *e = std::getenv("KB_LOST")) std::sscanf(e, "%d,%d", &l0, &l1);
        present[l0] = present[l1] = 0;
        ctx->plan_reconstruct(present.data(), false, true, plan);
    }
    const size_t nbytes = (size_t)(obj_mib * (1 << 20)), S = (nbytes + k - 1) / k;
    // pitch: S rounded to 16 B (the smallest the layout allows) below 4 KiB
    // shards, else to 256 B as the bench batches
    const size_t pitch = S < 4096 ? (S + 15) / 16 * 16 : (S + 255) / 256 * 256, stride = (size_t)n * pitch;
    const int nobj = (int)(((size_t)1300 << 20) / stride), NB = 4;
    uint8_t *d;
    uint32_t *bad;
    CK(hipMalloc(&d, stride * nobj * NB));
    CK(hipMalloc(&bad, nobj * 4));
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, d, stride * nobj * NB, 4242ull);
    CK(hipDeviceSynchronize());
    if (rsgpu_encode_dev(ctx, d, S, pitch, stride, nobj * NB, nullptr)) return 1;
    CK(hipDeviceSynchronize());
    hipStream_t st;
    CK(hipStreamCreate(&st));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<float> ms;
    // ~0.3 s of back-to-back launches first: the shader clock ramps up under
    // sustained load, and VALU-heavy passes read up to 40 % slow without it
    for (int it = 0; it < 1000; ++it)
        CK(launch_plan(*plan, Layout{d + (size_t)(it % NB) * stride * nobj, stride, pitch, S, nobj}, bad, st));
    CK(hipStreamSynchronize(st));
    for (int it = 0; it < rounds + 2; ++it)
        for (int j = 0; j < NB; ++j) {
            CK(hipEventRecord(e0, st));
            CK(launch_plan(*plan, Layout{d + (size_t)j * stride * nobj, stride, pitch, S, nobj}, bad, st));
            CK(hipEventRecord(e1, st));
            CK(hipEventSynchronize(e1));
            float t;
            CK(hipEventElapsedTime(&t, e0, e1));
            if (it >= 2) ms.push_back(t);
        }
    std::vector<uint32_t> hb(nobj);
    CK(hipMemcpy(hb.data(), bad, nobj * 4, hipMemcpyDeviceToHost));
    for (int o = 0; o < nobj; ++o)
        if (hb[o]) { std::printf("flagged object %d\n", o); return 1; }
    std::sort(ms.begin(), ms.end());
    const double med = ms[ms.size() / 2];
    const double alg = (double)nobj * (plan->K + plan->nw) * S;
    std::printf("lib %s@%g: K=%d R=%d nw=%d S=%zu nobj=%d (%s kernel), med %.1f us, %.1f GB/s, %.1f%% of 8 TB/s\n",
                spec.c_str(), obj_mib, plan->K, plan->R, plan->nw, S, nobj, plan->K > 16 ? "generic" : "specialised",
                med * 1e3, alg / (med * 1e-3) / 1e9, 100.0 * alg / (med * 1e-3) / 8e12);
    std::fflush(stdout);
    CK(hipFree(d));
    CK(hipFree(bad));
    return 0;
}

int main(int argc, char **argv) {
    std::string shape = argc > 1 ? argv[1] : "enc10_2";
    const int rounds = argc > 2 ? std::atoi(argv[2]) : 20;
    if (shape.rfind("lib:", 0) == 0) return lib_time(shape.substr(4), rounds);
    const bool sweep = shape.rfind("pitch:", 0) == 0;  // pitch:SHAPE
    if (sweep) shape = shape.substr(6);
    const bool rot = shape.rfind("rot:", 0) == 0;  // rot:SHAPE
    if (rot) shape = shape.substr(4);
    // SHAPE@M: object size M MiB (fractions allowed), launch kept near the
    // default footprint (1 GiB of objects for 10_2, 2 GiB for 10_4)
    double obj_mib = 0;
    if (shape.find('@') != std::string::npos) {
        obj_mib = std::atof(shape.substr(shape.find('@') + 1).c_str());
        shape = shape.substr(0, shape.find('@'));
    }
    const bool p4 = shape.find("10_4") != std::string::npos;
    int k = 10, p = p4 ? 4 : 2;
    {   // encK_P / verK_P for other code widths (K <= 16 specialised shapes)
        const size_t us = shape.find('_');
        if (us != std::string::npos && us > 3 && (shape.rfind("enc", 0) == 0 || shape.rfind("ver", 0) == 0)) {
            k = std::atoi(shape.substr(3, us - 3).c_str());
            p = std::atoi(shape.substr(us + 1).c_str());
        }
    }
    const int n = k + p;
    if (obj_mib <= 0) obj_mib = p4 ? 4 : 1;
    const size_t nbytes = (size_t)(obj_mib * (1 << 20));
    int nobj = std::max(1, (int)((p4 ? 2048 : 1024) / obj_mib));
    if (shape.find('x') != std::string::npos && shape.find('x') > shape.find('_')) {  // SHAPEx N objects
        nobj = std::atoi(shape.substr(shape.find('x') + 1).c_str());
        shape = shape.substr(0, shape.find('x'));
    }
    const size_t S = (nbytes + k - 1) / k;
    rsgpu_ctx *ctx;
    if (rsgpu_create(k, p, 0, 0, &ctx)) return 1;
    DeviceGuard dg_;
    if (ctx->use_device(dg_)) { std::printf("no device\n"); return 1; }
    std::vector<uint8_t> present(n, 1);
    std::shared_ptr<Plan> plan;
    if (shape.rfind("enc", 0) == 0) {
        plan = ctx->plan_encode();
    } else if (shape.rfind("ver", 0) == 0) {
        plan = ctx->plan_verify();
    } else if (shape == "dec10_2") {  // healthy Get: data {0,5} missing, fused decode
        present[0] = present[5] = 0;
        ctx->plan_reconstruct(present.data(), false, true, plan);
    } else if (shape == "rdata10_4") {  // config 3: 10 of 14 present, ReconstructData
        present[0] = present[5] = present[12] = present[13] = 0;
        ctx->plan_reconstruct(present.data(), true, false, plan);
    } else if (shape == "decx10_4") {  // fused decode with 2 extra (checked) parity shards
        present[0] = present[5] = 0;
        ctx->plan_reconstruct(present.data(), false, true, plan);
    } else {
        std::printf("unknown shape %s\n", shape.c_str());
        return 1;
    }
    const int K = plan->K, R = plan->R;
#define SHAPE(k_, r_)                                                                       \
    if (K == k_ && R == r_)                                                                 \
        return sweep ? pitch_sweep<k_, r_>(ctx, *plan, S, nobj, rounds, shape.c_str())      \
             : rot   ? rot_sweep<k_, r_>(ctx, *plan, S, nobj, rounds, shape.c_str())        \
                     : run<k_, r_>(ctx, *plan, S, nobj, rounds, shape.c_str());
    SHAPE(10, 2) SHAPE(10, 4) SHAPE(12, 2) SHAPE(12, 4) SHAPE(14, 4) SHAPE(16, 4) SHAPE(16, 2) SHAPE(8, 4)
#undef SHAPE
    std::printf("no instantiation for K=%d R=%d\n", K, R);
    return 1;
}
