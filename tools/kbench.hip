// kbench.hip — interleaved A/B timing of gf_apply_kernel launch variants on
// the BASELINE shape (RS(10+2), 1 MiB objects, batch 1024, [obj][row][pitch]).
//
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I../infinicache_amd/csrc kbench.hip -o kbench
//   ./kbench [rounds] [k p nbytes nobj]
//
// Every variant's parity is checked bit-exact against variant 0 (which the
// product's tests pin to the oracle).  A "xor-only" variant (same streams, no
// GF math) and a plain copy give the memory-system ceilings for this access
// pattern.  Timing: one HIP-event pair per launch, variants interleaved
// round-robin in one process (methodology rule 24); median and best reported.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "gf256.h"
#include "gf_device.h"

namespace rsgpu {
const GF &gf() {
    static const GF g;
    return g;
}
}  // namespace rsgpu

using namespace rsgpu;

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(1);                                                           \
        }                                                                           \
    } while (0)

static void tables(uint8_t c, uint32_t out[4]) {
    const GF &g = gf();
    for (int grp = 0; grp < 4; ++grp) {
        uint32_t w = 0;
        for (int j = 0; j < 4; ++j) w |= (uint32_t)g.mul(c, (uint8_t)(j << (2 * grp))) << (8 * j);
        out[grp] = w;
    }
}

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

// memory-pattern ceiling: identical loads/stores, XOR instead of GF multiply
template <int K, int R>
__global__ __launch_bounds__(256) void xor_only(const ApplyArgs<K, R> a) {
    const uint32_t v = blockIdx.x * 256 + threadIdx.x;
    if (v >= a.nvec) return;
    const uint8_t *ob = a.base + (uint64_t)blockIdx.y * a.obj_stride;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void *)ob, (short)0, (int)a.span, 0x00020000);
    u32x4 x[K];
#pragma unroll
    for (int c = 0; c < K; ++c) x[c] = __builtin_amdgcn_raw_buffer_load_b128(rs, v * 16u, a.in_off[c], 0);
    u32x4 acc[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        acc[r] = x[0] ^ (u32x4){(uint32_t)r, 0, 0, 0};
#pragma unroll
        for (int c = 1; c < K; ++c) acc[r] ^= x[c];
        __builtin_amdgcn_raw_buffer_store_b128(acc[r], rs, v * 16u, a.out_off[r], 0);
    }
}

__global__ void copy16(const uint4 *__restrict__ s, uint4 *__restrict__ d, size_t n) {
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    for (; i < n; i += (size_t)gridDim.x * blockDim.x) d[i] = s[i];
}

struct Variant {
    std::string name;
    void (*launch)(const void *args, dim3 grid, hipStream_t);
    int U, BS;
};

template <int K, int R, int U, int BS, int LA, int SA>
void launch_v(const void *args, dim3 grid, hipStream_t st) {
    const ApplyArgs<K, R> &a = *(const ApplyArgs<K, R> *)args;
    hipLaunchKernelGGL((gf_apply_kernel<K, R, U, BS, LA, SA>), grid, dim3(BS), 0, st, a);
}
template <int K, int R>
void launch_xor(const void *args, dim3 grid, hipStream_t st) {
    const ApplyArgs<K, R> &a = *(const ApplyArgs<K, R> *)args;
    hipLaunchKernelGGL((xor_only<K, R>), grid, dim3(256), 0, st, a);
}

constexpr int K = 10, R = 2;

int main(int argc, char **argv) {
    const int rounds = argc > 1 ? std::atoi(argv[1]) : 30;
    const size_t nbytes = 1 << 20;
    const int nobj = 1024;
    const size_t S = (nbytes + K - 1) / K;
    const size_t pitch = (S + 255) / 256 * 256;
    const int n = K + R;
    const size_t stride = n * pitch;
    const size_t total = stride * nobj;

    // RS(10+2) parity rows (upstream buildMatrix; see oracle KATs)
    const uint8_t rows[2][10] = {{0x81, 0x96, 0xaf, 0xb8, 0xd2, 0xc4, 0xfe, 0xe8, 0x03, 0x02},
                                 {0x96, 0x81, 0xb8, 0xaf, 0xc4, 0xd2, 0xe8, 0xfe, 0x02, 0x03}};
    ApplyArgs<K, R> a;
    std::memset(&a, 0, sizeof(a));
    a.obj_stride = stride;
    a.nvec = (uint32_t)((S + 15) / 16);
    a.tail = (uint32_t)(S - (a.nvec - 1) * 16);
    a.nw = R;
    a.span = (uint32_t)((n - 1) * pitch + a.nvec * 16);
    for (int c = 0; c < K; ++c) a.in_off[c] = (uint32_t)(c * pitch);
    for (int r = 0; r < R; ++r) a.out_off[r] = (uint32_t)((K + r) * pitch);
    for (int c = 0; c < K; ++c)
        for (int r = 0; r < R; ++r) tables(rows[r][c], &a.tab[(c * R + r) * 4]);

    uint8_t *d;
    CK(hipMalloc(&d, total));
    uint8_t *dcopy;
    CK(hipMalloc(&dcopy, total));
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, d, total, 12345ull);
    CK(hipDeviceSynchronize());
    a.base = d;

    std::vector<Variant> vs = {
        {"U1_B256", launch_v<K, R, 1, 256, 0, 0>, 1, 256},
        {"ldnt_B256", launch_v<K, R, 1, 256, 2, 0>, 1, 256},
        {"ldnt_B128", launch_v<K, R, 1, 128, 2, 0>, 1, 128},
        {"ldnt_B512", launch_v<K, R, 1, 512, 2, 0>, 1, 512},
        {"ldnt_U2_B256", launch_v<K, R, 2, 256, 2, 0>, 2, 256},
        {"ldnt_U2_B128", launch_v<K, R, 2, 128, 2, 0>, 2, 128},
        {"ldnt_stsc1", launch_v<K, R, 1, 256, 2, 16>, 1, 256},
        {"ldnt_stsc01", launch_v<K, R, 1, 256, 2, 17>, 1, 256},
        {"ldntsc1_B256", launch_v<K, R, 1, 256, 18, 0>, 1, 256},
        {"ldntsc0_B256", launch_v<K, R, 1, 256, 3, 0>, 1, 256},
        {"ldsc1_B256", launch_v<K, R, 1, 256, 16, 0>, 1, 256},
        {"ldsc0_B256", launch_v<K, R, 1, 256, 1, 0>, 1, 256},
        {"ldnt_stnt_B512", launch_v<K, R, 1, 512, 2, 2>, 1, 512},
        {"xor_only", launch_xor<K, R>, 1, 256},
    };
    const int nv = (int)vs.size();
    std::vector<uint8_t> ref(total), got(total);
    hipStream_t st;
    CK(hipStreamCreate(&st));
    // reference parity from variant 0
    vs[0].launch(&a, dim3((a.nvec + 255) / 256, nobj), st);
    CK(hipStreamSynchronize(st));
    CK(hipMemcpy(ref.data(), d, total, hipMemcpyDeviceToHost));
    std::vector<bool> exact(nv, true);
    for (int v = 1; v < nv - 1; ++v) {
        CK(hipMemset(d + 0, 0, 0));
        // clobber parity rows, rerun, compare
        for (int o = 0; o < nobj; o += 97) CK(hipMemset(d + o * stride + K * pitch, 0x5A, R * pitch));
        const unsigned gx = (a.nvec + vs[v].BS * vs[v].U - 1) / (vs[v].BS * vs[v].U);
        vs[v].launch(&a, dim3(gx, nobj), st);
        CK(hipStreamSynchronize(st));
        CK(hipMemcpy(got.data(), d, total, hipMemcpyDeviceToHost));
        for (int o = 0; o < nobj && exact[v]; ++o)
            for (int r = 0; r < R; ++r)
                if (std::memcmp(&got[o * stride + (K + r) * pitch], &ref[o * stride + (K + r) * pitch], S))
                    exact[v] = false;
    }
    // timing, interleaved
    std::vector<std::vector<float>> ms(nv + 1);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const size_t n16 = total / 16;
    for (int it = 0; it < rounds + 3; ++it) {
        for (int v = 0; v <= nv; ++v) {
            CK(hipEventRecord(e0, st));
            if (v < nv) {
                const unsigned gx = (a.nvec + vs[v].BS * vs[v].U - 1) / (vs[v].BS * vs[v].U);
                vs[v].launch(&a, dim3(gx, nobj), st);
            } else {
                hipLaunchKernelGGL(copy16, dim3(8192), dim3(256), 0, st, (const uint4 *)d, (uint4 *)dcopy, n16);
            }
            CK(hipEventRecord(e1, st));
            CK(hipEventSynchronize(e1));
            float t;
            CK(hipEventElapsedTime(&t, e0, e1));
            if (it >= 3) ms[v].push_back(t);
        }
    }
    const double alg = (double)nobj * (K + R) * S;
    std::printf("shape: RS(%d+%d) S=%zu pitch=%zu nobj=%d  algorithmic bytes/launch=%.0f\n", K, R, S,
                pitch, nobj, alg);
    for (int v = 0; v <= nv; ++v) {
        std::vector<float> x = ms[v];
        std::sort(x.begin(), x.end());
        const double med = x[x.size() / 2], best = x[0];
        const double bytes = v < nv ? alg : 2.0 * total;
        std::printf("%-16s med %8.1f us  best %8.1f us  %7.1f GB/s (med)  %5.1f%% of 8 TB/s  %s\n",
                    v < nv ? vs[v].name.c_str() : "copy16(2x total)", med * 1e3, best * 1e3,
                    bytes / (med * 1e-3) / 1e9, 100.0 * bytes / (med * 1e-3) / 8e12,
                    v < nv ? (v == 0 ? "ref" : (v == nv - 1 ? "(pattern ceiling)" : (exact[v] ? "bit-exact" : "MISMATCH")))
                           : "");
    }
    return 0;
}
