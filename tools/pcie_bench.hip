// pcie_bench.hip — host<->device copy rates on the MI355X box, in the shapes
// the batch pipeline (infinicache_amd/csrc/pipeline.cpp) issues:
//   1D pinned copies of various sizes, 1..4 streams;
//   2D copies repacking Split rows (pitch S = 104,858) to the 256-B device
//   pitch (104,960) — the encode H2D of a 1 MiB RS(10+2) object;
//   H2D and D2H at the same time (the pipeline's steady state).
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <algorithm>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            std::printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));      \
            std::exit(1);                                                              \
        }                                                                              \
    } while (0)

// zero-copy copy kernel: every lane moves U 16-B vectors per iteration
// (several PCIe requests in flight per lane), grid-stride over n vectors
template <int U>
__global__ __launch_bounds__(256) void kcopy(const uint4 *__restrict__ src, uint4 *__restrict__ dst, size_t n) {
    const size_t stride = (size_t)gridDim.x * blockDim.x * U;
    for (size_t i = (size_t)blockIdx.x * blockDim.x * U + threadIdx.x; i < n; i += stride) {
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (i + (size_t)u * blockDim.x < n) v[u] = src[i + (size_t)u * blockDim.x];
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (i + (size_t)u * blockDim.x < n) dst[i + (size_t)u * blockDim.x] = v[u];
    }
}

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
    const size_t total = 2ull << 30;  // 2 GiB per direction
    uint8_t *h, *h2, *d, *d2;
    CK(hipHostMalloc(&h, total, hipHostMallocDefault));
    CK(hipHostMalloc(&h2, total, hipHostMallocDefault));
    CK(hipMalloc(&d, total));
    CK(hipMalloc(&d2, total));
    for (size_t i = 0; i < total; i += 4096) h[i] = (uint8_t)i, h2[i] = (uint8_t)i;
    uint8_t *hd = nullptr, *h2d = nullptr;  // device views of the pinned buffers (zero-copy kernels)
    CK(hipHostGetDevicePointer((void **)&hd, h, 0));
    CK(hipHostGetDevicePointer((void **)&h2d, h2, 0));
    hipStream_t st[8];
    for (auto &s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));

    auto run = [&](const char *name, int nstreams, size_t chunk, int dir /*0 h2d 1 d2h 2 both*/,
                   bool twod) {
        const size_t S = 104858, P = 104960;
        // warm
        for (int rep = 0; rep < 2; ++rep) {
            const double t0 = now();
            size_t moved = 0;
            int i = 0;
            for (size_t off = 0; off + chunk <= total; off += chunk, ++i) {
                hipStream_t s = st[i % nstreams];
                if (dir == 0 || dir == 2) {
                    if (twod) {
                        const size_t rows = chunk / P;
                        CK(hipMemcpy2DAsync(d + off, P, h + off, S, S, rows, hipMemcpyHostToDevice, s));
                        moved += rows * S;
                    } else {
                        CK(hipMemcpyAsync(d + off, h + off, chunk, hipMemcpyHostToDevice, s));
                        moved += chunk;
                    }
                }
                if (dir == 1 || dir == 2) {
                    hipStream_t s2 = dir == 2 ? st[4 + i % 4] : s;
                    if (twod) {
                        const size_t rows = chunk / P;
                        CK(hipMemcpy2DAsync(h2 + off, S, d2 + off, P, S, rows, hipMemcpyDeviceToHost, s2));
                        moved += rows * S;
                    } else {
                        CK(hipMemcpyAsync(h2 + off, d2 + off, chunk, hipMemcpyDeviceToHost, s2));
                        moved += chunk;
                    }
                }
            }
            CK(hipDeviceSynchronize());
            const double el = now() - t0;
            if (rep == 1)
                std::printf("%-34s streams=%d chunk=%9zu  %7.2f GB/s\n", name, nstreams, chunk, moved / el / 1e9);
        }
    };
    for (size_t chunk : {1ull << 20, 8ull << 20, 64ull << 20, 512ull << 20}) run("H2D 1D", 1, chunk, 0, false);
    for (int ns : {2, 4}) run("H2D 1D", ns, 8ull << 20, 0, false);
    for (size_t chunk : {1ull << 20, 8ull << 20, 64ull << 20}) run("D2H 1D", 1, chunk, 1, false);
    run("D2H 1D", 4, 8ull << 20, 1, false);
    for (size_t chunk : {12 * 104960ull, 120 * 104960ull}) run("H2D 2D repack S->P", 1, chunk, 0, true);
    run("H2D 2D repack S->P", 4, 120 * 104960ull, 0, true);
    run("D2H 2D repack P->S", 4, 120 * 104960ull, 1, true);
    // device-side repack (D2D 2D copy): pitch S -> P over 1 GiB
    {
        const size_t S = 104858, P = 104960, rows = (1ull << 30) / P;
        for (int rep = 0; rep < 2; ++rep) {
            const double t0 = now();
            CK(hipMemcpy2DAsync(d2, P, d, S, S, rows, hipMemcpyDeviceToDevice, st[0]));
            CK(hipStreamSynchronize(st[0]));
            const double el = now() - t0;
            if (rep) std::printf("%-34s rows=%zu  %7.2f GB/s (read+write)\n", "D2D 2D repack S->P", rows,
                                 2.0 * rows * S / el / 1e9);
        }
    }
    run("H2D+D2H 1D (both dirs)", 4, 8ull << 20, 2, false);
    run("H2D+D2H 2D (both dirs)", 4, 120 * 104960ull, 2, true);

    // the coding pipeline's mix: H2D of 2 GiB beside D2H of 0.4 GiB (10 rows in,
    // 2 out), by the copy engines and by zero-copy kernels (the GPU's own loads
    // and stores over PCIe), each timed to its own completion
    auto mix = [&](const char *name, bool kh2d, bool kd2h, int wgs) {
        const size_t nh = total, nd = total / 5;
        for (int rep = 0; rep < 2; ++rep) {
            hipEvent_t a0, a1, b1;
            CK(hipEventCreate(&a0));
            CK(hipEventCreate(&a1));
            CK(hipEventCreate(&b1));
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(a0, st[0]));
            CK(hipStreamWaitEvent(st[1], a0, 0));
            if (kh2d) hipLaunchKernelGGL(kcopy<4>, dim3(wgs), dim3(256), 0, st[0], (const uint4 *)hd, (uint4 *)d, nh / 16);
            else CK(hipMemcpyAsync(d, h, nh, hipMemcpyHostToDevice, st[0]));
            CK(hipEventRecord(a1, st[0]));
            if (nd) {
                if (kd2h) hipLaunchKernelGGL(kcopy<4>, dim3(wgs / 4), dim3(256), 0, st[1], (const uint4 *)d2, (uint4 *)h2d, nd / 16);
                else CK(hipMemcpyAsync(h2, d2, nd, hipMemcpyDeviceToHost, st[1]));
            }
            CK(hipEventRecord(b1, st[1]));
            CK(hipDeviceSynchronize());
            float ta = 0, tb = 0;
            CK(hipEventElapsedTime(&ta, a0, a1));
            CK(hipEventElapsedTime(&tb, a0, b1));
            if (rep)
                std::printf("%-34s wgs=%5d  H2D %7.2f GB/s (%.1f ms)  D2H %7.2f GB/s (%.1f ms)  both %7.2f GB/s\n", name,
                            wgs, nh / (ta * 1e-3) / 1e9, ta, nd / (tb * 1e-3) / 1e9, tb,
                            (nh + nd) / (std::max(ta, tb) * 1e-3) / 1e9);
            CK(hipEventDestroy(a0));
            CK(hipEventDestroy(a1));
            CK(hipEventDestroy(b1));
        }
    };
    mix("mix 5:1 copy engines", false, false, 2048);
    for (int wgs : {512, 1024, 2048, 4096}) mix("mix 5:1 kernels", true, true, wgs);
    mix("mix 5:1 kernel H2D + engine D2H", true, false, 2048);
    // H2D alone by a kernel
    for (int wgs : {1024, 4096}) {
        for (int rep = 0; rep < 2; ++rep) {
            CK(hipDeviceSynchronize());
            const double t0 = now();
            hipLaunchKernelGGL(kcopy<4>, dim3(wgs), dim3(256), 0, st[0], (const uint4 *)hd, (uint4 *)d, total / 16);
            CK(hipStreamSynchronize(st[0]));
            const double el = now() - t0;
            if (rep) std::printf("%-34s wgs=%5d  %7.2f GB/s\n", "H2D kernel (zero-copy loads)", wgs, total / el / 1e9);
        }
    }
    return 0;
}
