// pcie_bench.hip — host<->device copy rates on the MI355X box, in the shapes
// the batch pipeline (infinicache_amd/csrc/pipeline.cpp) issues:
//   1D pinned copies of various sizes, 1..4 streams;
//   2D copies repacking Split rows (pitch S = 104,858) to the 256-B device
//   pitch (104,960) — the encode H2D of a 1 MiB RS(10+2) object;
//   H2D and D2H at the same time (the pipeline's steady state).
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
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
    return 0;
}
