// hostcopy_check.cpp — stress check of the host copy pool (hostcopy.cpp),
// built by tests/test_hostcopy.py under ThreadSanitizer and under ASan/UBSan.
//
// Several caller threads issue copy_rows batches at once (as concurrent
// per-object calls on pageable buffers do, rsgpu.cpp run_host): sizes on both
// sides of the 12 MiB pool threshold, ragged row lengths, empty rows and
// empty batches.  Every destination byte is checked against its source and
// the guard bytes around each row must stay untouched.
//
// usage: hostcopy_check <callers> <batches per caller> <seed>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

#include "devmem.h"

namespace {

constexpr size_t kGuard = 64;
constexpr uint8_t kGuardByte = 0xA5;

int one_caller(int id, int batches, uint64_t seed) {
    std::mt19937_64 rng(seed * 1000003u + (uint64_t)id);
    for (int b = 0; b < batches; ++b) {
        const size_t nrows = rng() % 15;  // 0 .. 14 rows (RS(10+4) at most)
        // half the batches total past the pool threshold (12 MiB)
        const bool big = rng() & 1;
        std::vector<size_t> len(nrows);
        for (auto &l : len) {
            l = big ? (size_t)(1 << 20) + rng() % (3u << 20) : rng() % (64u << 10);
            if (rng() % 8 == 0) l = 0;
            if (rng() % 4 == 0) l |= 1;  // odd lengths: pieces end mid-word
        }
        std::vector<std::vector<uint8_t>> src(nrows), dst(nrows);
        std::vector<rsgpu::CopyJob> jobs(nrows);
        for (size_t r = 0; r < nrows; ++r) {
            src[r].resize(len[r]);
            dst[r].assign(len[r] + 2 * kGuard, kGuardByte);
            uint64_t x = rng();
            for (size_t i = 0; i < len[r]; ++i) {
                x = x * 6364136223846793005ull + 1442695040888963407ull;
                src[r][i] = (uint8_t)(x >> 56);
            }
            jobs[r] = {dst[r].data() + kGuard, src[r].data(), len[r]};
        }
        rsgpu::copy_rows(jobs.data(), nrows);
        for (size_t r = 0; r < nrows; ++r) {
            if (len[r] && std::memcmp(dst[r].data() + kGuard, src[r].data(), len[r]) != 0) {
                std::fprintf(stderr, "caller %d batch %d row %zu (%zu B): bytes differ\n", id, b, r, len[r]);
                return 1;
            }
            for (size_t i = 0; i < kGuard; ++i)
                if (dst[r][i] != kGuardByte || dst[r][kGuard + len[r] + i] != kGuardByte) {
                    std::fprintf(stderr, "caller %d batch %d row %zu: guard byte overwritten\n", id, b, r);
                    return 1;
                }
        }
    }
    return 0;
}

}  // namespace

int main(int argc, char **argv) {
    const int callers = argc > 1 ? std::atoi(argv[1]) : 4;
    const int batches = argc > 2 ? std::atoi(argv[2]) : 20;
    const uint64_t seed = argc > 3 ? std::strtoull(argv[3], nullptr, 10) : 1;
    std::vector<int> rc(callers, 0);
    std::vector<std::thread> th;
    for (int c = 0; c < callers; ++c) th.emplace_back([&, c] { rc[c] = one_caller(c, batches, seed); });
    for (auto &t : th) t.join();
    int bad = 0;
    for (int r : rc) bad |= r;
    if (!bad) std::printf("hostcopy_check: %d callers x %d batches ok\n", callers, batches);
    return bad;
}
