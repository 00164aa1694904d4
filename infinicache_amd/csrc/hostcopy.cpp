// hostcopy.cpp — host-to-host row copies of the per-object calls, spread over
// a small thread pool when they are large.
//
// A per-object call on pageable buffers (the Go Split array an EcSet passes,
// client/ecRedis.go:384) stages its rows through the slot's pinned image
// (rsgpu.cpp run_host): k*S bytes copied in, the written rows copied out.
// One thread copies ~30 GB/s of bytes moved, so past ~10 MiB objects the copy
// is most of the call (pageable 16 MiB fused encode+verify 939 us against
// 379 us from pinned memory, profiles/r04_worker_split/lats_*).  The pool
// splits such copies into 256 KiB pieces that its threads and the caller
// take in turn.  One batch runs at a time: a caller that finds the pool busy
// copies alone, so concurrent callers never wait for each other here.
// RSGPU_COPY_THREADS sets the pool size (0: no pool); default min(4, cores/2).
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "devmem.h"

namespace rsgpu {

namespace {

constexpr size_t kPiece = (size_t)256 << 10;
// below this one memcpy wins: a single thread copies a source still in its
// CCD's L3 faster than threads spread over several CCDs (pageable fused
// encode+verify, p50, 0 / 4 / 8 threads: 8 MiB objects 341 / 411 / 454 us,
// 16 MiB 775 / 685 / 607 us, 64 MiB 4,088 / 2,223 / 2,510 us;
// profiles/r04_copy_pool_*.txt)
constexpr size_t kMinParallel = (size_t)12 << 20;

struct Pool {
    std::mutex mu;
    std::condition_variable cv;       // workers: a new batch
    std::condition_variable done_cv;  // the caller: the batch is finished
    std::mutex busy;                  // one batch at a time (callers try_lock)
    std::vector<CopyJob> pieces;
    std::atomic<size_t> next{0}, remaining{0};
    uint64_t gen = 0;
    int active = 0;  // workers inside run() (mu): the next batch waits for 0 before touching `pieces`
    int nthreads = 0;

    void run() {
        for (;;) {
            const size_t i = next.fetch_add(1, std::memory_order_relaxed);
            if (i >= pieces.size()) return;
            std::memcpy(pieces[i].dst, pieces[i].src, pieces[i].len);
            if (remaining.fetch_sub(1, std::memory_order_acq_rel) == 1) {
                std::lock_guard<std::mutex> l(mu);
                done_cv.notify_all();
            }
        }
    }
    void worker() {
        uint64_t seen = 0;
        for (;;) {
            {
                std::unique_lock<std::mutex> l(mu);
                cv.wait(l, [&] { return gen != seen; });
                seen = gen;
                ++active;
            }
            run();
            {
                std::lock_guard<std::mutex> l(mu);
                --active;
            }
            done_cv.notify_all();
        }
    }
};

Pool *pool() {
    // never destroyed: its threads are detached and may be blocked in wait at exit
    static Pool *p = [] {
        Pool *q = new Pool();
        const char *e = std::getenv("RSGPU_COPY_THREADS");
        const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
        q->nthreads = e ? std::max(0, std::atoi(e)) : (int)std::min(4u, std::max(1u, hw / 2));
        for (int i = 0; i < q->nthreads; ++i) std::thread([q] { q->worker(); }).detach();
        return q;
    }();
    return p;
}

}  // namespace

void copy_rows(const CopyJob *jobs, size_t n) {
    size_t total = 0;
    for (size_t i = 0; i < n; ++i) total += jobs[i].len;
    Pool *p = total >= kMinParallel ? pool() : nullptr;
    if (!p || p->nthreads == 0 || !p->busy.try_lock()) {
        // empty rows may carry null pointers (memcpy's arguments must not be)
        for (size_t i = 0; i < n; ++i)
            if (jobs[i].len) std::memcpy(jobs[i].dst, jobs[i].src, jobs[i].len);
        return;
    }
    {
        // workers still leaving the previous batch's run() read `pieces`:
        // wait for them before rewriting it (a worker enters run() only
        // after seeing a new generation, under mu)
        std::unique_lock<std::mutex> l(p->mu);
        p->done_cv.wait(l, [&] { return p->active == 0; });
        p->pieces.clear();
        for (size_t i = 0; i < n; ++i)
            for (size_t o = 0; o < jobs[i].len; o += kPiece)
                p->pieces.push_back({(uint8_t *)jobs[i].dst + o, (const uint8_t *)jobs[i].src + o,
                                     std::min(kPiece, jobs[i].len - o)});
        p->remaining.store(p->pieces.size(), std::memory_order_relaxed);
        p->next.store(0, std::memory_order_relaxed);
        ++p->gen;
    }
    p->cv.notify_all();
    p->run();  // the caller copies too
    {
        std::unique_lock<std::mutex> l(p->mu);
        p->done_cv.wait(l, [&] { return p->remaining.load(std::memory_order_acquire) == 0; });
    }
    p->busy.unlock();
}

}  // namespace rsgpu
