// devmem.cpp — the runtime calls of the library that must not wait for a
// resident worker kernel (gf_worker.hip, rsgpu_worker_start).
//
// hipFree and hipHostFree synchronise the device: they return only once
// every stream of it is idle, the worker's stream included, and a null-stream
// hipMemcpy waits for every blocking stream (profiles/r04_sync_probe.txt).
// A resident worker leaves only after idle_us without requests, so a call
// that grew a staging buffer while other callers kept the worker busy waited
// for as long as that traffic lasted.
//
//   * retire(): the library's frees.  With no worker running anywhere in the
//     process the buffer is freed at once; otherwise it is kept and freed when
//     the last worker has stopped (its kernel has left: worker_count(-1)).
//     The growth paths that retire buffers grow geometrically, so what waits
//     here is bounded by a small multiple of the largest buffer in use.
//     The lock is held across the frees, so no worker starts (and no kernel
//     of one is launched) while a free that may synchronise is running.
//   * upload(): host -> device copies of tables and statuses, as
//     hipMemcpyAsync on a per-device non-blocking stream and a wait on that
//     stream alone (never the null stream).
#include <hip/hip_runtime.h>

#include <mutex>
#include <utility>
#include <vector>

#include "ctx.h"

namespace rsgpu {

namespace {

struct Graveyard {
    std::mutex mu;
    int live = 0;  // workers started and not yet stopped, every device
    std::vector<std::pair<void *, bool>> kept;  // (pointer, pinned host memory)
};

Graveyard &graveyard() {
    static Graveyard *g = new Graveyard();  // never destroyed: used from atexit handlers
    return *g;
}

void free_now(void *p, bool host) {
    if (host) (void)hipHostFree(p);
    else (void)hipFree(p);
}

constexpr int kMaxDevices = 64;
struct UploadStreams {
    std::mutex mu[kMaxDevices];
    hipStream_t st[kMaxDevices] = {};
};
UploadStreams &uploads() {
    static UploadStreams *u = new UploadStreams();
    return *u;
}

}  // namespace

void retire(void *p, bool host) {
    if (!p) return;
    Graveyard &g = graveyard();
    std::lock_guard<std::mutex> l(g.mu);
    if (g.live > 0) {
        g.kept.emplace_back(p, host);
        return;
    }
    free_now(p, host);
}

void worker_count(int delta) {
    Graveyard &g = graveyard();
    std::lock_guard<std::mutex> l(g.mu);
    g.live += delta;
    if (g.live > 0) return;
    g.live = 0;
    for (auto &k : g.kept) free_now(k.first, k.second);
    g.kept.clear();
}

void drain_retired() {
    Graveyard &g = graveyard();
    std::lock_guard<std::mutex> l(g.mu);
    for (auto &k : g.kept) free_now(k.first, k.second);
    g.kept.clear();
}

size_t retired_pending() {
    Graveyard &g = graveyard();
    std::lock_guard<std::mutex> l(g.mu);
    return g.kept.size();
}

hipError_t upload(void *dst, const void *src, size_t bytes) {
    if (!bytes) return hipSuccess;
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    if (dev < 0 || dev >= kMaxDevices) return hipErrorInvalidDevice;
    UploadStreams &u = uploads();
    std::lock_guard<std::mutex> l(u.mu[dev]);
    if (!u.st[dev]) {
        e = hipStreamCreateWithFlags(&u.st[dev], hipStreamNonBlocking);
        if (e != hipSuccess) {
            u.st[dev] = nullptr;
            return e;
        }
    }
    e = hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, u.st[dev]);
    const hipError_t s = hipStreamSynchronize(u.st[dev]);
    return e != hipSuccess ? e : s;
}

}  // namespace rsgpu
