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
//   * retire(): the library's frees.  A free runs at once unless a worker
//     kernel is RESIDENT (launched and not finished: the probe gf_worker.hip
//     registers asks each started worker's stream); only then is the buffer
//     kept, and what was kept goes with the next free, relaunch, park or stop
//     that finds no kernel resident (round 4 held every free while
//     any worker was merely started, idle or not).  The lock is held across
//     the frees and across every worker launch (launch_guarded), so no kernel
//     is launched while a free that may synchronise is running.
//   * the bound: past kKeptCap bytes kept, a user free (rsgpu_host_free) and
//     the library's own safe points (relieve_retired: after a staging buffer
//     grew, at rsgpu_destroy — no lock of the library held) park the workers,
//     whose kernels then leave, and free everything kept.
//   * upload(): host -> device copies of tables and statuses, as
//     hipMemcpyAsync on a per-device non-blocking stream and a wait on that
//     stream alone (never the null stream).
#include <hip/hip_runtime.h>

#include <mutex>
#include <vector>

#include "ctx.h"

namespace rsgpu {

namespace {

struct Kept {
    void *p;
    bool host;
    size_t bytes;
};

struct Graveyard {
    std::mutex mu;
    int live = 0;  // workers started and not yet stopped, every device
    bool (*resident)() = nullptr;  // some worker kernel may be resident (gf_worker.hip)
    std::vector<Kept> kept;
    size_t kept_bytes = 0;
    uint64_t deferred = 0;  // frees ever deferred (diagnostics)
};

Graveyard &graveyard() {
    static Graveyard *g = new Graveyard();  // never destroyed: used from atexit handlers
    return *g;
}

void free_now(void *p, bool host) {
    if (host) (void)hipHostFree(p);
    else (void)hipFree(p);
}

size_t alloc_bytes(void *p) {
    size_t sz = 0;
    if (hipMemPtrGetInfo(p, &sz) == hipSuccess && sz) return sz;
    void *base = nullptr;
    sz = 0;
    return hipMemGetAddressRange(&base, &sz, p) == hipSuccess ? sz : 0;
}

// g.mu held
bool any_resident(Graveyard &g) { return g.live > 0 && (!g.resident || g.resident()); }

// g.mu held
void free_kept(Graveyard &g) {
    for (auto &k : g.kept) free_now(k.p, k.host);
    g.kept.clear();
    g.kept_bytes = 0;
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

void set_resident_probe(bool (*probe)()) {
    Graveyard &g = graveyard();
    std::lock_guard<std::mutex> l(g.mu);
    g.resident = probe;
}

void retire(void *p, bool host, size_t bytes) {
    if (!p) return;
    Graveyard &g = graveyard();
    std::lock_guard<std::mutex> l(g.mu);
    if (any_resident(g)) {
        const size_t b = bytes ? bytes : alloc_bytes(p);
        g.kept.push_back({p, host, b});
        g.kept_bytes += b;
        ++g.deferred;
        return;
    }
    free_kept(g);
    free_now(p, host);
}

int free_user(void *p, bool host, size_t bytes) {
    Graveyard &g = graveyard();
    {
        std::lock_guard<std::mutex> l(g.mu);
        if (!any_resident(g)) {
            free_kept(g);
            if (host) return hipHostFree(p) == hipSuccess ? RSGPU_OK : RSGPU_ERR_HIP;
            return hipFree(p) == hipSuccess ? RSGPU_OK : RSGPU_ERR_HIP;
        }
        if (g.kept_bytes < kKeptCap) {
            const size_t b = bytes ? bytes : alloc_bytes(p);
            g.kept.push_back({p, host, b});
            g.kept_bytes += b;
            ++g.deferred;
            return RSGPU_OK;
        }
    }
    // past the bound: park every worker (their kernels leave), free this
    // buffer; the park drains what was kept (with_workers_parked)
    return with_workers_parked([p, host] {
        const hipError_t e = host ? hipHostFree(p) : hipFree(p);
        return e == hipSuccess ? RSGPU_OK : hip_fail(e, "rsgpu_host_free");
    });
}

void relieve_retired() {
    {
        Graveyard &g = graveyard();
        std::lock_guard<std::mutex> l(g.mu);
        if (g.kept_bytes < kKeptCap) return;
        if (!any_resident(g)) {
            free_kept(g);
            return;
        }
    }
    // the kernels leave, the park drains what was kept
    (void)with_workers_parked([] { return RSGPU_OK; });
}

int device_sync_call(const std::function<int()> &fn) {
    Graveyard &g = graveyard();
    {
        std::lock_guard<std::mutex> l(g.mu);
        if (!any_resident(g)) {  // no kernel to wait for: no launch can start meanwhile
            free_kept(g);
            return fn();
        }
    }
    return with_workers_parked(fn);
}

hipError_t launch_guarded(const std::function<hipError_t()> &launch) {
    Graveyard &g = graveyard();
    std::lock_guard<std::mutex> l(g.mu);
    if (!g.kept.empty() && !any_resident(g)) free_kept(g);
    return launch();
}

void worker_count(int delta) {
    Graveyard &g = graveyard();
    std::lock_guard<std::mutex> l(g.mu);
    g.live += delta;
    if (g.live < 0) g.live = 0;
    if (!any_resident(g)) free_kept(g);
}

void drain_retired() {
    Graveyard &g = graveyard();
    std::lock_guard<std::mutex> l(g.mu);
    free_kept(g);
}

void retired_stats(size_t *count, size_t *bytes, uint64_t *deferred) {
    Graveyard &g = graveyard();
    std::lock_guard<std::mutex> l(g.mu);
    if (count) *count = g.kept.size();
    if (bytes) *bytes = g.kept_bytes;
    if (deferred) *deferred = g.deferred;
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

extern "C" int rsgpu_retired_stats(size_t *count, size_t *bytes, uint64_t *deferred) {
    rsgpu::retired_stats(count, bytes, deferred);
    return RSGPU_OK;
}
