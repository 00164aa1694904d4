// devmem.h — frees and uploads that never wait for a resident worker kernel
// (devmem.cpp; the worker: gf_worker.hip).
#pragma once
#include <cstddef>
#include <cstdint>
#include <functional>

#include <hip/hip_runtime_api.h>

namespace rsgpu {

// hipFree (host = false) / hipHostFree (host = true) now, or, while a worker
// kernel is resident, with the next free / launch / park / stop that finds
// none resident
// bytes: the allocation's size when the caller knows it (0: asked of the
// runtime, which may not know it), for the bound below
void retire(void *p, bool host, size_t bytes = 0);
// the bound on kept bytes: past it the workers are parked (their kernels
// leave) and everything kept is freed
constexpr size_t kKeptCap = (size_t)256 << 20;
// a user's free (rsgpu_host_free): as retire(), with the bound; bytes: the
// allocation's size when the caller knows it (0: asked of the runtime)
int free_user(void *p, bool host, size_t bytes = 0);
// the bound at the library's own safe points (no library lock held: it may
// park the workers)
void relieve_retired();
// a runtime call that synchronises the device on the user's behalf
// (hipHostUnregister): run at once when no worker kernel is resident, else
// with every worker parked (with_workers_parked)
int device_sync_call(const std::function<int()> &fn);
// the worker's probe: true when some started worker's kernel may be resident
void set_resident_probe(bool (*probe)());
// a worker launch, serialised with the frees (no kernel is launched while a
// free that may synchronise runs); what was kept is freed first when no
// kernel is resident
hipError_t launch_guarded(const std::function<hipError_t()> &launch);
// workers started (+1) / stopped (-1); frees what was kept when no kernel is resident
void worker_count(int delta);
// kept buffers now, their bytes, frees ever deferred
void retired_stats(size_t *count, size_t *bytes, uint64_t *deferred);
// frees everything retired (the caller guarantees no worker kernel is resident)
void drain_retired();
// host -> device copy on the current device's non-blocking upload stream;
// returns when the bytes have landed
hipError_t upload(void *dst, const void *src, size_t bytes);

// host memory copies of a per-object call's rows (hostcopy.cpp): large
// batches are spread over a small thread pool, small ones are one memcpy
struct CopyJob {
    void *dst;
    const void *src;
    size_t len;
};
void copy_rows(const CopyJob *jobs, size_t n);

}  // namespace rsgpu
