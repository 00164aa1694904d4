// devmem.h — frees and uploads that never wait for a resident worker kernel
// (devmem.cpp; the worker: gf_worker.hip).
#pragma once
#include <cstddef>

#include <hip/hip_runtime_api.h>

namespace rsgpu {

// hipFree (host = false) / hipHostFree (host = true) now, or, while a worker
// is started anywhere in the process, once the last one has stopped
void retire(void *p, bool host);
// workers started (+1) / stopped (-1); reaching zero frees what was retired
void worker_count(int delta);
size_t retired_pending();
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
