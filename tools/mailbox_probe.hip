// mailbox_probe.hip — host <-> GPU round-trip latency of the transports a
// resident per-object worker could use (DESIGN.md §6 "Per-object latency").
//
//   ./mailbox_probe [iters]
//
// launch   : empty kernel launch + hipStreamSynchronize (the per-call floor of
//            the stream path)
// hostpoll : a resident kernel (one workgroup) polls a word in coherent
//            pinned host memory; per request it reads 10 rows of a 1 KiB
//            RS(10+2) object (S = 103) from pinned host memory over PCIe,
//            XORs them into 2 rows, stores those into host memory and
//            publishes the request's sequence number.  Variants: the flag
//            published by a system-scope release store, or by write-through
//            (sc0 sc1) row stores + vmcnt(0) + a plain system-scope store.
// devpoll  : the same with the doorbell in fine-grained device memory written
//            by the host through the BAR (only if the runtime reports a host
//            mapping for it).
// devdirect: doorbell AND the 10 input rows in fine-grained device memory,
//            written by the CPU through the device pointer itself (unified
//            addresses; a SIGSEGV on the first CPU touch means the runtime
//            gives the CPU no mapping, reported and skipped): the worker's
//            poll and row reads stay on the GPU side of PCIe.
// Every kernel has an exit every wave reaches: a stop word, and an idle
// limit on the device's real-time clock.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <csetjmp>
#include <csignal>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(1);                                                                      \
        }                                                                                      \
    } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

struct Mailbox {           // one cache line per direction
    uint32_t seq;          // host -> GPU doorbell (request number)
    uint32_t stop;
    uint32_t S, pad;
    uint64_t in, out;      // device addresses of the host rows
    uint32_t pad2[8];
    uint32_t resp;         // GPU -> host: last request done
    uint32_t pad3[15];
};

constexpr int kSys = 1 | 16;  // buffer-op cache policy: sc0 | sc1 (system coherent)

__device__ __forceinline__ uint32_t ld_sys(const uint32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint64_t ld_sys64(const uint64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// VARIANT 0: release store of the flag; 1: write-through rows + vmcnt(0) + relaxed flag
// Control flow that decides the loop must be wave-UNIFORM: with a divergent
// `if (t == 0) poll` the compiler's structurizer let lanes 1-63 of wave 0
// run the request loop again and again (barrier to barrier) while lane 0
// waited to poll: a kernel that never ends.  So the whole of wave 0 polls,
// every polled value goes through readfirstlane (scalar), and the request
// number reaches the other waves through LDS + readfirstlane.
// Round 4: the pointers and S the kernel rebuilds from
// the mailbox are recorded in mb->pad2 (system-scope stores, completed with
// vmcnt(0) before any row access, so they reach the host even if a row
// access then faults) and compared with the values the host passed as kernel
// arguments; on a mismatch the kernel flags it (pad2[6]) and answers the
// request without touching a row.
template <int VARIANT, int SLEEP>
__global__ __launch_bounds__(256) void worker(Mailbox *mb, uint32_t *bell, uint64_t idle_ticks, uint64_t want_in,
                                              uint64_t want_out, uint32_t want_S) {
    __shared__ uint32_t s_seq;
    const uint32_t t = threadIdx.x;
    uint32_t last = 0;
    if (t == 0) __hip_atomic_store(&mb->pad, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);  // started
    for (;;) {
        if (t < 64) {  // wave 0, all lanes: uniform loop
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            uint32_t s;
            for (;;) {
                s = __builtin_amdgcn_readfirstlane(ld_sys(bell));
                if (s != last) break;
                if (__builtin_amdgcn_readfirstlane(ld_sys(&mb->stop))) { s = 0xffffffffu; break; }
                if (__builtin_amdgcn_s_memrealtime() - t0 > idle_ticks) { s = 0xffffffffu; break; }
                if (SLEEP) __builtin_amdgcn_s_sleep(SLEEP);
            }
            if (t == 0) s_seq = s;
        }
        __syncthreads();
        const uint32_t s = __builtin_amdgcn_readfirstlane(s_seq);
        __syncthreads();
        if (s == 0xffffffffu) return;
        last = s;
        const uint32_t S = __builtin_amdgcn_readfirstlane(ld_sys(&mb->S));
        const uint64_t inp = ld_sys64(&mb->in), outp = ld_sys64(&mb->out);
        const uint8_t *in = (const uint8_t *)(((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(inp >> 32)) << 32) |
                                              __builtin_amdgcn_readfirstlane((uint32_t)inp));
        uint8_t *out = (uint8_t *)(((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(outp >> 32)) << 32) |
                                   __builtin_amdgcn_readfirstlane((uint32_t)outp));
        const uint32_t nvec = (S + 15) / 16;
        const bool same = (uint64_t)in == want_in && (uint64_t)out == want_out && S == want_S;
        if (t == 0) {
            uint32_t rec[7] = {S, (uint32_t)(uint64_t)in, (uint32_t)((uint64_t)in >> 32), (uint32_t)(uint64_t)out,
                               (uint32_t)((uint64_t)out >> 32), s, same ? 0u : 1u};
            for (int i = 0; i < 7; ++i) __hip_atomic_store(&mb->pad2[i], rec[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        if (!__syncthreads_and(same)) {  // never dereference a pointer the host did not pass
            if (t == 0) __hip_atomic_store(&mb->resp, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            continue;
        }
        const __amdgpu_buffer_rsrc_t ri = __builtin_amdgcn_make_buffer_rsrc((void *)in, (short)0, (int)(12 * S + 64), 0x00020000);
        const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc((void *)out, (short)0, (int)(2 * nvec * 16), 0x00020000);
        if (t < nvec) {
            u32x4 a = {0, 0, 0, 0}, b = {0, 0, 0, 0};
            u32x4 x[10];
#pragma unroll
            for (int c = 0; c < 10; ++c) x[c] = __builtin_amdgcn_raw_buffer_load_b128(ri, t * 16, c * S, kSys);
#pragma unroll
            for (int c = 0; c < 10; ++c) {
                a ^= x[c];
                if (c & 1) b ^= x[c];
            }
            // output rows at a 16-B padded pitch (whole-vector stores)
            __builtin_amdgcn_raw_buffer_store_b128(a, ro, t * 16, 0, VARIANT ? kSys : 0);
            __builtin_amdgcn_raw_buffer_store_b128(b, ro, t * 16, nvec * 16, VARIANT ? kSys : 0);
        }
        if (VARIANT) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (t == 0) {
            if (VARIANT)
                __hip_atomic_store(&mb->resp, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            else
                __hip_atomic_store(&mb->resp, s, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

__global__ void empty_kernel(int *p) {
    if (p && threadIdx.x == 1000) *p = 1;
}

static double pct(std::vector<double> v, double p) {
    std::sort(v.begin(), v.end());
    return v[(size_t)(p * (v.size() - 1) + 0.5)];
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static sigjmp_buf g_probe_jmp;
static void on_segv(int) { siglongjmp(g_probe_jmp, 1); }

// can the CPU store to (and load from) p?  A fault is caught and reported.
static bool cpu_can_touch(volatile uint32_t *p) {
    struct sigaction sa = {}, old_segv = {}, old_bus = {};
    sa.sa_handler = on_segv;
    sigaction(SIGSEGV, &sa, &old_segv);
    sigaction(SIGBUS, &sa, &old_bus);
    bool ok = false;
    if (sigsetjmp(g_probe_jmp, 1) == 0) {
        p[0] = 0x5a5a5a5au;
        ok = p[0] == 0x5a5a5a5au;
        p[0] = 0;
    }
    sigaction(SIGSEGV, &old_segv, nullptr);
    sigaction(SIGBUS, &old_bus, nullptr);
    return ok;
}

template <int VARIANT, int SLEEP>
static void run_direct(const char *name, int iters);

template <int VARIANT, int SLEEP>
static void run_poll(const char *name, bool devbell, int iters) {
    Mailbox *mb = nullptr, *dmb = nullptr;
    CK(hipHostMalloc((void **)&mb, sizeof(Mailbox), hipHostMallocMapped | hipHostMallocCoherent));
    std::memset(mb, 0, sizeof(Mailbox));
    CK(hipHostGetDevicePointer((void **)&dmb, mb, 0));
    uint32_t *bell_host = &mb->seq, *bell_dev = &dmb->seq;
    uint32_t *fg = nullptr;
    if (devbell) {
        hipError_t e = hipExtMallocWithFlags((void **)&fg, 4096, hipDeviceMallocFinegrained);
        if (e != hipSuccess) {
            std::printf("%s: hipExtMallocWithFlags(finegrained) failed: %s\n", name, hipGetErrorString(e));
            return;
        }
        hipPointerAttribute_t at;
        CK(hipPointerGetAttributes(&at, fg));
        std::printf("%s: finegrained device memory: type %d device %d hostPointer %p devicePointer %p\n", name,
                    (int)at.type, at.device, at.hostPointer, at.devicePointer);
        if (!at.hostPointer) {
            std::printf("%s: no host mapping reported: skipped\n", name);
            (void)hipFree(fg);
            return;
        }
        bell_host = (uint32_t *)at.hostPointer;
        bell_dev = fg;
        *(volatile uint32_t *)bell_host = 0;
    }
    const uint32_t S = 103;
    uint8_t *in = nullptr, *out = nullptr, *din = nullptr, *dout = nullptr;
    // PROBE_ROWS_COHERENT=1: the rows as the product worker's images
    // (Mapped | Coherent); default: hipHostMallocDefault (the r03 run)
    const unsigned rflags = std::getenv("PROBE_ROWS_COHERENT") ? (hipHostMallocMapped | hipHostMallocCoherent)
                                                               : hipHostMallocDefault;
    CK(hipHostMalloc((void **)&in, 12 * S + 64, rflags));
    CK(hipHostMalloc((void **)&out, 2 * 112 + 64, rflags));
    CK(hipHostGetDevicePointer((void **)&din, in, 0));
    CK(hipHostGetDevicePointer((void **)&dout, out, 0));
    for (int i = 0; i < 2; ++i) {
        hipPointerAttribute_t at;
        const void *hp = i ? (const void *)out : (const void *)in;
        CK(hipPointerGetAttributes(&at, hp));
        std::printf("%s: %s host %p device %p: type %d allocationFlags 0x%x isManaged %d\n", name, i ? "out" : "in",
                    hp, i ? (void *)dout : (void *)din, (int)at.type, at.allocationFlags, at.isManaged);
    }
    mb->S = S;
    mb->in = (uint64_t)din;
    mb->out = (uint64_t)dout;
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    std::printf("%s: launching\n", name);
    hipLaunchKernelGGL((worker<VARIANT, SLEEP>), dim3(1), dim3(256), 0, st, dmb, bell_dev, (uint64_t)200000000,
                       (uint64_t)din, (uint64_t)dout, S);  // 2 s idle
    CK(hipGetLastError());
    std::vector<double> lat;
    int bad = 0;
    uint8_t want[2][112];
    for (int it = 1; it <= iters; ++it) {
        for (uint32_t i = 0; i < 12 * S; ++i) in[i] = (uint8_t)(i * 7 + it * 13);
        for (uint32_t j = 0; j < S; ++j) {
            uint8_t a = 0, b = 0;
            for (int c = 0; c < 10; ++c) {
                a ^= in[c * S + j];
                if (c & 1) b ^= in[c * S + j];
            }
            want[0][j] = a;
            want[1][j] = b;
        }
        const double t0 = now_us();
        __atomic_store_n(bell_host, (uint32_t)it, __ATOMIC_RELEASE);
        while (__atomic_load_n(&mb->resp, __ATOMIC_ACQUIRE) != (uint32_t)it) {
            if (now_us() - t0 > 1e6) {
                std::printf("%s: no response after 1 s at request %d (kernel started: %u)\n", name, it,
                            __atomic_load_n(&mb->pad, __ATOMIC_ACQUIRE));
                std::printf("%s: kernel read S %u in 0x%08x%08x out 0x%08x%08x at request %u, mismatch %u "
                            "(host passed S %u in %p out %p)\n",
                            name, mb->pad2[0], mb->pad2[2], mb->pad2[1], mb->pad2[4], mb->pad2[3], mb->pad2[5],
                            mb->pad2[6], S, (void *)din, (void *)dout);
                mb->stop = 1;
                CK(hipStreamSynchronize(st));
                return;
            }
        }
        const double t1 = now_us();
        if (mb->pad2[6]) {
            std::printf("%s: request %d: the kernel read S %u in 0x%08x%08x out 0x%08x%08x, not what the host passed\n",
                        name, it, mb->pad2[0], mb->pad2[2], mb->pad2[1], mb->pad2[4], mb->pad2[3]);
            ++bad;
            mb->pad2[6] = 0;
        }
        if (std::memcmp(out, want[0], S) || std::memcmp(out + 112, want[1], S)) ++bad;
        lat.push_back(t1 - t0);
    }
    __atomic_store_n(&mb->stop, 1u, __ATOMIC_RELEASE);
    std::printf("%s: stop sent, waiting for the kernel\n", name);
    CK(hipStreamSynchronize(st));
    std::printf("%-34s p50 %6.2f us  p90 %6.2f  p99 %6.2f  min %6.2f  (%d iters, %d wrong)\n", name, pct(lat, 0.5),
                pct(lat, 0.9), pct(lat, 0.99), pct(lat, 0.0), iters, bad);
    CK(hipStreamDestroy(st));
    (void)hipHostFree(in);
    (void)hipHostFree(out);
    (void)hipHostFree(mb);
    if (fg) (void)hipFree(fg);
}

// devdirect: bell + input rows in fine-grained VRAM written by the CPU
template <int VARIANT, int SLEEP>
static void run_direct(const char *name, int iters) {
    Mailbox *mb = nullptr, *dmb = nullptr;
    CK(hipHostMalloc((void **)&mb, sizeof(Mailbox), hipHostMallocMapped | hipHostMallocCoherent));
    std::memset(mb, 0, sizeof(Mailbox));
    CK(hipHostGetDevicePointer((void **)&dmb, mb, 0));
    const uint32_t S = 103;
    uint8_t *vram = nullptr;
    hipError_t e = hipExtMallocWithFlags((void **)&vram, 1 << 16, hipDeviceMallocFinegrained);
    if (e != hipSuccess) {
        std::printf("%s: hipExtMallocWithFlags(finegrained) failed: %s\n", name, hipGetErrorString(e));
        return;
    }
    CK(hipMemset(vram, 0, 1 << 16));
    CK(hipDeviceSynchronize());
    if (!cpu_can_touch((volatile uint32_t *)vram)) {
        std::printf("%s: the CPU cannot access fine-grained device memory through its device pointer: skipped\n", name);
        (void)hipFree(vram);
        return;
    }
    std::printf("%s: CPU access to fine-grained device memory works\n", name);
    uint32_t *bell = (uint32_t *)vram;          // first 256 B: the doorbell line
    uint8_t *din = vram + 256;                  // input rows
    uint8_t *out = nullptr, *dout = nullptr;
    CK(hipHostMalloc((void **)&out, 2 * 112 + 64, hipHostMallocDefault));
    CK(hipHostGetDevicePointer((void **)&dout, out, 0));
    mb->S = S;
    mb->in = (uint64_t)din;
    mb->out = (uint64_t)dout;
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    hipLaunchKernelGGL((worker<VARIANT, SLEEP>), dim3(1), dim3(256), 0, st, dmb, bell, (uint64_t)200000000,
                       (uint64_t)din, (uint64_t)dout, S);
    CK(hipGetLastError());
    std::vector<double> lat, wr;
    int bad = 0;
    std::vector<uint8_t> in(12 * S + 64);
    uint8_t want[2][112];
    for (int it = 1; it <= iters; ++it) {
        for (uint32_t i = 0; i < 12 * S; ++i) in[i] = (uint8_t)(i * 7 + it * 13);
        for (uint32_t j = 0; j < S; ++j) {
            uint8_t a = 0, b = 0;
            for (int c = 0; c < 10; ++c) {
                a ^= in[c * S + j];
                if (c & 1) b ^= in[c * S + j];
            }
            want[0][j] = a;
            want[1][j] = b;
        }
        const double t0 = now_us();
        std::memcpy(din, in.data(), 10 * S + 16);  // the rows the worker reads (through the BAR)
        __atomic_thread_fence(__ATOMIC_SEQ_CST);    // rows land before the doorbell
        const double tw = now_us();
        __atomic_store_n(bell, (uint32_t)it, __ATOMIC_RELEASE);
        // the BAR mapping is write-combining: without a fence the doorbell
        // store waits in the CPU's WC buffer (first run: p50 2.96 ms)
        __atomic_thread_fence(__ATOMIC_SEQ_CST);
        while (__atomic_load_n(&mb->resp, __ATOMIC_ACQUIRE) != (uint32_t)it) {
            if (now_us() - t0 > 1e6) {
                std::printf("%s: no response after 1 s at request %d\n", name, it);
                mb->stop = 1;
                CK(hipStreamSynchronize(st));
                return;
            }
        }
        const double t1 = now_us();
        if (std::memcmp(out, want[0], S) || std::memcmp(out + 112, want[1], S)) ++bad;
        lat.push_back(t1 - t0);
        wr.push_back(tw - t0);
    }
    __atomic_store_n(&mb->stop, 1u, __ATOMIC_RELEASE);
    CK(hipStreamSynchronize(st));
    std::printf("%-34s p50 %6.2f us  p90 %6.2f  p99 %6.2f  min %6.2f  (%d iters, %d wrong; CPU row copy p50 %.2f us)\n",
                name, pct(lat, 0.5), pct(lat, 0.9), pct(lat, 0.99), pct(lat, 0.0), iters, bad, pct(wr, 0.5));
    CK(hipStreamDestroy(st));
    (void)hipHostFree(out);
    (void)hipHostFree(mb);
    (void)hipFree(vram);
}

int main(int argc, char **argv) {
    setvbuf(stdout, nullptr, _IONBF, 0);
    const int iters = argc > 1 ? std::atoi(argv[1]) : 2000;
    const int only = argc > 2 ? std::atoi(argv[2]) : -1;  // run one variant
    CK(hipSetDevice(0));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    {
        std::vector<double> lat;
        for (int i = 0; i < iters + 50; ++i) {
            const double t0 = now_us();
            hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, st, nullptr);
            CK(hipStreamSynchronize(st));
            if (i >= 50) lat.push_back(now_us() - t0);
        }
        std::printf("%-34s p50 %6.2f us  p90 %6.2f  p99 %6.2f  min %6.2f\n", "launch+sync (empty kernel)",
                    pct(lat, 0.5), pct(lat, 0.9), pct(lat, 0.99), pct(lat, 0.0));
    }
    if (only < 0 || only == 0) run_poll<0, 1>("hostpoll release-flag sleep1", false, iters);
    if (only < 0 || only == 1) run_poll<1, 1>("hostpoll wt-rows+flag sleep1", false, iters);
    if (only < 0 || only == 2) run_poll<1, 0>("hostpoll wt-rows+flag nosleep", false, iters);
    if (only < 0 || only == 3) run_poll<1, 4>("hostpoll wt-rows+flag sleep4", false, iters);
    if (only == 4) run_poll<1, 1>("devpoll wt-rows+flag sleep1", true, iters);
    if (only == 5) run_direct<1, 1>("devdirect wt-rows+flag sleep1", iters);
    return 0;
}
