// ctx.h — internal: the rsgpu_ctx behind the opaque handle of include/rsgpu.h
// (coding matrix, inverse/plan caches, staging slots, batch pipeline).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/rsgpu.h"
#include "gf256.h"
#include "gf_apply.h"

namespace rsgpu {


// One staging slot for the host-memory API: pinned host image + device image
// of an object laid out [row][pitch], a stream and a mismatch flag.
struct Slot {
    uint8_t *h = nullptr, *d = nullptr;
    uint8_t *hdev = nullptr;  // device address of the pinned staging image h
    size_t cap = 0;
    hipStream_t stream = nullptr;
#ifdef RSGPU_MEASURE_DMA_SPLIT
    // a second stream (and its event) for the copy-engine share of a split
    // per-object call (rsgpu.cpp run_host_once; measurement builds only)
    hipStream_t stream2 = nullptr;
    hipEvent_t ev2 = nullptr;
#endif
    uint32_t *d_bad = nullptr, *h_bad = nullptr;
    uint32_t *m_bad = nullptr;  // device address of h_bad (mapped pinned memory)
    ~Slot() {
#ifdef RSGPU_MEASURE_DMA_SPLIT
        if (ev2) (void)hipEventDestroy(ev2);
        if (stream2) (void)hipStreamDestroy(stream2);
#endif
        if (stream) (void)hipStreamDestroy(stream);
        retire(h, true, cap);
        retire(d, false, cap);
        retire(d_bad, false, 4);
        retire(h_bad, true, 4);
    }
};

inline size_t round_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// Staged image bytes (rows x shard length) above which the host calls code
// one object in column slabs (rsgpu.cpp run_host; the batch pipelines hand
// such objects to it).  Read once: RSGPU_SLAB_BYTES at the first call, or
// rsgpu_set_slab_bytes (tests) — no getenv on the call path (a
// per-call getenv raced with setenv from other threads).
constexpr size_t kSlabDefault = (size_t)1 << 30;
inline std::atomic<size_t> &slab_setting() {
    static std::atomic<size_t> v{[] {
        const char *e = std::getenv("RSGPU_SLAB_BYTES");
        const long long b = e ? std::atoll(e) : 0;
        return b >= 4096 ? (size_t)b : kSlabDefault;
    }()};
    return v;
}
inline size_t slab_bytes() { return slab_setting().load(std::memory_order_relaxed); }

// Pinned host memory that kernels read and write in place over PCIe (the
// Split images of rsgpu_host_alloc, the stream path's staging images):
// Mapped | Coherent, the kind the resident worker's mailboxes always used.
// hipHostMallocDefault — the kind the round-3 probe faulted on
// — only with RSGPU_HOST_ALLOC=default (read once).
inline unsigned host_image_flags() {
    static const unsigned f = [] {
        const char *e = std::getenv("RSGPU_HOST_ALLOC");
        return e && std::strcmp(e, "default") == 0 ? (unsigned)hipHostMallocDefault
                                                   : (unsigned)(hipHostMallocMapped | hipHostMallocCoherent);
    }();
    return f;
}

inline bool debug_on() {
    static const bool on = std::getenv("RSGPU_DEBUG") != nullptr;
    return on;
}

inline int hip_fail(hipError_t e, const char *what) {
    if (debug_on()) std::fprintf(stderr, "rsgpu: %s failed: %s\n", what, hipGetErrorString(e));
    return RSGPU_ERR_HIP;
}

#define HIP_TRY(expr)                                   \
    do {                                                \
        hipError_t e_ = (expr);                         \
        if (e_ != hipSuccess) return hip_fail(e_, #expr); \
    } while (0)

// Restores the calling thread's current device when an API call returns
// (rsgpu_ctx::use_device).
struct DeviceGuard {
    int prev = -1;
    DeviceGuard() = default;
    DeviceGuard(const DeviceGuard &) = delete;
    DeviceGuard &operator=(const DeviceGuard &) = delete;
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

// Batch pipeline (pipeline.cpp): a ring of device slots, one stream each, so
// H2D of object o+1 overlaps the kernel / D2H of object o.
struct PipeSlot {
    uint8_t *d = nullptr;
    size_t cap = 0;
    hipStream_t stream = nullptr;
    uint32_t *d_bad = nullptr;
    ~PipeSlot() {
        if (stream) (void)hipStreamDestroy(stream);
        retire(d, false, cap);
        retire(d_bad, false, 4);
    }
};

struct Pipeline {
    std::mutex mu;  // one batch at a time per context
    std::vector<std::unique_ptr<PipeSlot>> slots;
    uint32_t *h_bad = nullptr;  // pinned, one flag per object of the batch
    size_t h_bad_cap = 0;
    ~Pipeline() { retire(h_bad, true); }
};

// Device atlas of every erasure pattern of one operation (gf_masked.h),
// built and uploaded on the first *_dev_masks call, then immutable.  The
// host part is built once per code: a multi-device context's per-GPU
// sub-contexts share their parent's (rsgpu_ctx::atlas_host); each uploads
// its own device copy.  A failed upload (e.g. HBM momentarily exhausted)
// frees what it allocated and is retried by the next call.
struct Atlas {
    std::once_flag host_once;  // host build (no device needed)
    int host_err = 0;
    std::mutex dev_mu;         // guards the upload below
    bool dev_done = false;
    int32_t *d_pat = nullptr;
    void *d_recs = nullptr;
    uint32_t *d_tabs = nullptr;
    std::vector<int32_t> h_pat;   // pattern table, kept (host-flag calls validate with it)
    std::vector<uint8_t> h_recs;  // PatRec image (freed after the upload unless shared)
    std::vector<uint32_t> h_tabs; // kernel tables (freed after the upload unless shared)
    AtlasView view;
    void free_dev() {
        retire(d_pat, false);
        retire(d_recs, false);
        retire(d_tabs, false);
        d_pat = nullptr;
        d_recs = nullptr;
        d_tabs = nullptr;
    }
    ~Atlas() { free_dev(); }
};
// Estimated bytes of an atlas's kernel tables (before building it): the
// host-flag *_dev_multi calls take the atlas path only below a modest size
// and keep the host-planned path for codes whose atlas would be large.
size_t atlas_estimate(int k, int p, bool check);
enum AtlasMode { kAtlasReconstruct = 0, kAtlasData = 1, kAtlasDecode = 2 };

// The resident per-object coder (gf_worker.hip, rsgpu_worker_start).
struct Worker;
constexpr int kWorkerDeclined = 1;  // worker_run: not served here, take the stream path

}  // namespace rsgpu

using namespace rsgpu;

struct rsgpu_ctx {
    rsgpu::Pipeline pipe;  // batch host API (pipeline.cpp)
    rsgpu::MultiWorkspace multi_ws;  // mixed-pattern device launches
    rsgpu::Atlas atlas[3];           // device-resolved patterns, per AtlasMode
    uint32_t *d_ctab = nullptr;      // [256][8] coefficient tables (gf_apply_lanes)
    std::mutex ctab_mu;              // guards the d_ctab upload (retried after a failure)
    rsgpu::StatusScratch scratch;    // multi-reporter status of the masked decode
    // rsgpu_worker_start (null: off).  `worker` owns it (starts, stops,
    // parks and stats; std::atomic_load / _store).  The per-object calls read
    // `worker_raw` inside a reader epoch (WorkerRef, gf_worker.hip): a stop
    // detaches the pointer, flips the epoch and waits for the readers counted
    // in the old one before it drops its reference, so a call never touches a
    // freed worker and no shared lock sits on the per-call path (the
    // shared_ptr atomics of the first round-4 build took libstdc++'s mutex
    // pool on every call: 16 callers' pairs/s halved, r04_lat_worker_1k_host.txt).
    std::shared_ptr<rsgpu::Worker> worker;
    std::atomic<rsgpu::Worker *> worker_raw{nullptr};
    std::atomic<uint32_t> worker_epoch{0};
    std::atomic<int32_t> worker_readers[2] = {};
    std::mutex worker_mu;            // starts and stops
    // Multi-device context (rsgpu_create_multi / RSGPU_ALL_DEVICES): one
    // single-device context per entry of the device list.  Per-object calls
    // go round-robin, batch calls split objects o -> entry o mod N and run the
    // entries in parallel, device-resident calls go to an entry that owns the
    // memory (round-robin when a device is listed more than once: each entry
    // has its own streams, staging slots and pipeline).
    std::vector<std::unique_ptr<rsgpu_ctx>> subs;
    rsgpu_ctx *parent = nullptr;      // a sub-context's multi-device context (shared host atlas)
    std::atomic<unsigned> rr{0};
    std::atomic<uint64_t> calls{0};   // compute calls that reached this (sub-)context's device
    bool multi() const { return !subs.empty(); }
    rsgpu_ctx *pick() { return subs[rr.fetch_add(1, std::memory_order_relaxed) % subs.size()].get(); }
    rsgpu_ctx *sub_for(const void *dev_ptr);  // rsgpu.cpp; nullptr: not memory of one of our devices
    ~rsgpu_ctx() { retire(d_ctab, false); }
    int k = 0, p = 0, n = 0;
    unsigned kind = 0;
    int device = 0;
    std::vector<uint8_t> m;  // n x k coding matrix

    std::mutex mu;  // guards everything below
    std::map<std::string, std::vector<uint8_t>> inverses;  // survivors -> k x k inverse
    std::map<std::string, std::shared_ptr<Plan>> plans;
    std::vector<std::unique_ptr<Slot>> free_slots;
    int dev_state = 0;  // 0 unknown, 1 ok, <0 error code
    static constexpr size_t kMaxCached = 8192;  // plans / inverses kept per context

    const uint8_t *row(int r) const { return &m[(size_t)r * k]; }

    // ---- device bring-up (lazy).  Every call makes ctx->device current for
    // its own duration and gives the calling thread its previous device back
    // on return (the guard), so a process driving several GPUs from one thread
    // never finds its current device switched under it.
    // compute = false: worker start / stop (not counted in `calls`)
    int use_device(DeviceGuard &g, bool compute = true) {
        {
            std::lock_guard<std::mutex> l(mu);
            if (dev_state == 0) dev_state = rsgpu_device_ok(device) ? 1 : RSGPU_ERR_NO_DEVICE;
            if (dev_state < 0) return dev_state;
        }
        if (compute) calls.fetch_add(1, std::memory_order_relaxed);
        int cur = -1;
        HIP_TRY(hipGetDevice(&cur));
        if (cur != device) {
            HIP_TRY(hipSetDevice(device));
            g.prev = cur;
        }
        return RSGPU_OK;
    }

    // ---- survivors' inverse (upstream inversionTree.GetInvertedMatrix /
    // InsertInvertedMatrix, keyed here by the survivor list, which is a
    // function of upstream's invalidIndices key)
    int inverse(const std::vector<int> &surv, std::vector<uint8_t> &inv) {
        std::string key(surv.begin(), surv.end());
        {
            std::lock_guard<std::mutex> g(mu);
            auto it = inverses.find(key);
            if (it != inverses.end()) { inv = it->second; return RSGPU_OK; }
        }
        std::vector<uint8_t> sub((size_t)k * k);
        for (int i = 0; i < k; ++i) std::memcpy(&sub[(size_t)i * k], row(surv[i]), k);
        inv.assign((size_t)k * k, 0);
        if (!gf_invert(sub.data(), k, inv.data())) return RSGPU_ERR_SINGULAR;
        std::lock_guard<std::mutex> g(mu);
        if (inverses.size() >= kMaxCached) inverses.clear();  // bound memory under random patterns
        inverses.emplace(key, inv);
        return RSGPU_OK;
    }

    std::shared_ptr<Plan> cached(const std::string &key) {
        std::lock_guard<std::mutex> g(mu);
        auto it = plans.find(key);
        return it == plans.end() ? nullptr : it->second;
    }
    std::shared_ptr<Plan> remember(const std::string &key, std::shared_ptr<Plan> p) {
        p->build_tables();
        std::lock_guard<std::mutex> g(mu);
        // bound memory: upstream's inversionTree keeps every pattern, but a
        // 256-shard code has far more patterns than are worth caching.  Plans
        // are shared_ptr, so launches holding one keep it alive.
        if (plans.size() >= kMaxCached) plans.clear();
        return plans.emplace(key, std::move(p)).first->second;
    }

    // Encode: rows [k, n) <- M[k:] x rows [0, k)
    std::shared_ptr<Plan> plan_encode() {
        if (auto p = cached("E")) return p;
        auto p = std::make_shared<Plan>();
        p->K = k; p->R = this->p; p->nw = this->p;
        for (int c = 0; c < k; ++c) p->in_rows.push_back(c);
        for (int r = k; r < n; ++r) {
            p->out_rows.push_back(r);
            p->coef.insert(p->coef.end(), row(r), row(r) + k);
        }
        return remember("E", p);
    }

    // Verify: check rows M[j] x data XOR parity_j == 0 for j in [k, n)
    std::shared_ptr<Plan> plan_verify() {
        if (auto p = cached("V")) return p;
        auto p = std::make_shared<Plan>();
        build_verify(*p);
        return remember("V", p);
    }

    // Reconstruct (upstream reconstruct()): survivors = first k present rows.
    // Missing data row i = inv[i] x survivors; missing parity row j =
    // (M[j] x inv) x survivors — the same bytes as upstream's second
    // codeSomeShards over the (reconstructed) data rows, in one pass.
    // With check = true (fused Client.decode), every present row beyond
    // the survivors becomes a check row (M[j] x inv) x survivors XOR row_j:
    // exactly the comparisons upstream's Verify-after-Reconstruct can fail;
    // the survivors' own comparisons are identities (M[V] x inv = I).
    // fast path for n <= 64: plans keyed by (mode, present bitmask)
    std::unordered_map<uint64_t, std::shared_ptr<Plan>> fast_plans[3];

    int plan_reconstruct(const uint8_t *present, bool data_only, bool check,
                         std::shared_ptr<Plan> &out) {
        const int mode = check ? 2 : (data_only ? 1 : 0);
        uint64_t mask = 0;
        if (n <= 64) {
            for (int i = 0; i < n; ++i)
                if (present[i]) mask |= 1ull << i;
            std::lock_guard<std::mutex> g(mu);
            auto it = fast_plans[mode].find(mask);
            if (it != fast_plans[mode].end()) {
                out = it->second;
                return RSGPU_OK;
            }
        }
        int e = plan_reconstruct_slow(present, data_only, check, out);
        if (e == RSGPU_OK && n <= 64) {
            std::lock_guard<std::mutex> g(mu);
            if (fast_plans[mode].size() >= kMaxCached) fast_plans[mode].clear();
            fast_plans[mode].emplace(mask, out);
        }
        return e;
    }

    int plan_reconstruct_slow(const uint8_t *present, bool data_only, bool check,
                              std::shared_ptr<Plan> &out) {
        std::string key = check ? "D" : (data_only ? "d" : "R");
        for (int i = 0; i < n; ++i) key.push_back(present[i] ? '1' : '0');
        if ((out = cached(key))) return RSGPU_OK;
        auto p = std::make_shared<Plan>();
        int e = build_reconstruct(present, data_only, check, *p);
        if (e) return e;
        out = remember(key, p);
        return RSGPU_OK;
    }

    // The plan of one erasure pattern (no caching of the plan itself; the
    // survivors' inverse goes through the inverse cache).  Tables not built.
    int build_reconstruct(const uint8_t *present, bool data_only, bool check, Plan &pl) {
        Plan *p = &pl;
        std::vector<int> surv, extra, miss;
        for (int i = 0; i < n; ++i) {
            if (present[i]) (surv.size() < (size_t)k ? surv : extra).push_back(i);
            else miss.push_back(i);
        }
        std::vector<uint8_t> inv;
        int e = inverse(surv, inv);
        if (e) return e;
        const GF &g = gf();
        p->in_rows = surv;
        if (check) p->in_rows.insert(p->in_rows.end(), extra.begin(), extra.end());
        p->K = (int)p->in_rows.size();
        // coefficient row over survivors for an arbitrary matrix row j
        auto over_surv = [&](int j, std::vector<uint8_t> &cr) {
            cr.assign(p->K, 0);
            if (j < k) {
                std::memcpy(cr.data(), &inv[(size_t)j * k], k);
                return;
            }
            for (int c = 0; c < k; ++c) {
                const uint8_t mj = row(j)[c];
                if (!mj) continue;
                for (int s = 0; s < k; ++s) cr[s] ^= g.mul(mj, inv[(size_t)c * k + s]);
            }
        };
        std::vector<uint8_t> cr;
        for (int i : miss) {
            if (data_only && i >= k) continue;
            over_surv(i, cr);
            p->out_rows.push_back(i);
            p->coef.insert(p->coef.end(), cr.begin(), cr.end());
        }
        p->nw = (int)p->out_rows.size();
        if (check) {
            for (size_t x = 0; x < extra.size(); ++x) {
                const int j = extra[x];
                if (j < k) continue;  // upstream Verify compares parity rows only
                over_surv(j, cr);
                cr[k + x] ^= 1;
                p->out_rows.push_back(-1);
                p->coef.insert(p->coef.end(), cr.begin(), cr.end());
            }
        }
        p->R = (int)p->out_rows.size();
        return RSGPU_OK;
    }

    // Verify's plan: check rows M[j] x data XOR parity_j (j in [k, n)),
    // tables not built
    void build_verify(Plan &p) {
        p.K = n; p.R = this->p; p.nw = 0;
        p.in_rows.clear(); p.out_rows.clear(); p.coef.clear();
        for (int c = 0; c < n; ++c) p.in_rows.push_back(c);
        for (int j = k; j < n; ++j) {
            p.out_rows.push_back(-1);
            for (int c = 0; c < n; ++c) p.coef.push_back(c < k ? row(j)[c] : (uint8_t)(c == j));
        }
    }

    // rsgpu.cpp: the atlas's host part (pattern table; no device needed), and
    // the uploaded atlas the kernels read
    int atlas_host(AtlasMode mode, const Atlas *&out);
    int atlas_view(AtlasMode mode, AtlasView &out);

    // ---- staging slots
    int get_slot(size_t bytes, std::unique_ptr<Slot> &s) {
        {
            std::lock_guard<std::mutex> g(mu);
            if (!free_slots.empty()) { s = std::move(free_slots.back()); free_slots.pop_back(); }
        }
        if (!s) {
            s.reset(new Slot());
            HIP_TRY(hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking));
            HIP_TRY(hipMalloc(&s->d_bad, 4));
            HIP_TRY(hipHostMalloc(&s->h_bad, 4, hipHostMallocMapped | hipHostMallocCoherent));
            HIP_TRY(hipHostGetDevicePointer((void **)&s->m_bad, s->h_bad, 0));
        }
        if (s->cap < bytes) {
            // the old images are retired (freed at once unless a worker kernel
            // is resident, devmem.cpp); growth at least 1.5x
            retire(s->h, true, s->cap);
            retire(s->d, false, s->cap);
            const size_t cap = round_up(std::max(bytes, s->cap + s->cap / 2), (size_t)1 << 20);
            s->h = nullptr; s->d = nullptr; s->hdev = nullptr; s->cap = 0;
            HIP_TRY(hipHostMalloc(&s->h, cap, host_image_flags()));
            HIP_TRY(hipHostGetDevicePointer((void **)&s->hdev, s->h, 0));
            HIP_TRY(hipMalloc(&s->d, cap));
            s->cap = cap;
            relieve_retired();  // (no lock held here) the kept bytes stay bounded
        }
        return RSGPU_OK;
    }
    void put_slot(std::unique_ptr<Slot> s) {
        std::lock_guard<std::mutex> g(mu);
        free_slots.push_back(std::move(s));
    }
};

namespace rsgpu {
// upstream checkShards(shards, nilok): size = first non-empty length
int check_shards(const size_t *lens, int n, bool nilok, size_t *size);
// true if [p, p+len) lies in one range pinned through rsgpu_host_register /
// rsgpu_host_alloc (pipeline.cpp): the per-object host API then DMAs
// straight from / to it instead of staging through its own pinned buffer
bool host_pinned(const void *p, size_t len);
// the device address of such a range (kernels read/write it over PCIe), or
// nullptr when [p, p+len) is not inside one pinned range
void *host_device_ptr(const void *p, size_t len);
// One object through the resident worker (gf_worker.hip): rows[0..n) the
// object's shards (every one a buffer of S bytes; missing ones receive their
// reconstruction), mask the present rows (reconstruct / decode).  RSGPU_OK
// with *bad = 0 / 1 (a check failed), kWorkerDeclined (no worker, too large,
// every mailbox busy: the caller takes the stream path) or an error.
int worker_run(rsgpu_ctx *ctx, uint32_t op, size_t S, uint32_t mask, uint8_t *const *rows, uint32_t *bad);
// Runs fn with every worker of the process parked: calls in flight finish,
// each resident kernel leaves, later calls take the stream path until fn
// returns (the next one relaunches).  For runtime calls that synchronise the
// device on behalf of the user (rsgpu_host_free / _unregister): they then
// return at once instead of waiting for the workers to idle out.
int with_workers_parked(const std::function<int()> &fn);
}  // namespace rsgpu
