// pipeline.cpp — batched host-memory API: the path "starts and ends in host
// memory" (the proxy socket buffer on Set, the gathered shard buffers on Get,
// /root/reference/client/ecRedis.go:96 and :161-173), so a batch of objects is
// streamed through the GPU as H2D -> gf_apply -> D2H over a ring of device
// slots, one HIP stream per slot: the copy of object o+1 overlaps the kernel
// and the copy-back of object o, and H2D / D2H use the two DMA directions.
//
//   rsgpu_encode_batch : Split-layout objects (rows contiguous, pitch = S as
//                        produced by Split, ecRedis.go:384) -> parity in place
//   rsgpu_decode_batch : per-object shard tables as gathered by EcGet
//                        (12 separate buffers, ecRedis.go:161-170) -> missing
//                        shards written, Verify-after-Reconstruct result
//
// (Batches of pinned Split objects coded in place over PCIe, as the
// per-object API does, ran at the same rate: 40.4-41.9 vs 40.3-41.2 GiB/s on
// the config-5 trace, same box; the DMA pipeline is kept, it leaves the CUs
// free while the copies run.)
//
// PCIe copies are always 1D (tools/pcie_bench.hip on MI355X: a pinned 1D
// H2D runs at 53-57 GB/s, a 2D host<->device copy with 105-KB rows at
// 8.7 GB/s).  The device image of an object is byte-packed (pitch = S, any
// S; the pass's packed mode, gf_device.h store_row), so a Split-layout object
// is one H2D and its parity one D2H, with no device-side repack.  Host
// buffers should be pinned (rsgpu_host_register / _alloc) for the copies to
// run async.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <limits>
#include <map>
#include <mutex>
#include <thread>
#include <vector>

#include "ctx.h"

namespace {

constexpr int kSlots = 4;
// slots in the ring (RSGPU_PIPE_SLOTS overrides, measurement only)
int pipe_slots() {
    static const int n = [] {
        const char *e = std::getenv("RSGPU_PIPE_SLOTS");
        const int v = e ? std::atoi(e) : kSlots;
        return v >= 1 && v <= 16 ? v : kSlots;
    }();
    return n;
}

// Adjacent small objects share one H2D (16 MiB groups; RSGPU_PIPE_GROUP=
// <bytes> overrides, 0 = off; read once).  A copy command carries a fixed
// ≈14 us (tools/pcie_bench: back-to-back 1 MiB H2D at 32 GB/s, 512 MiB at
// 57), so a batch of objects that lie back to back in host memory (Split
// images of one arena) moves its small ones — images up to kGroupObjMax — as
// one copy of their whole images, each then coded in place in the slot;
// written rows go back per object.  Config 5's trace: 42.47-42.64 -> 43.10-
// 43.14 GiB/s end to end (profiles/r05_trace_group/, same box, interleaved).
constexpr size_t kGroupObjMax = (size_t)4 << 20;
constexpr size_t kGroupDefault = (size_t)16 << 20;
size_t group_bytes() {
    static const size_t v = [] {
        const char *e = std::getenv("RSGPU_PIPE_GROUP");
        if (!e) return kGroupDefault;
        const long long b = std::atoll(e);
        return b > 0 ? (size_t)b : (size_t)0;
    }();
    return v;
}

// `piped` cut into groups [begin, end): objects adjacent in host memory
// (image o+1 starts where image o ends), each image at most kGroupObjMax,
// the span at most group_bytes(); single objects otherwise.  img(o) /
// base(o): an object's image bytes and first byte.  *slot_bytes grows to hold
// every group's span (+16 readable bytes).
struct Group {
    size_t begin, end, span;
};
template <class Img, class Base>
std::vector<Group> make_groups(const std::vector<int> &piped, Img img, Base base, size_t *slot_bytes) {
    std::vector<Group> out;
    const size_t G = group_bytes();
    for (size_t i = 0; i < piped.size();) {
        size_t j = i + 1, sp = G ? img(piped[i]) : 0;
        if (G && sp <= kGroupObjMax)
            while (j < piped.size()) {
                const int a = piped[j - 1], b = piped[j];
                if (img(b) > kGroupObjMax || sp + img(b) > G || base(b) != base(a) + img(a)) break;
                sp += img(b);
                ++j;
            }
        if (j - i > 1) *slot_bytes = std::max(*slot_bytes, sp + 16);
        out.push_back({i, j, sp});
        i = j;
    }
    return out;
}

// relieve_retired() for a scope, run when it ends: declared before the
// scope's lock_guard on ctx->pipe.mu, so it runs after the lock is released
// (relieve_retired may park every worker: no library lock may be held,
// devmem.h)
struct RelieveAfter {
    bool on = false;
    ~RelieveAfter() {
        if (on) relieve_retired();
    }
};

// *grew: a slot's buffer was replaced (the old one retired): the caller runs
// relieve_retired() once ctx->pipe.mu is released (RelieveAfter)
int ensure_slots(rsgpu_ctx *ctx, size_t bytes, bool *grew) {
    auto &P = ctx->pipe;
    while ((int)P.slots.size() < pipe_slots()) {
        std::unique_ptr<PipeSlot> s(new PipeSlot());
        HIP_TRY(hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking));
        HIP_TRY(hipMalloc(&s->d_bad, 4));
        P.slots.push_back(std::move(s));
    }
    for (auto &s : P.slots) {
        if (s->cap >= bytes) continue;
        HIP_TRY(hipStreamSynchronize(s->stream));
        retire(s->d, false, s->cap);  // (held while a worker kernel is resident: devmem.cpp)
        const size_t cap = round_up(std::max(bytes, s->cap + s->cap / 2), (size_t)1 << 20);
        s->d = nullptr;
        s->cap = 0;
        HIP_TRY(hipMalloc(&s->d, cap));
        s->cap = cap;
        *grew = true;  // the kept bytes stay bounded: relieve_retired, after the lock (devmem.cpp)
    }
    return RSGPU_OK;
}

int ensure_flags(rsgpu_ctx *ctx, int nobj) {
    auto &P = ctx->pipe;
    if (P.h_bad_cap >= (size_t)nobj) return RSGPU_OK;
    retire(P.h_bad, true, P.h_bad_cap * 4);
    const size_t cap = std::max<size_t>({(size_t)nobj, 1, P.h_bad_cap * 2});
    P.h_bad = nullptr;
    P.h_bad_cap = 0;
    HIP_TRY(hipHostMalloc(&P.h_bad, cap * 4, hipHostMallocDefault));
    P.h_bad_cap = cap;
    return RSGPU_OK;
}

// one object in a pipeline slot (capacity >= n*S + 16: readable slack)
Layout slack_layout(uint8_t *d, size_t pitch, size_t S) {
    Layout L{d, 0, pitch, S, 1};
    L.slack = true;
    return L;
}

int drain(rsgpu_ctx *ctx) {
    hipError_t first = hipSuccess;
    for (auto &s : ctx->pipe.slots) {
        hipError_t e = hipStreamSynchronize(s->stream);
        if (first == hipSuccess) first = e;
    }
    return first == hipSuccess ? RSGPU_OK : hip_fail(first, "pipeline drain");
}

// ranges pinned through this API: start -> (length, readable length, device
// address of start).  readable >= length: rsgpu_host_alloc's slack that
// kernels reading the range directly may over-read into (a row's last 16-B
// vector).
struct PinnedRange {
    size_t len, readable;
    uintptr_t dev;
};
std::mutex g_pin_mu;
std::map<uintptr_t, PinnedRange> g_pinned;

void pin_add(void *p, size_t len, size_t readable) {
    void *d = nullptr;
    if (hipHostGetDevicePointer(&d, p, 0) != hipSuccess) d = nullptr;
    std::lock_guard<std::mutex> g(g_pin_mu);
    g_pinned[(uintptr_t)p] = {len, readable, (uintptr_t)d};
}
// removes p's range; returns its readable length (0: p was not pinned here)
size_t pin_del(const void *p) {
    std::lock_guard<std::mutex> g(g_pin_mu);
    auto it = g_pinned.find((uintptr_t)p);
    if (it == g_pinned.end()) return 0;
    const size_t readable = it->second.readable;
    g_pinned.erase(it);
    return readable;
}

}  // namespace

namespace rsgpu {
bool host_pinned(const void *p, size_t len) {
    const uintptr_t a = (uintptr_t)p;
    std::lock_guard<std::mutex> g(g_pin_mu);
    auto it = g_pinned.upper_bound(a);
    if (it == g_pinned.begin()) return false;
    --it;
    return a >= it->first && a + len <= it->first + it->second.len;
}

void *host_device_ptr(const void *p, size_t len) {
    const uintptr_t a = (uintptr_t)p;
    std::lock_guard<std::mutex> g(g_pin_mu);
    auto it = g_pinned.upper_bound(a);
    if (it == g_pinned.begin()) return nullptr;
    --it;
    if (a < it->first || a + len > it->first + it->second.readable || !it->second.dev) return nullptr;
    return (void *)(it->second.dev + (a - it->first));
}
}  // namespace rsgpu

extern "C" {

int rsgpu_host_register(void *p, size_t len) {
    if (!p || !len) return RSGPU_ERR_INVALID_ARG;
    if (rsgpu_device_count() == 0) return RSGPU_ERR_NO_DEVICE;
    HIP_TRY(hipHostRegister(p, len, hipHostRegisterMapped));
    pin_add(p, len, len);
    return RSGPU_OK;
}

// hipHostUnregister / hipHostFree synchronise the device
// (profiles/r04_sync_probe*.txt): with a resident worker kernel they would
// wait until it idles out.  With no worker kernel resident they run at once
// (devmem.cpp holds off relaunches meanwhile); otherwise an unregister parks
// every worker around it (with_workers_parked: calls in flight finish, later
// ones take the stream path, the next one relaunches) and a free is deferred
// to the next moment no kernel is resident, up to kUserKeptCap bytes kept,
// past which it parks the workers too (a Go stagePool that frees
// on put no longer parks the workers on every free).
int rsgpu_host_unregister(void *p) {
    if (!p) return RSGPU_ERR_INVALID_ARG;
    pin_del(p);
    return device_sync_call([p] {
        HIP_TRY(hipHostUnregister(p));
        return RSGPU_OK;
    });
}

int rsgpu_host_alloc(size_t len, void **out) {
    if (!out || !len) return RSGPU_ERR_INVALID_ARG;
    *out = nullptr;
    if (rsgpu_device_count() == 0) return RSGPU_ERR_NO_DEVICE;
    // 64 B of slack past the caller's length: kernels may read a Split buffer
    // in place, and a row's last 16-B vector can run past the buffer's end.
    // Mapped | Coherent (host_image_flags, ctx.h; RSGPU_HOST_ALLOC=default
    // takes hipHostMallocDefault)
    HIP_TRY(hipHostMalloc(out, len + 64, host_image_flags()));
    pin_add(*out, len, len + 64);
    return RSGPU_OK;
}

int rsgpu_set_slab_bytes(size_t bytes) {
    slab_setting().store(bytes >= 4096 ? bytes : kSlabDefault, std::memory_order_relaxed);
    return RSGPU_OK;
}

int rsgpu_host_free(void *p) {
    if (!p) return RSGPU_OK;
    // the allocation's size from the pin table (the runtime's address-range
    // queries do not know every hipHostMalloc'd pointer): the kept-bytes bound
    // counts a held-back user free by it
    const size_t bytes = pin_del(p);
    return free_user(p, true, bytes);
}

}  // extern "C"

namespace {

// Multi-device batch: objects o -> device o mod N, each device's share run
// on its own host thread (its own pipeline, streams and PCIe link); returns
// the first error.
template <class F>
int split_devices(rsgpu_ctx *ctx, int nobj, F run) {
    const int N = (int)ctx->subs.size();
    std::vector<std::vector<int>> objs(N);
    for (int o = 0; o < nobj; ++o) objs[o % N].push_back(o);
    std::vector<int> err(N, RSGPU_OK);
    std::vector<std::thread> th;
    for (int d = 1; d < N; ++d)
        if (!objs[d].empty()) th.emplace_back([&, d] { err[d] = run(ctx->subs[d].get(), objs[d]); });
    if (!objs[0].empty()) err[0] = run(ctx->subs[0].get(), objs[0]);
    for (auto &t : th) t.join();
    for (int e : err)
        if (e) return e;
    return RSGPU_OK;
}

}  // namespace

extern "C" {

int rsgpu_encode_batch(rsgpu_ctx *ctx, uint8_t *const *objs, const size_t *shard_lens, int nobj) {
    if (!ctx || (nobj > 0 && (!objs || !shard_lens)) || nobj < 0) return RSGPU_ERR_INVALID_ARG;
    if (ctx->multi()) {
        for (int o = 0; o < nobj; ++o) {  // argument errors before any device work
            if (!objs[o]) return RSGPU_ERR_INVALID_ARG;
            if (shard_lens[o] == 0) return RSGPU_ERR_SHARD_NO_DATA;
        }
        return split_devices(ctx, nobj, [&](rsgpu_ctx *sub, const std::vector<int> &os) {
            std::vector<uint8_t *> o2;
            std::vector<size_t> l2;
            for (int o : os) {
                o2.push_back(objs[o]);
                l2.push_back(shard_lens[o]);
            }
            return rsgpu_encode_batch(sub, o2.data(), l2.data(), (int)os.size());
        });
    }
    const int k = ctx->k, p = ctx->p, n = ctx->n;
    // objects past the slab size go through the per-object host path (coded
    // in column slabs, rsgpu.cpp run_host), the rest through the pipeline
    const size_t lim = slab_bytes();
    std::vector<int> piped, big;
    size_t maxbytes = 0;
    for (int o = 0; o < nobj; ++o) {
        if (!objs[o]) return RSGPU_ERR_INVALID_ARG;
        if (shard_lens[o] == 0) return RSGPU_ERR_SHARD_NO_DATA;
        if ((size_t)n * shard_lens[o] + 16 > lim) {
            big.push_back(o);
            continue;
        }
        piped.push_back(o);
        maxbytes = std::max(maxbytes, (size_t)n * shard_lens[o] + 16);
    }
    if (nobj == 0) return RSGPU_OK;
    DeviceGuard dg_;
    int e = ctx->use_device(dg_);
    if (e) return e;
    for (int o : big)
        if ((e = rsgpu_encode_image(ctx, objs[o], shard_lens[o], n))) return e;
    if (piped.empty()) return RSGPU_OK;
    auto plan = ctx->plan_encode();
    auto img = [&](int o) { return (size_t)n * shard_lens[o]; };
    auto base = [&](int o) { return (const uint8_t *)objs[o]; };
    const std::vector<Group> groups = make_groups(piped, img, base, &maxbytes);
    RelieveAfter relieve;  // destroyed after g: runs with pipe.mu released
    std::lock_guard<std::mutex> g(ctx->pipe.mu);
    if ((e = ensure_slots(ctx, maxbytes, &relieve.on))) return e;
    hipError_t he = hipSuccess;
    for (size_t gi = 0; gi < groups.size() && he == hipSuccess; ++gi) {
        size_t q = groups[gi].begin;
        const size_t qe = groups[gi].end, span = groups[gi].span;
        PipeSlot &s = *ctx->pipe.slots[gi % pipe_slots()];
        // one object: its k data rows; a group: the whole images
        he = hipMemcpyAsync(s.d, objs[piped[q]], qe - q > 1 ? span : (size_t)k * shard_lens[piped[q]],
                            hipMemcpyHostToDevice, s.stream);
        for (size_t off = 0; q < qe && he == hipSuccess; ++q) {
            const int o = piped[q];
            const size_t S = shard_lens[o];
            Layout L{s.d + off, 0, S, S, 1};
            L.slack = true;  // slot capacity >= n*S + 16 past the image
            he = launch_plan(*plan, L, nullptr, s.stream);
            if (he == hipSuccess)
                he = hipMemcpyAsync(objs[o] + (size_t)k * S, s.d + off + (size_t)k * S, (size_t)p * S,
                                    hipMemcpyDeviceToHost, s.stream);
            off += (size_t)n * S;
        }
    }
    e = drain(ctx);
    if (he != hipSuccess) return hip_fail(he, "rsgpu_encode_batch");
    return e;
}

int rsgpu_decode_batch(rsgpu_ctx *ctx, uint8_t *const *shards, const uint8_t *present,
                       const size_t *shard_lens, int nobj, int *ok) {
    if (!ctx || nobj < 0 || (nobj > 0 && (!shards || !present || !shard_lens || !ok)))
        return RSGPU_ERR_INVALID_ARG;
    const int k = ctx->k, n = ctx->n;
    if (ctx->multi()) {
        for (int o = 0; o < nobj; ++o) {  // argument errors before any device work
            const uint8_t *pr = present + (size_t)o * n;
            int np = 0;
            for (int i = 0; i < n; ++i) np += pr[i] != 0;
            if (shard_lens[o] == 0) return RSGPU_ERR_SHARD_NO_DATA;
            if (np < k) return RSGPU_ERR_TOO_FEW_SHARDS;
            for (int i = 0; i < n; ++i)
                if (!shards[(size_t)o * n + i]) return RSGPU_ERR_INVALID_ARG;
        }
        return split_devices(ctx, nobj, [&](rsgpu_ctx *sub, const std::vector<int> &os) {
            std::vector<uint8_t *> s2;
            std::vector<uint8_t> p2;
            std::vector<size_t> l2;
            std::vector<int> ok2(os.size());
            for (int o : os) {
                s2.insert(s2.end(), shards + (size_t)o * n, shards + (size_t)(o + 1) * n);
                p2.insert(p2.end(), present + (size_t)o * n, present + (size_t)(o + 1) * n);
                l2.push_back(shard_lens[o]);
            }
            const int e = rsgpu_decode_batch(sub, s2.data(), p2.data(), l2.data(), (int)os.size(), ok2.data());
            for (size_t i = 0; i < os.size(); ++i) ok[os[i]] = ok2[i];
            return e;
        });
    }
    const size_t lim = slab_bytes();  // larger objects: per-object host path (encode_batch)
    std::vector<int> piped, big;
    size_t maxbytes = 0;
    std::vector<std::shared_ptr<Plan>> plans(nobj);
    for (int o = 0; o < nobj; ++o) {
        const uint8_t *pr = present + (size_t)o * n;
        int np = 0;
        for (int i = 0; i < n; ++i) np += pr[i] != 0;
        if (shard_lens[o] == 0) return RSGPU_ERR_SHARD_NO_DATA;
        if (np < k) return RSGPU_ERR_TOO_FEW_SHARDS;
        for (int i = 0; i < n; ++i)
            if (!shards[(size_t)o * n + i]) return RSGPU_ERR_INVALID_ARG;  // outputs need buffers
        int e = np == n ? (plans[o] = ctx->plan_verify(), RSGPU_OK)
                        : ctx->plan_reconstruct(pr, false, true, plans[o]);
        if (e) return e;
        if ((size_t)n * shard_lens[o] + 16 > lim) {
            big.push_back(o);
            continue;
        }
        piped.push_back(o);
        maxbytes = std::max(maxbytes, (size_t)n * shard_lens[o] + 16);
    }
    if (nobj == 0) return RSGPU_OK;
    DeviceGuard dg_;
    int e = ctx->use_device(dg_);
    if (e) return e;
    for (int o : big) {
        std::vector<size_t> lens(n);
        for (int i = 0; i < n; ++i) lens[i] = present[(size_t)o * n + i] ? shard_lens[o] : 0;
        if ((e = rsgpu_decode(ctx, shards + (size_t)o * n, lens.data(), n, &ok[o]))) return e;
    }
    if (piped.empty()) return RSGPU_OK;
    // grouping (RSGPU_PIPE_GROUP): objects whose shards form one Split image
    // each, back to back in host memory, and whose plans have no check rows
    // (a Get of exactly k bodies); the group's H2D carries every row, the
    // absent ones included (the pass overwrites them)
    auto split_image = [&](int o) {
        uint8_t *const *row = shards + (size_t)o * n;
        for (int i = 1; i < n; ++i)
            if (row[i] != row[0] + (size_t)i * shard_lens[o]) return false;
        return plans[o]->nw == plans[o]->R;
    };
    auto img = [&](int o) {
        return group_bytes() && split_image(o) ? (size_t)n * shard_lens[o] : std::numeric_limits<size_t>::max();
    };
    auto base = [&](int o) { return (const uint8_t *)shards[(size_t)o * n]; };
    const std::vector<Group> groups = make_groups(piped, img, base, &maxbytes);
    RelieveAfter relieve;  // destroyed after g: runs with pipe.mu released
    std::lock_guard<std::mutex> g(ctx->pipe.mu);
    if ((e = ensure_slots(ctx, maxbytes, &relieve.on))) return e;
    if ((e = ensure_flags(ctx, nobj))) return e;
    hipError_t he = hipSuccess;
    for (size_t gi = 0; gi < groups.size() && he == hipSuccess; ++gi) {
        size_t q = groups[gi].begin;
        const size_t qe = groups[gi].end, span = groups[gi].span;
        PipeSlot &s = *ctx->pipe.slots[gi % pipe_slots()];
        if (qe - q > 1) {
            he = hipMemcpyAsync(s.d, base(piped[q]), span, hipMemcpyHostToDevice, s.stream);
            for (size_t off = 0; q < qe && he == hipSuccess; ++q) {
                const int o = piped[q];
                Plan &plan = *plans[o];
                uint8_t *const *row = shards + (size_t)o * n;
                const size_t S = shard_lens[o];
                he = launch_plan(plan, slack_layout(s.d + off, S, S), nullptr, s.stream);
                for (int r = 0; r < plan.nw && he == hipSuccess;) {  // rebuilt rows, runs merged
                    const int r0 = plan.out_rows[r];
                    int m = 1;
                    while (r + m < plan.nw && plan.out_rows[r + m] == r0 + m) ++m;
                    he = hipMemcpyAsync(row[r0], s.d + off + (size_t)r0 * S, (size_t)m * S, hipMemcpyDeviceToHost,
                                        s.stream);
                    r += m;
                }
                ctx->pipe.h_bad[o] = 0;  // (no check rows)
                off += (size_t)n * S;
            }
            continue;
        }
        const int o = piped[q++];
        Plan &plan = *plans[o];
        uint8_t *const *row = shards + (size_t)o * n;
        const size_t S = shard_lens[o], P = S;  // packed rows
        const bool checks = plan.nw < plan.R;
        // rows that are neighbours both in the object and in host memory (a
        // Split image's) go as one copy: per-copy overhead is what a 10-row
        // Get of a small object spends its time on
        for (int c = 0; c < plan.K && he == hipSuccess;) {
            const int r0 = plan.in_rows[c];
            int m = 1;
            while (c + m < plan.K && plan.in_rows[c + m] == r0 + m && row[r0 + m] == row[r0] + (size_t)m * S) ++m;
            he = hipMemcpyAsync(s.d + (size_t)r0 * P, row[r0], (size_t)m * S, hipMemcpyHostToDevice, s.stream);
            c += m;
        }
        if (he == hipSuccess && checks) he = hipMemsetAsync(s.d_bad, 0, 4, s.stream);
        if (he == hipSuccess)
            he = launch_plan(plan, slack_layout(s.d, P, S), checks ? s.d_bad : nullptr, s.stream);
        for (int r = 0; r < plan.nw && he == hipSuccess;) {
            const int r0 = plan.out_rows[r];
            int m = 1;
            while (r + m < plan.nw && plan.out_rows[r + m] == r0 + m && row[r0 + m] == row[r0] + (size_t)m * S) ++m;
            he = hipMemcpyAsync(row[r0], s.d + (size_t)r0 * P, (size_t)m * S, hipMemcpyDeviceToHost, s.stream);
            r += m;
        }
        if (he == hipSuccess) {
            if (checks)
                he = hipMemcpyAsync(ctx->pipe.h_bad + o, s.d_bad, 4, hipMemcpyDeviceToHost, s.stream);
            else
                ctx->pipe.h_bad[o] = 0;
        }
    }
    e = drain(ctx);
    if (he != hipSuccess) return hip_fail(he, "rsgpu_decode_batch");
    if (e) return e;
    for (int o : piped) ok[o] = ctx->pipe.h_bad[o] == 0;
    return RSGPU_OK;
}

}  // extern "C"
