// gf_masked.hip — launchers of the device-resolved mixed-pattern passes
// (gf_masked.h): rsgpu_{decode,reconstruct}_dev_masks and the host-flag
// *_dev_multi calls for codes of <= 16 shards.  Launch policy (nt loads and
// stores, XCD-contiguous order, occupancy cap) as gf_kernels.hip.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "gf_apply.h"
#include "gf_launch.h"
#include "gf_masked.h"

namespace rsgpu {

namespace {

template <int KMAX, int R>
hipError_t launch_masked_t(const AtlasView &A, const Layout &L, const uint32_t *masks, uint32_t *status,
                           uint32_t *acc, uint32_t *cnt, hipStream_t st) {
    MaskedArgs a{};
    a.obj_stride = L.obj_stride;
    a.pat = A.pat;
    a.recs = (const PatRec *)A.recs;
    a.tabs = A.tabs;
    a.ctab = A.ctab;
    a.nmask = (uint32_t)((1ull << A.n) - 1);
    a.kfix = (uint32_t)A.kfix;
    a.nsub = (uint32_t)A.nsub;
    a.nvec = (uint32_t)((L.shard_len + 15) / 16);
    a.tail = (uint32_t)(L.shard_len - (size_t)(a.nvec - 1) * 16);
    a.pitch = (uint32_t)L.pitch;
    a.span = (uint32_t)((size_t)(A.n - 1) * L.pitch + (size_t)a.nvec * 16);
    a.nobj = (uint32_t)L.nobj;
    // occupancy cap for the common pattern (a healthy Get: k inputs, rows written)
    const unsigned cap = store_lds(A.kcap);
    // tuning knob (measurement only): workgroups per CU of the lanes kernel
    static const int lanes_w = [] {
        const char *e = std::getenv("RSGPU_LANES_WG");
        return e ? std::atoi(e) : 0;
    }();
    const unsigned lanes_cap = lanes_w > 0 ? 160u * 1024u / (unsigned)lanes_w - 256u : cap;
    // Short rows: a workgroup codes opw whole objects (gf_apply_lanes), all
    // lanes addressing them from the group's first object in one 32-bit range
    uint32_t opw = 1;
    if (a.nvec * 2 <= kBlock) {
        opw = kBlock / a.nvec;
        while (opw > 1 && (uint64_t)(opw - 1) * L.obj_stride + a.span >= 0x7fffffffull) opw /= 2;
    }
    for (int s = 0; s < A.nsub; ++s) {
        a.sub = (uint32_t)s;
        if (opw > 1) {
            a.opw = opw;
            a.gspan = (uint32_t)((uint64_t)(opw - 1) * L.obj_stride + a.span);
            constexpr unsigned stat = sizeof(u32x4) * 256 * 2 + 4 * 256;  // gf_apply_lanes' static LDS
            const unsigned dyn = lanes_cap > stat ? lanes_cap - stat : 0u;
            const size_t groups = ((size_t)L.nobj + opw - 1) / opw;
            for (size_t g0 = 0; g0 < groups; g0 += (size_t)max_items(1)) {
                const size_t ng = std::min((size_t)max_items(1), groups - g0);
                const size_t o0 = g0 * opw;
                a.base = L.base + o0 * L.obj_stride;
                a.masks = masks + o0;
                a.status = status ? status + o0 : nullptr;
                a.acc = acc ? acc + o0 : nullptr;
                a.cnt = cnt ? cnt + o0 : nullptr;
                a.nobj = (uint32_t)std::min<size_t>(ng * opw, (size_t)L.nobj - o0);
                unsigned grid;
                a.ord = make_order(1, (uint32_t)ng, (size_t)a.nobj * L.obj_stride, grid);
                hipLaunchKernelGGL((gf_apply_lanes<KMAX, R, kLoadAux, kStoreAux>), dim3(grid), dim3(kBlock), dyn, st, a);
                hipError_t e = hipGetLastError();
                if (e != hipSuccess) return e;
            }
            continue;
        }
        const unsigned gx = (a.nvec + kBlock - 1) / kBlock;
        const int step = max_items(gx);
        for (int o0 = 0; o0 < L.nobj; o0 += step) {
            const int no = std::min(step, L.nobj - o0);
            a.base = L.base + (size_t)o0 * L.obj_stride;
            a.masks = masks + o0;
            a.status = status ? status + o0 : nullptr;
            a.acc = acc ? acc + o0 : nullptr;
            a.cnt = cnt ? cnt + o0 : nullptr;
            a.opw = 1;
            a.gspan = 0;
            unsigned grid;
            a.ord = make_order(gx, (uint32_t)no, objs_span(L, no, a.span), grid);
            hipLaunchKernelGGL((gf_apply_masked<KMAX, R, kLoadAux, kStoreAux>), dim3(grid), dim3(kBlock), cap, st, a);
            hipError_t e = hipGetLastError();
            if (e != hipSuccess) return e;
        }
    }
    return hipSuccess;
}

typedef hipError_t (*masked_fn)(const AtlasView &, const Layout &, const uint32_t *, uint32_t *, uint32_t *,
                                uint32_t *, hipStream_t);

template <int K>
masked_fn pick_masked_r(int R) {
    return R == 1 ? &launch_masked_t<K, 1> : R == 2 ? &launch_masked_t<K, 2>
         : R == 3 ? &launch_masked_t<K, 3> : &launch_masked_t<K, 4>;
}

masked_fn pick_masked(int K, int R) {
    switch (K) {
#define RSGPU_K(k) case k: return pick_masked_r<k>(R);
        RSGPU_K(1) RSGPU_K(2) RSGPU_K(3) RSGPU_K(4) RSGPU_K(5) RSGPU_K(6) RSGPU_K(7) RSGPU_K(8)
        RSGPU_K(9) RSGPU_K(10) RSGPU_K(11) RSGPU_K(12) RSGPU_K(13) RSGPU_K(14) RSGPU_K(15)
        RSGPU_K(16)
#undef RSGPU_K
        default: return nullptr;
    }
}

}  // namespace

hipError_t launch_masked(const AtlasView &A, const Layout &L, const uint32_t *d_masks, uint32_t *d_status,
                         uint32_t *acc, uint32_t *cnt, hipStream_t st) {
    if (L.nobj <= 0) return hipSuccess;
    if (L.in_base || L.out_base || (L.pitch % 16) != 0 || A.R < 1 || A.R > kMaxR) return hipErrorInvalidValue;
    masked_fn f = pick_masked(A.kmax, A.R);
    if (!f) return hipErrorInvalidValue;
    return f(A, L, d_masks, d_status, acc, cnt, st);
}

hipError_t StatusScratch::acquire(size_t nobj, hipStream_t stream, Slot *&s) {
    mu.lock();  // held until release(): one call in flight per ring position
    s = &slot[next++ % kRing];
    hipError_t e = hipSuccess;
    if (s->done) e = hipEventSynchronize(s->done);  // the call that used it kRing calls ago
    else e = hipEventCreateWithFlags(&s->done, hipEventDisableTiming);
    if (e == hipSuccess && s->cap < nobj) {
        const size_t cap = std::max<size_t>({nobj, 1024, s->cap * 2});
        retire(s->d, false);  // (held while a worker kernel is resident: devmem.cpp)
        s->d = nullptr;
        s->cap = 0;
        e = hipMalloc(&s->d, cap * 2 * sizeof(uint32_t));
        if (e == hipSuccess) e = hipMemsetAsync(s->d, 0, cap * 2 * sizeof(uint32_t), stream);
        if (e == hipSuccess) s->cap = cap;
    }
    if (e != hipSuccess) mu.unlock();
    return e;
}

hipError_t StatusScratch::release(Slot *s, hipStream_t stream, bool ok) {
    hipError_t e = ok ? hipEventRecord(s->done, stream) : hipSuccess;
    if (!ok || e != hipSuccess) {
        // a failed launch may leave counters set: re-zero on the next use
        (void)hipStreamSynchronize(stream);
        retire(s->d, false);
        s->d = nullptr;
        s->cap = 0;
    }
    mu.unlock();
    return e;
}

StatusScratch::~StatusScratch() {
    for (auto &s : slot) {
        if (s.done) (void)hipEventDestroy(s.done);
        retire(s.d, false);
    }
}

}  // namespace rsgpu
