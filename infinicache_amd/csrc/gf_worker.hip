// gf_worker.hip — the resident per-object coder (gf_worker.h): its kernel,
// and the host side that starts it, posts requests and waits for them.
//
// Measured first with tools/mailbox_probe.hip (profiles/r03_mailbox_probe_hostpoll.txt):
// an empty kernel launch + stream synchronisation costs 10.8 us p50; a
// resident workgroup that polls a host word, reads a 1 KiB object's 10 rows
// over PCIe, writes 2 rows back and publishes a flag answers in 7.5 us.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <set>
#include <thread>

#include "ctx.h"
#include "gf_device.h"
#include "gf_masked.h"
#include "gf_worker.h"

namespace rsgpu {

// sc0 | sc1: system-coherent buffer loads and stores (pinned host memory over
// PCIe; the loads miss in the GPU caches, so a request re-reading a buffer
// the host has rewritten sees the new bytes — tested in test_gpu_worker.py)
constexpr int kSysAux = 1 | 16;

__device__ __forceinline__ uint32_t rfl(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }

// Every value that steers a loop or a branch is wave-uniform (readfirstlane):
// a divergent `if (t == 0) poll` let the compiler's structurizer run lanes
// 1-63 of wave 0 around the request loop forever while lane 0 waited to
// poll (tools/mailbox_probe.hip, first version: a kernel that never ended).
//
// Latency path of one request (RSGPU_WORKER_TRACE):
//   * all four waves poll the request line, staggered, so a poll read is
//     always in flight;
//   * the input rows follow from the operation and the present mask alone
//     (the first k present rows, upstream's survivor rule; the fused decode
//     also reads the extras its check rows compare), so the data loads go out
//     before the atlas lookup of the pattern's record, which overlaps them;
//   * small objects are coded lane-parallel: lane = (input, vector), each
//     lane multiplies ONE input vector into every row and the partial rows
//     are XOR-reduced through LDS.  The first form (lane = vector, every
//     input and row in one lane) kept 7 lanes of one wave busy for a 1 KiB
//     object and spent 3.9 us in dependent table lookups and VALU work after
//     the data had arrived;
//   * larger objects (more vectors than the lanes hold) go lane = vector,
//     256 vectors per chunk.
constexpr uint32_t kLaneVecs = 64;  // lane-parallel path: vectors per pass at most
constexpr uint32_t kLaneU = 4;      // ... and passes (their loads issued up front)

// Encode+Verify's check of a parity vector as stored in host memory: the
// read is issued right behind the store, so the store's completion and the
// read's PCIe round trip overlap (r03: the read waited for the store before,
// 1.3 us + 1.8 us).  Both go to the same address with system-coherent
// policy, and a PCIe read does not pass the posted writes before it, so the
// read should see the new bytes; should it ever see old ones, the wave waits
// for every store to complete and reads again, so only a mismatch that
// survives the second read is reported.  `valid`: bytes of the vector
// compared (0: none).
__device__ __forceinline__ bool readback_check(const u32x4 &want, __amdgpu_buffer_rsrc_t rs, uint32_t voff,
                                               uint32_t soff, uint32_t valid) {
    asm volatile("" ::: "memory");  // the load stays behind the store in program order
    u32x4 b = __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff, kSysAux);
    bool mm = false;
#pragma unroll
    for (int d = 0; d < 4; ++d) mm |= ((b[d] ^ want[d]) & tail_mask(d, valid)) != 0;
    if (__builtin_amdgcn_ballot_w64(mm) != 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        b = __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff, kSysAux);
        mm = false;
#pragma unroll
        for (int d = 0; d < 4; ++d) mm |= ((b[d] ^ want[d]) & tail_mask(d, valid)) != 0;
    }
    return mm;
}

// the c-th set bit of m (per lane; m < 2^16)
__device__ __forceinline__ uint32_t nth_bit(uint32_t m, uint32_t c) {
#pragma unroll
    for (uint32_t i = 0; i < kWorkerMaxN; ++i) m = i < c ? (m & (m - 1u)) : m;
    return m ? (uint32_t)__builtin_ctz(m) : 0u;
}

template <int RM>
__global__ __launch_bounds__(256) void gf_worker(const WorkerArgs a) {
    __shared__ u32x4 lt[256][2];                 // coefficient c: words 0-3, word 4 (gf_apply_lanes' layout)
    __shared__ u32x4 red[RM][kWorkerMaxN][kLaneVecs];  // lane-parallel partial rows
    __shared__ uint32_t sreq[8];
    __shared__ uint32_t sfound;   // the request number a poll found, or ~0u: leave
    const uint32_t t = threadIdx.x, lane = t & 63u, wave = t >> 6;
    {
        const u32x4 *ct = (const u32x4 *)(a.ctab + t * kCtabStride);
        lt[t][0] = ct[0];
        lt[t][1] = ct[1];
    }
    WorkerSlot *ms = a.slots + blockIdx.x;
    // the request line: in pinned host memory (host transport) or in
    // fine-grained VRAM the host writes through the BAR (VRAM transport)
    const WorkerReq *rl = a.vreq ? a.vreq + blockIdx.x : &ms->req;
    uint32_t *mark = a.vreq ? a.vmark + blockIdx.x * 16u : &ms->resp.started;
    // the start mark (beside the request line) is stored before this
    // workgroup's first poll of the line: a caller that sees no mark after
    // taking its request back knows no poll of this launch can have read it
    // (post_and_wait's deadline)
    if (t == 0) __hip_atomic_store(mark, a.gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "");  // store -> later loads (system scope; once per launch)
    // the last request served on this slot (by this or an earlier launch)
    uint32_t last = rfl((uint32_t)__hip_atomic_load(&ms->resp.done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
    uint64_t t_last = __builtin_amdgcn_s_memrealtime();
    if (t == 0) sfound = last;
    __syncthreads();
    for (;;) {
        const uint32_t want = last + 1;
        // stagger the waves' polls by ~1/4 of a PCIe round trip
        if (wave == 1) __builtin_amdgcn_s_sleep(12);
        if (wave == 2) __builtin_amdgcn_s_sleep(24);
        if (wave == 3) __builtin_amdgcn_s_sleep(36);
        uint32_t polls = 0;
        for (;;) {
            uint64_t gv = 0;
            if (lane < 8) gv = __hip_atomic_load(&rl->g[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            const bool ok = lane >= 8 || (uint32_t)(gv >> 32) == want;
            if (__builtin_amdgcn_ballot_w64(!ok) == 0) {  // all eight granules carry the number
                uint32_t pl[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) pl[j] = __builtin_amdgcn_readlane((uint32_t)gv, j);
                if (worker_req_sum(pl) == pl[kWfSum]) {  // else a payload caught mid-write: poll again
                    if (lane < 8) sreq[lane] = (uint32_t)gv;
                    if (lane == 0) sfound = want;  // (several waves may find it: same bytes)
                    break;
                }
            }
            const uint32_t f = rfl(sfound);
            if (f == want || f == ~0u) break;  // another wave found it, or the launch closes
            if (wave == 0 && (++polls & 63u) == 0) {
                // the launch closes as a whole: once one workgroup found every
                // slot idle for idle_ticks it raises `closing`, and the others
                // follow within a few polls (a caller whose slot was left
                // waits for the whole launch to end, then relaunches it)
                bool leave = rfl((uint32_t)__hip_atomic_load(a.activity + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) != 0;
                if (!leave) {
                    const uint64_t now = __builtin_amdgcn_s_memrealtime();
                    uint64_t act = __hip_atomic_load(a.activity, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    act = rfl((uint32_t)act) | ((uint64_t)rfl((uint32_t)(act >> 32)) << 32);
                    const uint64_t ref = act > t_last ? act : t_last;
                    leave = now > ref && now - ref > a.idle_ticks;
                    if (leave && lane == 0)
                        __hip_atomic_store(a.activity + 1, (uint64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                if (leave) {
                    if (lane == 0) sfound = ~0u;
                    break;
                }
            }
            __builtin_amdgcn_s_sleep(4);
        }
        __syncthreads();
        const uint32_t found = rfl(sfound);
        const uint32_t op = rfl(sreq[kWfOp]) & 0xffu;
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        if (found != want || op > kWopDecode) {
            // idle (or a stop request): tell the host this slot's workgroup is gone
            if (t == 0) {
                if (found == want) {  // a stop request: answer it, close the launch
                    __hip_atomic_store(a.activity + 1, (uint64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(&ms->resp.done, (uint64_t)want, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                }
                __hip_atomic_store(&ms->resp.exited, a.gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
            return;
        }
        // S bytes of each row at `pitch` apart: a whole Split image (pitch ==
        // S) or one column slice of a larger object (worker_run_split)
        const uint32_t S = rfl(sreq[kWfShardLen]), mask = (rfl(sreq[kWfOp]) >> 8) & a.nmask;
        const uint32_t pitch = rfl(sreq[kWfPitch]) ? rfl(sreq[kWfPitch]) : S;
        const uint64_t inb = (uint64_t)rfl(sreq[kWfInLo]) | ((uint64_t)rfl(sreq[kWfInHi]) << 32);
        const uint64_t outb = (uint64_t)rfl(sreq[kWfOutLo]) | ((uint64_t)rfl(sreq[kWfOutHi]) << 32);
        __syncthreads();  // sreq is rewritten by the next poll

        // input rows, ascending: Encode the data rows, Verify every row,
        // Reconstruct(Data) the first k present rows, the fused decode every
        // present row (survivors, then the extras its check rows compare)
        uint32_t rows = a.nmask;
        if (op <= kWopEncodeVerify) {
            rows = (1u << a.k) - 1u;
        } else if (op == kWopDecode) {
            rows = mask;
        } else if (op != kWopVerify) {
            uint32_t m = mask;
            rows = 0;
            for (uint32_t i = 0; i < a.k && m; ++i) {
                const uint32_t b = m & (0u - m);
                rows |= b;
                m ^= b;
            }
        }
        const uint32_t kact = (uint32_t)__builtin_popcount(rows);
        const uint32_t nvec = (S + 15) / 16, tail = S - (nvec - 1) * 16;
        // the last vector's bytes past S are not written: the next row's
        // (pitch == S), or the next column slice's (another workgroup's)
        const uint32_t part = tail < 16 ? tail : 0u;
        const uint32_t span = (a.n - 1) * pitch + nvec * 16;
        const __amdgpu_buffer_rsrc_t rsi = __builtin_amdgcn_make_buffer_rsrc((void *)inb, (short)0, (int)span, 0x00020000);
        const __amdgpu_buffer_rsrc_t rso = __builtin_amdgcn_make_buffer_rsrc((void *)outb, (short)0, (int)span, 0x00020000);
        // lane-parallel geometry: vc vectors per pass, np passes
        const uint32_t vc = kact ? (256u / kact < kLaneVecs ? 256u / kact : kLaneVecs) : 1u;
        const uint32_t np = (nvec + vc - 1) / vc;
        const bool lanepar = np <= kLaneU;
        const uint32_t my_c = t / vc, my_v = t - my_c * vc;  // lane-parallel role: (input, vector)
        const bool in_lane = my_c < kact;
        const uint32_t my_row = nth_bit(rows, my_c);

        u32x4 x[kWorkerMaxN];  // lane = vector: every input
        u32x4 xl[kLaneU];      // lane-parallel: this lane's input, one vector per pass
        auto load_chunk = [&](uint32_t c0) {  // lane = vector c0 + t, every input
            const uint32_t v = c0 + t;
            const uint32_t voff = v < nvec ? v * 16u : 0xfffffff0u;  // past every range: reads 0
            uint32_t m = rows;
#pragma unroll
            for (int c = 0; c < (int)kWorkerMaxN; ++c) {
                const uint32_t row = m ? (uint32_t)__builtin_ctz(m) : 0u;
                m &= m - 1u;
                x[c] = u32x4{0u, 0u, 0u, 0u};
                if ((uint32_t)c < kact) x[c] = __builtin_amdgcn_raw_buffer_load_b128(rsi, voff, row * pitch, kSysAux);
            }
        };
        if (lanepar) {
#pragma unroll
            for (uint32_t u = 0; u < kLaneU; ++u) {
                const uint32_t v = u * vc + my_v;
                xl[u] = u32x4{0u, 0u, 0u, 0u};
                if (u < np && in_lane && v < nvec)
                    xl[u] = __builtin_amdgcn_raw_buffer_load_b128(rsi, v * 16u, my_row * pitch, kSysAux);
            }
        } else {
            load_chunk(0);
        }
        asm volatile("" ::: "memory");  // the loads go out before the lookup below waits

        // the operation's records (uniform, scalar loads from device memory)
        constant_ptr<PatRec> rec = nullptr;
        uint32_t nsub = 0;
        if (op <= kWopEncodeVerify) {
            rec = (constant_ptr<PatRec>)a.enc_rec;
            nsub = a.enc_nsub;
        } else if (op == kWopVerify) {
            rec = (constant_ptr<PatRec>)a.ver_rec;
            nsub = a.ver_nsub;
        } else {
            const uint32_t m = op - kWopReconstruct;
            const int32_t slot = ((constant_ptr<int32_t>)a.pat[m])[mask];
            if (slot >= 0) {  // else nothing to do (the host rejected too-few / singular patterns)
                nsub = a.nsub[m];
                rec = (constant_ptr<PatRec>)a.recs[m] + (uint32_t)slot * nsub;
            }
        }
        uint64_t t1 = 0, t2 = 0, t3 = 0, t4 = 0;  // trace: loaded, computed, stored, read back
        bool mismatch = false;
        if (nsub && lanepar) {
#pragma unroll
            for (uint32_t u = 0; u < kLaneU; ++u) {  // compile-time index into xl[] (a runtime one puts it in scratch)
              if (u < np) {
                if (a.trace && u == 0) {
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    t1 = __builtin_amdgcn_s_memrealtime();
                }
                GfIdx g[4];
#pragma unroll
                for (int d = 0; d < 4; ++d) g[d] = gf_idx(xl[u][d]);
                for (uint32_t s = 0; s < nsub; ++s) {
                    const constant_ptr<uint32_t> rw = (constant_ptr<uint32_t>)(rec + s);
                    const uint32_t h0 = rw[0], orow = rw[2];
                    const uint32_t nr = (h0 >> 8) & 0xffu, nw = (h0 >> 16) & 0xffu;
                    // this lane's input times every row of the sub-pass -> LDS
                    if (in_lane && my_v < vc) {
#pragma unroll
                        for (int r = 0; r < RM; ++r) {
                            const uint32_t q = my_c >> 2;
                            const uint32_t w0 = rw[4 + r * 4], w1 = rw[5 + r * 4], w2 = rw[6 + r * 4], w3 = rw[7 + r * 4];
                            const uint32_t cw = q == 0 ? w0 : q == 1 ? w1 : q == 2 ? w2 : w3;
                            const uint32_t cf = (cw >> (8 * (my_c & 3))) & 0xffu;
                            const u32x4 tw = lt[cf][0];
                            const uint32_t t4w = lt[cf][1][0];
                            u32x4 pr;
#pragma unroll
                            for (int d = 0; d < 4; ++d) pr[d] = gf_mac_w(0u, tw, t4w, g[d]);
                            red[r][my_c][my_v] = pr;
                        }
                    }
                    __syncthreads();
                    if (a.trace && u == 0 && s == 0) t2 = __builtin_amdgcn_s_memrealtime();
                    // lane = (row, vector): XOR over the inputs, then store or check
                    const uint32_t r = t / vc, vv = t - r * vc, v = u * vc + vv;
                    u32x4 acc = {0u, 0u, 0u, 0u};
                    if (r < nr && vv < vc && v < nvec) {
                        for (uint32_t c = 0; c < kact; ++c) acc ^= red[r][c][vv];
                        const uint32_t valid = v == nvec - 1 ? tail : 16u;
                        if (r < nw) {
                            const uint32_t row = (orow >> (8 * r)) & 0xffu;
                            store_row<kSysAux>(acc, rso, v * 16u, row * pitch, v == nvec - 1 ? part : 0u);
                            if (op == kWopEncodeVerify) {
                                // Verify on the parity row as stored: read it back over
                                // PCIe (readback_check: issued behind the store, confirmed
                                // after the stores complete on a mismatch)
                                if (a.trace && u == 0 && s == 0 && t == 0) t3 = __builtin_amdgcn_s_memrealtime();
                                mismatch |= readback_check(acc, rso, v * 16u, row * pitch, valid);
                                if (a.trace && u == 0 && s == 0 && t == 0) t4 = __builtin_amdgcn_s_memrealtime();
                            }
                        } else {
#pragma unroll
                            for (int d = 0; d < 4; ++d) mismatch |= (acc[d] & tail_mask(d, valid)) != 0;
                        }
                    }
                    __syncthreads();  // red is rewritten by the next sub-pass / pass
                }
              }
            }
        }
        for (uint32_t c0 = 0; nsub && !lanepar;) {  // larger objects: lane = vector
            const uint32_t v = c0 + t;
            const bool live = v < nvec;
            const uint32_t voff = live ? v * 16u : 0xfffffff0u;  // stores there are dropped
            const uint32_t valid = v == nvec - 1 ? tail : 16u;
            if (a.trace && c0 == 0) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                t1 = __builtin_amdgcn_s_memrealtime();
            }
            for (uint32_t s = 0; s < nsub; ++s) {
                const constant_ptr<uint32_t> rw = (constant_ptr<uint32_t>)(rec + s);
                const uint32_t h0 = rw[0], orow = rw[2];
                const uint32_t nr = (h0 >> 8) & 0xffu, nw = (h0 >> 16) & 0xffu;
                uint32_t acc[RM][4];
#pragma unroll
                for (int r = 0; r < RM; ++r)
#pragma unroll
                    for (int d = 0; d < 4; ++d) acc[r][d] = 0;
#pragma unroll
                for (int c = 0; c < (int)kWorkerMaxN; ++c) {
                    if ((uint32_t)c < kact) {
                        GfIdx g[4];
#pragma unroll
                        for (int d = 0; d < 4; ++d) g[d] = gf_idx(x[c][d]);
#pragma unroll
                        for (int r = 0; r < RM; ++r) {
                            const uint32_t cf = (rw[4 + r * 4 + (c >> 2)] >> (8 * (c & 3))) & 0xffu;
                            const u32x4 tw = lt[cf][0];
                            const uint32_t t4w = lt[cf][1][0];
#pragma unroll
                            for (int d = 0; d < 4; ++d) acc[r][d] = gf_mac_w(acc[r][d], tw, t4w, g[d]);
                        }
                    }
                    // input at a time (the table reads are not all hoisted)
#pragma unroll
                    for (int r = 0; r < RM; ++r)
#pragma unroll
                        for (int d = 0; d < 4; ++d) asm volatile("" : "+v"(acc[r][d]));
                    __builtin_amdgcn_sched_barrier(0);
                }
                if (a.trace && c0 == 0 && s == 0) t2 = __builtin_amdgcn_s_memrealtime();
#pragma unroll
                for (int r = 0; r < RM; ++r) {
                    if ((uint32_t)r >= nr) continue;
                    if ((uint32_t)r < nw) {
                        const uint32_t row = (orow >> (8 * r)) & 0xffu;
                        const u32x4 o = {acc[r][0], acc[r][1], acc[r][2], acc[r][3]};
                        store_row<kSysAux>(o, rso, voff, row * pitch, v == nvec - 1 ? part : 0u);
                    } else if (live) {
#pragma unroll
                        for (int d = 0; d < 4; ++d) mismatch |= (acc[r][d] & tail_mask(d, valid)) != 0;
                    }
                }
                if (op == kWopEncodeVerify && nw > 0) {
                    if (a.trace && c0 == 0 && s == 0) t3 = __builtin_amdgcn_s_memrealtime();
#pragma unroll
                    for (int r = 0; r < RM; ++r) {
                        if ((uint32_t)r >= nw) continue;
                        const uint32_t row = (orow >> (8 * r)) & 0xffu;
                        const u32x4 o = {acc[r][0], acc[r][1], acc[r][2], acc[r][3]};
                        mismatch |= readback_check(o, rso, voff, row * pitch, live ? valid : 0u);
                    }
                    if (a.trace && c0 == 0 && s == 0) {
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                        t4 = __builtin_amdgcn_s_memrealtime();
                    }
                }
            }
            c0 += 256;
            if (c0 >= nvec) break;
            load_chunk(c0);
        }
        // every wave's stores complete before the response is published
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (a.trace && !t3) t3 = __builtin_amdgcn_s_memrealtime();
        const int bad = __syncthreads_or(mismatch);
        if (t == 0) {
            if (a.trace) {  // stamps (s_memrealtime ticks of 10 ns) after the request was seen
                const uint64_t t5 = __builtin_amdgcn_s_memrealtime();
                ms->resp.pad[0] = (uint32_t)(t1 ? t1 - t0 : 0);
                ms->resp.pad[1] = (uint32_t)(t2 ? t2 - t0 : 0);
                ms->resp.pad[2] = (uint32_t)(t3 ? t3 - t0 : 0);
                ms->resp.pad[3] = (uint32_t)(t4 ? t4 - t0 : 0);
                ms->resp.pad[4] = (uint32_t)(t5 - t0);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            __hip_atomic_store(&ms->resp.done, (uint64_t)want | ((uint64_t)(bad ? 1u : 0u) << 32), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(a.activity, __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        last = want;
        t_last = __builtin_amdgcn_s_memrealtime();
    }
}

}  // namespace rsgpu

// ============================================================ host side

namespace rsgpu {

struct Worker {
    int nslots = 0;
    size_t max_shard = 0;
    WorkerSlot *h_slots = nullptr, *d_slots = nullptr;  // coherent pinned mailboxes
    std::vector<uint8_t *> stage_h, stage_d;            // per slot: a coherent pinned object image
    size_t stage_cap = 0;
    // VRAM transport (the default on large-BAR devices; RSGPU_WORKER_TRANSPORT
    // =host keeps round 3's): request lines, start marks and per-slot input
    // images in one fine-grained VRAM allocation the CPU writes through the
    // BAR (same address on both sides); the input rows are copied there, so
    // the kernel's poll and its row loads stay on the device side of PCIe.
    // Outputs and responses stay in host memory.  1 KiB objects: fused
    // encode+verify 8.4 -> 6.9 us p50, decode 7.3 -> 5.7 us
    // (profiles/r04_lat_worker_1k_{host,vram}.txt, same box).
    bool vram = false;
    uint8_t *vmem = nullptr;
    WorkerReq *v_req = nullptr;
    uint32_t *v_mark = nullptr;                         // 16 words (64 B) per slot
    std::vector<uint8_t *> v_img;
    std::vector<uint32_t> seq;                          // per slot: last request number posted
    std::atomic<uint64_t> free_mask{0};                 // bit i: slot i free
    std::atomic<bool> closed{false};                    // stopped: every later call is declined
    std::atomic<int> parked{0};                         // parked (with_workers_parked): calls are declined
    hipStream_t stream = nullptr;                       // its own hardware queue (worker_stream)
    uint64_t *d_state = nullptr;                        // [0] activity (realtime), [1] closing
    void *d_enc = nullptr, *d_ver = nullptr;            // Encode / Verify records
    uint32_t *d_enc_tab = nullptr, *d_ver_tab = nullptr;  // their v_perm tables [nsub][K][R][5]
    uint32_t enc_nsub = 0, ver_nsub = 0, enc_r = 0, ver_r = 0;
    int rm = 4;                                         // kernel instantiation: min(4, parity)
    AtlasView views[3];
    uint64_t idle_ticks = 0;
    std::chrono::nanoseconds timeout{0};                // post_and_wait's deadline for an unstarted workgroup
    std::mutex mu;                                      // launches
    std::atomic<uint32_t> gen{1};                       // the launch the mailboxes belong to
    std::atomic<uint64_t> served{0}, declined{0}, launches{0}, retracted{0};  // rsgpu_worker_stats
    int k = 0;
    bool trace = false;                                 // RSGPU_WORKER_TRACE: device stamps per request
    // trace sums per op: [op][0] requests, [1..5] device stamps (10 ns), [6] host post->response (ns)
    std::atomic<uint64_t> tr[6][7] = {};
    ~Worker() {
        // (the kernel has left: rsgpu_worker_stop; these free at once
        // unless another worker still runs, devmem.cpp)
        if (stream) (void)hipStreamDestroy(stream);
        retire(h_slots, true);
        for (uint8_t *p : stage_h) retire(p, true);
        retire(vmem, false);
        retire(d_state, false);
        retire(d_enc, false);
        retire(d_ver, false);
        retire(d_enc_tab, false);
        retire(d_ver_tab, false);
    }
};

namespace {

// PatRec records of a plan whose inputs are rows [0, K) in index order
// (Encode: the data rows; Verify: every row), one per sub-pass of <= 4 rows
std::vector<PatRec> plan_records(const Plan &p) {
    const int nsub = std::max(1, (p.R + 3) / 4);
    std::vector<PatRec> recs(nsub);
    std::memset(recs.data(), 0, recs.size() * sizeof(PatRec));
    int nchk = 0;
    for (int s = 0; s < nsub; ++s) {
        const int nr = std::max(0, std::min(4, p.R - 4 * s)), nw = std::max(0, std::min(nr, p.nw - 4 * s));
        nchk += nw < nr;
    }
    for (int s = 0; s < nsub; ++s) {
        PatRec &rc = recs[s];
        const int r0 = 4 * s, nr = std::max(0, std::min(4, p.R - r0)), nw = std::max(0, std::min(nr, p.nw - r0));
        rc.kact = (uint8_t)p.K;
        rc.nr = (uint8_t)nr;
        rc.nw = (uint8_t)nw;
        rc.nchk = (uint8_t)nchk;
        for (int c = 0; c < p.K; ++c) rc.in_row[c] = (uint8_t)p.in_rows[c];
        for (int r = 0; r < nr; ++r) {
            if (r < nw) rc.out_row[r] = (uint8_t)p.out_rows[r0 + r];
            for (int c = 0; c < p.K; ++c) rc.coef[r][c] = p.coef[(size_t)(r0 + r) * p.K + c];
        }
    }
    return recs;
}

// v_perm tables of those records, [nsub][K][R][kTabWords], R = min(4, plan rows)
std::vector<uint32_t> record_tables(const std::vector<PatRec> &recs, int K, int R) {
    std::vector<uint32_t> t(recs.size() * K * R * kTabWords, 0);
    for (size_t s = 0; s < recs.size(); ++s)
        for (int c = 0; c < K; ++c)
            for (int r = 0; r < R; ++r)
                coef_tables(recs[s].coef[r][c], &t[(((s * K) + c) * R + r) * kTabWords]);
    return t;
}

hipError_t upload_records(const std::vector<PatRec> &r, void *&d) {
    hipError_t e = hipMalloc(&d, r.size() * sizeof(PatRec));
    if (e == hipSuccess) e = upload(d, r.data(), r.size() * sizeof(PatRec));
    return e;
}

// The resident kernel's stream.  It must be a hardware queue of its own (a
// stream sharing the worker's queue runs nothing while the kernel is
// resident) and non-blocking (a blocking stream makes every null-stream call
// of the process — a synchronous hipMemcpy, PyTorch's default stream — wait
// for the kernel to idle out).  Measured with a resident kernel on each kind
// (tools/sync_probe.hip, profiles/r04_sync_probe.txt):
//   * hipExtStreamCreateWithCUMask (round 3): own queue, but blocking —
//     null-stream hipMemcpy and hipMallocAsync/hipFreeAsync on another
//     stream waited for it;
//   * a plain non-blocking stream: shares the 4 normal-priority queues —
//     kernels on other streams waited for it;
//   * non-blocking at the greatest priority: kernels on 8 other streams, the
//     null stream and stream-ordered allocation ran at once.
// So the worker takes the last (RSGPU_WORKER_STREAM=cumask keeps round 3's).
// The device-wide calls (hipFree, hipHostFree, hipHostUnregister) wait on
// every kind: devmem.cpp and with_workers_parked keep them off the paths
// that run beside the worker.
hipError_t worker_stream(int device, hipStream_t &out) {
    const char *kind = std::getenv("RSGPU_WORKER_STREAM");
    if (kind && std::strcmp(kind, "cumask") == 0) {
        int cus = 0;
        hipError_t e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
        if (e != hipSuccess) return e;
        std::vector<uint32_t> cu_mask((size_t)(cus + 31) / 32, 0xffffffffu);
        if (cus % 32) cu_mask.back() = (1u << (cus % 32)) - 1;
        return hipExtStreamCreateWithCUMask(&out, (uint32_t)cu_mask.size(), cu_mask.data());
    }
    int least = 0, greatest = 0;
    hipError_t e = hipDeviceGetStreamPriorityRange(&least, &greatest);
    if (e != hipSuccess) return e;
    return hipStreamCreateWithPriority(&out, hipStreamNonBlocking, greatest);
}

// launch generation `g` of the worker (w->mu held)
hipError_t launch(Worker &w, uint32_t g) {
    WorkerArgs a{};
    a.slots = w.d_slots;
    a.vreq = w.vram ? w.v_req : nullptr;
    a.vmark = w.vram ? w.v_mark : nullptr;
    for (int m = 0; m < 3; ++m) {
        a.pat[m] = w.views[m].pat;
        a.recs[m] = w.views[m].recs;
        a.tabs[m] = w.views[m].tabs;
        a.nsub[m] = (uint32_t)w.views[m].nsub;
        a.tk[m] = (uint32_t)w.views[m].kmax;
        a.tr[m] = (uint32_t)w.views[m].R;
    }
    a.enc_rec = w.d_enc;
    a.ver_rec = w.d_ver;
    a.enc_tab = w.d_enc_tab;
    a.ver_tab = w.d_ver_tab;
    a.enc_r = w.enc_r;
    a.ver_r = w.ver_r;
    a.enc_nsub = w.enc_nsub;
    a.ver_nsub = w.ver_nsub;
    a.ctab = w.views[0].ctab;
    a.activity = w.d_state;
    a.idle_ticks = w.idle_ticks;
    a.gen = g;
    a.n = (uint32_t)w.views[0].n;
    a.nmask = (uint32_t)((1u << w.views[0].n) - 1);
    a.k = (uint32_t)w.k;
    a.trace = w.trace ? 1u : 0u;
    hipError_t e = hipMemsetAsync(w.d_state, 0, 16, w.stream);
    if (e != hipSuccess) return e;
    switch (w.rm) {
        case 1: hipLaunchKernelGGL(gf_worker<1>, dim3(w.nslots), dim3(256), 0, w.stream, a); break;
        case 2: hipLaunchKernelGGL(gf_worker<2>, dim3(w.nslots), dim3(256), 0, w.stream, a); break;
        case 3: hipLaunchKernelGGL(gf_worker<3>, dim3(w.nslots), dim3(256), 0, w.stream, a); break;
        default: hipLaunchKernelGGL(gf_worker<4>, dim3(w.nslots), dim3(256), 0, w.stream, a); break;
    }
    return hipGetLastError();
}

hipError_t upload_zero(void *d, size_t bytes) {
    std::vector<uint8_t> z(bytes, 0);
    return upload(d, z.data(), bytes);
}

int worker_create(rsgpu_ctx *ctx, int nslots, unsigned idle_us, size_t max_shard, std::unique_ptr<Worker> &out) {
    std::unique_ptr<Worker> w(new Worker());
    w->nslots = nslots;
    w->max_shard = max_shard;
    w->k = ctx->k;
    w->trace = std::getenv("RSGPU_WORKER_TRACE") != nullptr;
    w->idle_ticks = (uint64_t)idle_us * 100;  // s_memrealtime: 100 MHz
    {
        // RSGPU_WORKER_TIMEOUT_US: how long a posted request may wait for its
        // slot's workgroup to start polling before it is taken back and the
        // call takes the stream path (post_and_wait)
        const char *t = std::getenv("RSGPU_WORKER_TIMEOUT_US");
        const long long us = t ? std::atoll(t) : 0;
        w->timeout = std::chrono::microseconds(us > 0 ? us : 200000);
    }
    for (int m = 0; m < 3; ++m) {
        int e = ctx->atlas_view((AtlasMode)m, w->views[m]);
        if (e) return e;
    }
    std::vector<PatRec> er = plan_records(*ctx->plan_encode()), vr = plan_records(*ctx->plan_verify());
    w->enc_nsub = (uint32_t)er.size();
    w->ver_nsub = (uint32_t)vr.size();
    w->rm = std::min(4, ctx->p);
    w->enc_r = w->ver_r = (uint32_t)w->rm;
    for (int m = 0; m < 3; ++m)
        if (w->views[m].R > w->rm) return RSGPU_ERR_INVALID_ARG;  // (atlas rows per sub-pass <= min(4, p))
    HIP_TRY(upload_records(er, w->d_enc));
    HIP_TRY(upload_records(vr, w->d_ver));
    const std::vector<uint32_t> et = record_tables(er, ctx->k, w->rm), vt = record_tables(vr, ctx->n, w->rm);
    HIP_TRY(hipMalloc(&w->d_enc_tab, et.size() * 4));
    HIP_TRY(upload(w->d_enc_tab, et.data(), et.size() * 4));
    HIP_TRY(hipMalloc(&w->d_ver_tab, vt.size() * 4));
    HIP_TRY(upload(w->d_ver_tab, vt.data(), vt.size() * 4));
    HIP_TRY(hipMalloc(&w->d_state, 16));
    HIP_TRY(worker_stream(ctx->device, w->stream));
    HIP_TRY(hipHostMalloc((void **)&w->h_slots, sizeof(WorkerSlot) * nslots, hipHostMallocMapped | hipHostMallocCoherent));
    std::memset((void *)w->h_slots, 0, sizeof(WorkerSlot) * nslots);
    for (int i = 0; i < nslots; ++i) w->h_slots[i].resp.exited = 1;  // generation 1: not running
    HIP_TRY(hipHostGetDevicePointer((void **)&w->d_slots, w->h_slots, 0));
    w->stage_cap = (size_t)ctx->n * max_shard + 64;
    w->stage_h.assign(nslots, nullptr);
    w->stage_d.assign(nslots, nullptr);
    for (int i = 0; i < nslots; ++i) {
        HIP_TRY(hipHostMalloc((void **)&w->stage_h[i], w->stage_cap, hipHostMallocMapped | hipHostMallocCoherent));
        HIP_TRY(hipHostGetDevicePointer((void **)&w->stage_d[i], w->stage_h[i], 0));
    }
    w->seq.assign(nslots, 0);
    {
        const char *tp = std::getenv("RSGPU_WORKER_TRANSPORT");
        int large_bar = 0;
        (void)hipDeviceGetAttribute(&large_bar, hipDeviceAttributeIsLargeBar, ctx->device);
        // the CPU writes fine-grained VRAM through its device pointer only
        // when the whole VRAM is mapped through the BAR (large BAR)
        if (!(tp && std::strcmp(tp, "host") == 0) && large_bar) {
            const size_t img = round_up(w->stage_cap, 256);
            const size_t bytes = (size_t)nslots * (64 + 64 + img);
            HIP_TRY(hipExtMallocWithFlags((void **)&w->vmem, bytes, hipDeviceMallocFinegrained));
            w->v_req = (WorkerReq *)w->vmem;
            w->v_mark = (uint32_t *)(w->vmem + (size_t)nslots * 64);
            HIP_TRY(upload_zero(w->vmem, (size_t)nslots * 128));
            w->v_img.resize(nslots);
            for (int i = 0; i < nslots; ++i) w->v_img[i] = w->vmem + (size_t)nslots * 128 + (size_t)i * img;
            w->vram = true;
        }
    }
    w->free_mask.store(nslots >= 64 ? ~0ull : ((1ull << nslots) - 1));
    out = std::move(w);
    return RSGPU_OK;
}

uint64_t all_slots(const Worker &w) { return w.nslots >= 64 ? ~0ull : ((1ull << w.nslots) - 1); }

int acquire_slot(Worker &w) {
    uint64_t m = w.free_mask.load(std::memory_order_relaxed);
    while (m) {
        const int i = __builtin_ctzll(m);
        if (w.free_mask.compare_exchange_weak(m, m & ~(1ull << i), std::memory_order_acquire)) return i;
    }
    return -1;
}
void release_slot(Worker &w, int i) { w.free_mask.fetch_or(1ull << i, std::memory_order_release); }

// slot i's request line: pinned host memory, or VRAM through the BAR
WorkerReq &req_line(Worker &w, int i) { return w.vram ? w.v_req[i] : w.h_slots[i].req; }
// slot i's start mark (VRAM: read through the BAR, on the deadline path only)
uint32_t start_mark(Worker &w, int i) {
    return w.vram ? __atomic_load_n(&w.v_mark[(size_t)i * 16], __ATOMIC_ACQUIRE)
                  : __atomic_load_n(&w.h_slots[i].resp.started, __ATOMIC_ACQUIRE);
}

// every granule of slot i's request line: payload rq[g], tag `tag`, each
// one aligned 8-B store; the check word is rq[kWfSum]
void post_line(Worker &w, int i, const uint32_t (&rq)[8], uint32_t tag) {
    WorkerReq &r = req_line(w, i);
    for (int g = 0; g < 8; ++g)
        __atomic_store_n(&r.g[g], (uint64_t)rq[g] | ((uint64_t)tag << 32), __ATOMIC_RELEASE);
    // the BAR mapping is write-combining: flush the line now (a doorbell left
    // in the WC buffer waited milliseconds in r03_mailbox_probe_vram_direct)
    if (w.vram) __builtin_ia32_sfence();
}

// Posts request `rq` (payloads) on slot i and waits for its response;
// relaunches the resident kernel when it had left (idle) before serving it.
// Returns RSGPU_OK (status set), kWorkerDeclined (the request was taken back
// before any workgroup could have read it: the caller takes the stream
// path) or an error.
//
// Waiting: a spin of ~50 us (a request is answered in ~7-10 us), then
// yields, then 20 us sleeps, so a slow answer does not burn a core.
//
// Deadline (w.timeout, 200 ms by default): a request whose slot has no
// workgroup of the current launch polling it yet (its launch is waiting for
// CUs behind other work) is taken back: the tags are rewound to the last
// number served, which no workgroup accepts, and the start mark is read
// again.  Each workgroup writes its mark and fences before its first poll of
// the line, and the caller fences between rewinding the tags and reading the
// mark, so a mark still absent means no poll of this launch has read the
// request: the call is declined and the caller's buffers are its own again.
// A mark that appeared meanwhile means the workgroup may hold the request,
// so it is posted again (the same number and payloads: served once either
// way) and waited for.  A request whose workgroup is running is never taken
// back — it would write into buffers the caller may have freed — and is
// answered in microseconds; a kernel that dies is caught by hipStreamQuery.
uint32_t post(Worker &w, int i, const uint32_t (&rq)[8]) {
    const uint32_t n = ++w.seq[i];
    post_line(w, i, rq, n);
    return n;
}

int wait_for(Worker &w, int i, const uint32_t (&rq)[8], const uint32_t n, uint32_t &status) {
    using clk = std::chrono::steady_clock;
    WorkerSlot &s = w.h_slots[i];
    auto retract = [&] {
        post_line(w, i, rq, n - 1);
        --w.seq[i];
    };
    auto fail = [&](int err) {
        retract();
        return err;
    };
    uint32_t cur = w.gen.load(std::memory_order_acquire);
    const auto t_post = clk::now();
    auto t_deadline = t_post + w.timeout;
    auto t_query = t_post + std::chrono::milliseconds(1);
    for (uint64_t spins = 1;; ++spins) {
        const uint64_t d = __atomic_load_n(&s.resp.done, __ATOMIC_ACQUIRE);
        if ((uint32_t)d == n) {
            status = (uint32_t)(d >> 32);
            if (w.trace && (rq[kWfOp] & 0xffu) < 6) {
                auto &tr = w.tr[rq[kWfOp] & 0xffu];
                tr[0].fetch_add(1);
                for (int j = 0; j < 5; ++j) tr[1 + j].fetch_add(s.resp.pad[j]);
                tr[6].fetch_add((uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(clk::now() - t_post).count());
            }
            return RSGPU_OK;
        }
        if (__atomic_load_n(&s.resp.exited, __ATOMIC_ACQUIRE) == cur) {
            // this slot's workgroup of launch `cur` is gone (idle, parked, or
            // never launched): the request line stays posted, a new launch serves it
            std::lock_guard<std::mutex> l(w.mu);
            if (w.gen.load() == cur) {
                // every workgroup of `cur` leaves promptly
                hipError_t he = hipStreamSynchronize(w.stream);
                if (he != hipSuccess) return fail(hip_fail(he, "resident worker"));
                // serialised with the library's frees (devmem.cpp), which
                // also go now if no other worker kernel is resident
                he = launch_guarded([&] { return launch(w, cur + 1); });
                if (he != hipSuccess) return fail(hip_fail(he, "resident worker launch"));
                w.gen.store(cur + 1, std::memory_order_release);
                w.launches.fetch_add(1, std::memory_order_relaxed);
            }
            cur = w.gen.load(std::memory_order_acquire);
            t_deadline = clk::now() + w.timeout;  // (the new launch gets the whole period to start)
            continue;
        }
        if (spins & 15u) {
            __builtin_ia32_pause();
            continue;
        }
        const auto now = clk::now();
        const auto waited = now - t_post;
        if (waited > std::chrono::milliseconds(2)) std::this_thread::sleep_for(std::chrono::microseconds(20));
        else if (waited > std::chrono::microseconds(50)) std::this_thread::yield();
        if (now >= t_query) {  // a kernel that died without answering
            t_query = now + std::chrono::milliseconds(1);
            const hipError_t q = hipStreamQuery(w.stream);
            if (q != hipSuccess && q != hipErrorNotReady) return fail(hip_fail(q, "resident worker"));
        }
        if (now >= t_deadline) {
            cur = w.gen.load(std::memory_order_acquire);
            if (start_mark(w, i) != cur) {
                retract();
                std::atomic_thread_fence(std::memory_order_seq_cst);
                if (start_mark(w, i) != cur && (uint32_t)__atomic_load_n(&s.resp.done, __ATOMIC_ACQUIRE) != n) {
                    w.retracted.fetch_add(1, std::memory_order_relaxed);
                    return kWorkerDeclined;
                }
                ++w.seq[i];  // == n again
                post_line(w, i, rq, n);
            }
            t_deadline = now + w.timeout;
        }
    }
}

int post_and_wait(Worker &w, int i, const uint32_t (&rq)[8], uint32_t &status) {
    return wait_for(w, i, rq, post(w, i, rq), status);
}

// Takes every mailbox (calls in flight finish first; w.closed / w.parked
// make later calls decline), then ends the resident launch and waits for it.
// The mailboxes stay taken: a stop keeps them, a park gives them back.
int quiesce(Worker &w) {
    const uint64_t all = all_slots(w);
    uint64_t got = 0;
    while (got != all) {
        const int i = acquire_slot(w);
        if (i >= 0) got |= 1ull << i;
        else std::this_thread::yield();
    }
    std::lock_guard<std::mutex> l(w.mu);
    const uint32_t cur = w.gen.load();
    if (__atomic_load_n(&w.h_slots[0].resp.exited, __ATOMIC_ACQUIRE) != cur) {
        // running (or its launch pending): a stop request on slot 0; its
        // workgroup raises `closing` and every other one leaves on its next
        // poll (the other mailboxes' request numbers stay as they are)
        uint32_t rq[8] = {0xffu, 0, 0, 0, 0, 0, 0, 0};
        rq[kWfSum] = worker_req_sum(rq);
        post_line(w, 0, rq, ++w.seq[0]);
    }
    const hipError_t he = hipStreamSynchronize(w.stream);
    return he == hipSuccess ? RSGPU_OK : hip_fail(he, "worker stop");
}

void print_trace(Worker &w) {
    static const char *names[6] = {"encode", "encode+verify", "verify", "reconstruct", "reconstruct-data", "decode"};
    for (int op = 0; op < 6; ++op) {
        const uint64_t nreq = w.tr[op][0].load();
        if (!nreq) continue;
        auto avg = [&](int j, double unit) { return w.tr[op][j].load() * unit / nreq; };
        std::fprintf(stderr,
                     "rsgpu worker trace %-16s %7llu requests; avg us after the request was seen: inputs "
                     "loaded %.2f, computed %.2f, stores done %.2f, read back %.2f, response %.2f; host post -> "
                     "response %.2f\n",
                     names[op], (unsigned long long)nreq, avg(1, 0.01), avg(2, 0.01), avg(3, 0.01), avg(4, 0.01),
                     avg(5, 0.01), avg(6, 0.001));
    }
}

// Contexts with a worker: for parking (every worker of the process) and for
// the process-exit guard — a resident kernel still polling when the HIP
// runtime tears down would read freed pinned mailboxes (a GPU memory fault),
// and a Go or C host that exits without rsgpu_destroy is normal.  The guard
// is registered with atexit after the HIP runtime has initialised (its own
// teardown was registered before), so it runs first and stops every worker.
std::mutex g_live_mu;
std::set<rsgpu_ctx *> g_live;
// stops in progress: from before the stopping worker leaves the probe's view
// (ctx->worker_raw cleared) until its kernel has left (quiesce), the probe
// counts it as resident
std::atomic<int> g_stopping{0};
// parks, starts and stops one at a time (each takes every mailbox of the
// workers it touches; two of them interleaving would each hold a part)
std::mutex g_park_mu;

bool workers_resident();  // below (devmem.cpp's probe)

void stop_all_workers() {
    std::vector<rsgpu_ctx *> live;
    {
        std::lock_guard<std::mutex> l(g_live_mu);
        live.assign(g_live.begin(), g_live.end());
    }
    for (rsgpu_ctx *c : live) (void)rsgpu_worker_stop(c);
}
void track_worker(rsgpu_ctx *ctx, bool on) {
    static std::once_flag once;
    std::call_once(once, [] {
        std::atexit(stop_all_workers);
        set_resident_probe(workers_resident);
    });
    std::lock_guard<std::mutex> l(g_live_mu);
    if (on) g_live.insert(ctx);
    else g_live.erase(ctx);
}

// A reader epoch on ctx's worker (rsgpu_ctx::worker_raw): counted in the
// parity of the epoch current when the pointer is read (the epoch is read
// again after counting: a reader counted in a parity that flipped meanwhile
// tries again), so stop_locked's wait covers every reader that can hold it.
struct WorkerRef {
    rsgpu_ctx *c;
    uint32_t p;
    Worker *w;
    explicit WorkerRef(rsgpu_ctx *ctx) : c(ctx) {
        for (;;) {
            const uint32_t e = c->worker_epoch.load(std::memory_order_seq_cst);
            p = e & 1u;
            c->worker_readers[p].fetch_add(1, std::memory_order_seq_cst);
            if (c->worker_epoch.load(std::memory_order_seq_cst) == e) break;
            c->worker_readers[p].fetch_sub(1, std::memory_order_seq_cst);
        }
        w = c->worker_raw.load(std::memory_order_seq_cst);
    }
    ~WorkerRef() { c->worker_readers[p].fetch_sub(1, std::memory_order_release); }
    WorkerRef(const WorkerRef &) = delete;
    WorkerRef &operator=(const WorkerRef &) = delete;
};

// devmem.cpp's probe (called with its lock held): some started worker's
// kernel is launched and not finished.  Each worker is read inside a reader
// epoch, so a concurrent stop cannot free it meanwhile (and this never drops
// the last reference).
bool workers_resident() {
    if (g_stopping.load(std::memory_order_seq_cst) > 0) return true;
    std::lock_guard<std::mutex> l(g_live_mu);
    for (rsgpu_ctx *c : g_live) {
        const WorkerRef ref(c);
        if (ref.w && hipStreamQuery(ref.w->stream) == hipErrorNotReady) return true;
    }
    return false;
}

// ctx's worker stopped and detached (ctx->worker_mu and g_park_mu held)
int stop_locked(rsgpu_ctx *ctx) {
    std::shared_ptr<Worker> w = std::atomic_exchange(&ctx->worker, std::shared_ptr<Worker>());
    if (!w) {
        track_worker(ctx, false);
        return RSGPU_OK;
    }
    g_stopping.fetch_add(1, std::memory_order_seq_cst);  // resident to the probe until quiesce is done
    track_worker(ctx, false);
    // no new call finds it; the calls that may hold it finish (they are
    // declined below, or finish a request they already posted)
    ctx->worker_raw.store(nullptr, std::memory_order_seq_cst);
    const uint32_t old = ctx->worker_epoch.fetch_add(1, std::memory_order_seq_cst) & 1u;
    w->closed.store(true, std::memory_order_release);
    DeviceGuard dg_;
    int e = ctx->use_device(dg_, false);
    if (!e) e = quiesce(*w);
    g_stopping.fetch_sub(1, std::memory_order_seq_cst);
    while (ctx->worker_readers[old].load(std::memory_order_acquire) != 0) std::this_thread::yield();
    if (w->trace) print_trace(*w);
    // its kernel has left: what was retired while it ran may be freed now
    worker_count(-1);
    return e;
}

}  // namespace

// Objects past max_shard, up to kSplitMaxShard per shard, when their rows
// form one pinned Split image: the rows' byte columns go to several
// mailboxes at once (every operation is a byte-column map), each request a
// column slice [b0, b0 + len) of every row at the image's pitch, read and
// written in place over PCIe.  The workgroups of those mailboxes code their
// slices side by side, so the object moves at the rate of several PCIe read
// streams without a kernel launch or a stream synchronisation.  Slices are
// whole 16-B vectors except the last, so no two workgroups write the same
// bytes; the check flags are OR-ed.  A slice taken back at its deadline
// declines the whole call (the stream path recodes every column: each
// operation is idempotent on its outputs).
constexpr size_t kSplitMaxShard = (size_t)64 << 10;  // objects of up to ~640 KiB at k = 10 (crossover: below)
// RSGPU_WORKER_SPLIT_MAX (bytes per shard) overrides it: measurement
size_t split_max_shard() {
    static const size_t v = [] {
        const char *e = std::getenv("RSGPU_WORKER_SPLIT_MAX");
        const long long b = e ? std::atoll(e) : 0;
        return b > 0 ? (size_t)b : kSplitMaxShard;
    }();
    return v;
}
constexpr size_t kSplitMinSlice = 1536;             // bytes per slice at least (a lane-parallel pass)
// staged slices (pageable rows copied into the mailboxes' images): up to 16
// KiB shards.  Past it the copies through the BAR cost more than the launch
// the worker saves: pageable 256 KiB decode 24.2 us stream vs 31.5 us staged,
// 640 KiB 37.9 vs 76.0 (64 KiB 18.7 -> 13.1, 128 KiB 20.0 -> 16.3;
// profiles/r04_worker_split/staged_*)
constexpr size_t kStagedSplitMaxShard = (size_t)16 << 10;

// Two forms.  In place (img: the device view of one pinned Split image):
// each slice is read and written there at the image's pitch.  Staged (img ==
// nullptr: pageable rows, e.g. the Go Split array an EcSet passes): each
// slice's input rows are copied into its mailbox's image (VRAM through the
// BAR, or pinned host memory) at pitch = slice length, the written rows come
// back through the mailbox's pinned image; slices then fit max_shard, so
// this form may take every mailbox.  rd / wr: the rows the op reads / writes.
int worker_run_split(Worker &w, uint32_t op, size_t S, uint32_t mask, const uint8_t *img, uint8_t *const *rows,
                     int n, uint32_t rd, uint32_t wr, uint32_t *bad) {
    const bool staged = img == nullptr;
    if (staged && (S > kStagedSplitMaxShard || w.max_shard < 16)) {
        w.declined.fetch_add(1, std::memory_order_relaxed);
        return kWorkerDeclined;
    }
    const size_t smax = w.max_shard & ~(size_t)15;  // a staged slice fits its mailbox's image
    const int need = staged ? (int)((S + smax - 1) / smax) : 1;
    const int cap = staged ? w.nslots : std::max(2, w.nslots / 2);  // in place: leave mailboxes to other callers
    const int want = std::max(need, (int)std::min<size_t>((size_t)cap, (S + kSplitMinSlice - 1) / kSplitMinSlice));
    int got[64], m = 0;
    if (want <= cap && !w.closed.load(std::memory_order_acquire) && !w.parked.load(std::memory_order_acquire))
        for (; m < want; ++m) {
            const int i = acquire_slot(w);
            if (i < 0) break;
            got[m] = i;
        }
    if (m < need || m == 0 || (m == 1 && want > 1 && S > 4 * kSplitMinSlice)) {  // too few mailboxes free
        for (int j = 0; j < m; ++j) release_slot(w, got[j]);
        w.declined.fetch_add(1, std::memory_order_relaxed);
        return kWorkerDeclined;
    }
    const size_t slice = round_up((S + m - 1) / m, 16);
    const int used = (int)((S + slice - 1) / slice);
    for (int j = used; j < m; ++j) release_slot(w, got[j]);
    m = used;
    uint32_t rqs[64][8], ns[64];
    for (int j = 0; j < m; ++j) {
        const int i = got[j];
        const size_t b0 = (size_t)j * slice, len = std::min(slice, S - b0);
        uintptr_t pin = staged ? 0 : (uintptr_t)(img + b0), pout = pin;
        size_t pitch = S;
        if (staged) {
            uint8_t *dst = w.vram ? w.v_img[i] : w.stage_h[i];
            for (int r = 0; r < n; ++r)
                if ((rd >> r) & 1) std::memcpy(dst + (size_t)r * len, rows[r] + b0, len);
            if (w.vram) __builtin_ia32_sfence();  // the rows before the request line (post_line)
            pin = (uintptr_t)(w.vram ? w.v_img[i] : w.stage_d[i]);
            pout = wr ? (uintptr_t)w.stage_d[i] : pin;
            pitch = len;
        }
        uint32_t *rq = rqs[j];
        rq[kWfOp] = worker_opmask(op, mask);
        rq[kWfShardLen] = (uint32_t)len;
        rq[kWfPitch] = (uint32_t)pitch;
        rq[kWfInLo] = (uint32_t)pin;
        rq[kWfInHi] = (uint32_t)(pin >> 32);
        rq[kWfOutLo] = (uint32_t)pout;
        rq[kWfOutHi] = (uint32_t)(pout >> 32);
        rq[kWfSum] = worker_req_sum(rq);
        ns[j] = post(w, i, rqs[j]);
    }
    int e = RSGPU_OK;
    bool declined = false;
    uint32_t any = 0;
    for (int j = 0; j < m; ++j) {  // every slice is answered or taken back before its mailbox is freed
        uint32_t st = 0;
        const int r = wait_for(w, got[j], rqs[j], ns[j], st);
        if (r == kWorkerDeclined) declined = true;
        else if (r) e = e ? e : r;
        else any |= st;
    }
    if (staged && !e && !declined)  // the written rows back to the caller's buffers
        for (int j = 0; j < m; ++j) {
            const size_t b0 = (size_t)j * slice, len = std::min(slice, S - b0);
            for (int r = 0; r < n; ++r)
                if ((wr >> r) & 1) std::memcpy(rows[r] + b0, w.stage_h[got[j]] + (size_t)r * len, len);
        }
    for (int j = 0; j < m; ++j) release_slot(w, got[j]);
    if (e) return e;
    if (declined) {
        w.declined.fetch_add(1, std::memory_order_relaxed);
        return kWorkerDeclined;
    }
    w.served.fetch_add(1, std::memory_order_relaxed);
    *bad = any;
    return RSGPU_OK;
}

// The worker serves one object when it can: returns RSGPU_OK with *bad set
// (0 / 1), kWorkerDeclined to use the stream path, or an error.
int worker_run(rsgpu_ctx *ctx, uint32_t op, size_t S, uint32_t mask, uint8_t *const *rows, uint32_t *bad) {
    // a reader epoch: a concurrent rsgpu_worker_stop detaches the worker and
    // frees it only after this call is done with it
    const WorkerRef ref(ctx);
    Worker *w = ref.w;
    if (!w || S == 0) return kWorkerDeclined;
    const int n = ctx->n, k = ctx->k;
    const uint32_t full = (1u << n) - 1;
    // rows the op reads and writes
    uint32_t rd, wr;
    switch (op) {
        case kWopEncode: case kWopEncodeVerify: rd = (1u << k) - 1; wr = full & ~rd; break;
        case kWopVerify: rd = full; wr = 0; break;
        case kWopReconstructData: rd = mask; wr = ~mask & ((1u << k) - 1); break;
        default: rd = mask; wr = ~mask & full; break;
    }
    if (S > w->max_shard) {
        // larger objects: column slices over several mailboxes, in place in
        // one pinned Split image, else staged through the mailboxes' images
        if (S > split_max_shard() || S > 0xffffffffu / (uint32_t)n) {
            w->declined.fetch_add(1, std::memory_order_relaxed);
            return kWorkerDeclined;
        }
        bool split = true;
        for (int r = 1; r < n && split; ++r) split = rows[r] == rows[0] + (size_t)r * S;
        const uint8_t *img = split ? (const uint8_t *)host_device_ptr(rows[0], (size_t)(n - 1) * S + (S + 15) / 16 * 16)
                                   : nullptr;
        return worker_run_split(*w, op, S, mask, img, rows, n, rd, wr, bad);
    }
    // stopped or parked: decline (checked before and after taking a mailbox;
    // a stop / park takes every mailbox, so one of the two checks sees it)
    const int i = w->closed.load(std::memory_order_acquire) || w->parked.load(std::memory_order_acquire)
                      ? -1
                      : acquire_slot(*w);
    if (i < 0) {  // every mailbox busy: the stream path takes this call
        w->declined.fetch_add(1, std::memory_order_relaxed);
        return kWorkerDeclined;
    }
    // one Split image in pinned memory readable past its last row's 16-B
    // vector: the worker reads and writes it in place (zero copy)
    bool split = true;
    for (int r = 1; r < n && split; ++r) split = rows[r] == rows[0] + (size_t)r * S;
    const uint8_t *img = split ? (const uint8_t *)host_device_ptr(rows[0], (size_t)(n - 1) * S + (S + 15) / 16 * 16)
                               : nullptr;
    const uint8_t *in = img, *out = img;
    if (w->vram) {
        // the rows it reads go to the slot's VRAM image (write-combined
        // through the BAR); the fence orders them before the request line
        // (posted writes to one device land in order)
        uint8_t *vi = w->v_img[i];
        for (int r = 0; r < n; ++r)
            if ((rd >> r) & 1) std::memcpy(vi + (size_t)r * S, rows[r], S);
        __builtin_ia32_sfence();
        in = vi;
        if (!out) out = w->stage_d[i];  // the written rows come back through host memory
        if (op == kWopVerify || !wr) out = in;  // (nothing written)
    } else if (!img) {  // stage through the slot's image
        in = out = w->stage_d[i];
        for (int r = 0; r < n; ++r)
            if ((rd >> r) & 1) std::memcpy(w->stage_h[i] + (size_t)r * S, rows[r], S);
    }
    uint32_t rq[8] = {worker_opmask(op, mask), (uint32_t)S, (uint32_t)S, 0, (uint32_t)(uintptr_t)in, (uint32_t)((uintptr_t)in >> 32),
                      (uint32_t)(uintptr_t)out, (uint32_t)((uintptr_t)out >> 32)};
    rq[kWfSum] = worker_req_sum(rq);
    uint32_t status = 0;
    int e = post_and_wait(*w, i, rq, status);
    if (e == RSGPU_OK && out == w->stage_d[i])
        for (int r = 0; r < n; ++r)
            if ((wr >> r) & 1) std::memcpy(rows[r], w->stage_h[i] + (size_t)r * S, S);
    release_slot(*w, i);
    if (e == kWorkerDeclined) {
        w->declined.fetch_add(1, std::memory_order_relaxed);
        return kWorkerDeclined;
    }
    if (e) return e;
    w->served.fetch_add(1, std::memory_order_relaxed);
    *bad = status;
    return RSGPU_OK;
}

int with_workers_parked(const std::function<int()> &fn) {
    std::lock_guard<std::mutex> pl(g_park_mu);
    std::vector<std::shared_ptr<Worker>> ws;
    {
        std::lock_guard<std::mutex> l(g_live_mu);
        for (rsgpu_ctx *c : g_live)
            if (auto w = std::atomic_load(&c->worker)) ws.push_back(std::move(w));
    }
    if (ws.empty()) return fn();
    int e = RSGPU_OK;
    for (auto &w : ws) {
        w->parked.fetch_add(1, std::memory_order_acq_rel);
        const int q = quiesce(*w);
        if (!e) e = q;
    }
    const int r = fn();
    if (!e) drain_retired();  // no worker kernel is resident: the kept buffers go too
    for (auto &w : ws) {
        w->free_mask.store(all_slots(*w), std::memory_order_release);
        w->parked.fetch_sub(1, std::memory_order_acq_rel);
    }
    return e ? e : r;
}

}  // namespace rsgpu

// ============================================================== C ABI

extern "C" {

int rsgpu_worker_start(rsgpu_ctx *ctx, int nslots, unsigned idle_us, size_t max_shard) {
    if (!ctx || nslots < 0 || nslots > 64) return RSGPU_ERR_INVALID_ARG;
    if (ctx->multi()) {
        for (size_t i = 0; i < ctx->subs.size(); ++i) {
            const int e = rsgpu_worker_start(ctx->subs[i].get(), nslots, idle_us, max_shard);
            if (e) {  // no entry is left with a worker
                for (size_t j = 0; j < i; ++j) (void)rsgpu_worker_stop(ctx->subs[j].get());
                return e;
            }
        }
        return RSGPU_OK;
    }
    if (ctx->n > (int)kWorkerMaxN) return RSGPU_ERR_NOT_IMPLEMENTED;
    if (atlas_estimate(ctx->k, ctx->p, true) > ((size_t)32 << 20)) return RSGPU_ERR_NOT_IMPLEMENTED;
    if (!nslots) nslots = 8;
    if (!idle_us) idle_us = 50000;
    if (!max_shard) max_shard = 4096;  // worker ahead of the stream path up to ~40 KB objects (r03_lat_*_sizes.txt)
    if (max_shard > ((size_t)1 << 24)) return RSGPU_ERR_INVALID_ARG;
    DeviceGuard dg_;
    int e = ctx->use_device(dg_, false);
    if (e) return e;
    std::lock_guard<std::mutex> l(ctx->worker_mu);
    std::lock_guard<std::mutex> pl(g_park_mu);
    if ((e = stop_locked(ctx))) return e;  // restart with the new settings
    std::unique_ptr<Worker> w;
    if ((e = worker_create(ctx, nslots, idle_us, max_shard, w))) return e;
    worker_count(+1);  // before its first launch (the first request's)
    std::shared_ptr<Worker> sp(w.release());
    // in the probe's view before any caller can find it (and so launch it)
    track_worker(ctx, true);
    ctx->worker_raw.store(sp.get(), std::memory_order_seq_cst);
    std::atomic_store(&ctx->worker, std::move(sp));
    return RSGPU_OK;
}

int rsgpu_worker_stats(const rsgpu_ctx *ctx, uint64_t *served, uint64_t *declined, uint64_t *launches) {
    if (!ctx) return RSGPU_ERR_INVALID_ARG;
    uint64_t s = 0, d = 0, l = 0;
    auto add = [&](const rsgpu_ctx *c) {
        if (const std::shared_ptr<Worker> w = std::atomic_load(&c->worker)) {
            s += w->served.load();
            d += w->declined.load();
            l += w->launches.load();
        }
    };
    add(ctx);
    for (auto &c : ctx->subs) add(c.get());
    if (served) *served = s;
    if (declined) *declined = d;
    if (launches) *launches = l;
    return RSGPU_OK;
}

int rsgpu_worker_stop(rsgpu_ctx *ctx) {
    if (!ctx) return RSGPU_ERR_INVALID_ARG;
    if (ctx->multi()) {
        int first = RSGPU_OK;
        for (auto &c : ctx->subs) {
            const int e = rsgpu_worker_stop(c.get());
            if (!first) first = e;
        }
        return first;
    }
    std::lock_guard<std::mutex> l(ctx->worker_mu);
    std::lock_guard<std::mutex> pl(g_park_mu);
    return stop_locked(ctx);
}

}  // extern "C"
