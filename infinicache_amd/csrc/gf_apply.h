// gf_apply.h — host-side description of one GF(2^8) "coding-matrix x shards"
// pass, and the launcher that runs it on gfx950.
//
// Every codec operation of reedsolomon.Encoder (Encode, Verify, Reconstruct,
// ReconstructData, Update, and the fused Client.decode) is ONE linear map over
// GF(2^8) from K input rows of an object to R output rows:
//     out[r] = XOR_c coef[r][c] (x) in[c]
// Rows [0, nw) are written to HBM; rows [nw, R) are "check rows" whose value
// must be all-zero (a parity comparison folded into the matrix) and only set
// a per-object mismatch flag.  The host derives coef from the coding matrix
// (upstream buildMatrix / cached inverses); the kernel never branches on the
// operation.
#pragma once
#include <array>
#include <atomic>
#include <cstddef>
#include <cstdint>
#include <mutex>
#include <vector>

#include <hip/hip_runtime_api.h>

#include "devmem.h"

namespace rsgpu {

// Kernel coefficient format: a coefficient c is stored as five u32 words of
// byte lookup tables over the bit groups [2:0], [5:3], [7:6] of the input
// byte (layout in gf_device.h, kTabWords).  Because multiplication by c is
// GF(2)-linear, c (x) x = c(x)(x & 7) ^ c(x)(x & 0x38) ^ c(x)(x & 0xC0), each
// term one v_perm_b32 lookup for four bytes at once.
constexpr int kCoefWords = 5;  // == kTabWords (gf_device.h; static_assert there)
void coef_tables(uint8_t c, uint32_t out[kCoefWords]);

struct Plan {
    int K = 0;                   // inputs
    int R = 0;                   // outputs
    int nw = 0;                  // rows [0, nw) written, [nw, R) checked
    std::vector<int> in_rows;    // K row indices within an object
    std::vector<int> out_rows;   // R row indices (checked rows: unused)
    std::vector<uint8_t> coef;   // R x K
    std::vector<uint32_t> tab;   // [R][K][kCoefWords] kernel tables
    int ki = 0;                  // trailing identity inputs (gf_apply_kernel)
    // device copies for the generic (K > 16) kernel; uploaded by the first
    // launch that succeeds, then immutable (safe for concurrent launches).  A
    // failed upload frees what it allocated and the next launch retries.
    uint32_t *d_tab = nullptr;     // [K][R][kCoefWords] (input-major)
    uint32_t *d_in_row = nullptr;  // [K]
    uint32_t *d_tab3 = nullptr;    // [K/3][R][16] input-triple tables (gf_apply_generic)
    std::mutex dev_mu;
    std::atomic<bool> dev_done{false};
    // serialized Pass images for mixed-pattern launches, keyed by (pitch and
    // flags, first row, vectors per row): the image's span depends on all three
    std::mutex img_mu;
    std::vector<std::pair<std::array<uint64_t, 3>, std::vector<uint8_t>>> pass_imgs;
    void build_tables();
    int identity_inputs() const;  // trailing identity inputs (ki) of coef
    ~Plan();
};

struct Layout {
    uint8_t *base;        // object 0
    size_t obj_stride;    // bytes between objects
    size_t pitch;         // bytes between rows of an object
    size_t shard_len;     // bytes per shard (S)
    int nobj;
    // one object only (nobj == 1), passes with K <= kRedirectMaxK: rows read
    // from in_base / written to out_base (same offsets), e.g. pinned host memory
    uint8_t *out_base = nullptr;
    bool out_dual = false;        // written rows to base as well
    const uint8_t *in_base = nullptr;
    size_t in_span = 0;           // bytes readable from in_base
    bool copy_in = false;         // input rows copied into base as well
    // at least 16 readable bytes follow the last object's rows (the library's
    // own staging images).  Without it, a layout whose rows' last 16-B vector
    // reaches past the pitch (pitch < 16 * ceil(S / 16)) codes its last object
    // through a scratch copy, so no load runs past the caller's buffer.
    bool slack = false;
    // shard-major batch seen as one object (launch_plan): Pass::sub_*
    uint32_t sub_stride = 0, sub_len = 0, sub_n = 0;
};
constexpr int kRedirectMaxK = 16;  // passes that can redirect their written rows

// Device workspace for mixed-pattern launches (pass images + object lists),
// reused across calls once the previous call's kernels finished with it.
struct MultiWorkspace {
    static constexpr int kRing = 4;  // images in flight before a host wait
    struct Slot {
        void *d = nullptr, *h = nullptr;
        size_t cap = 0;
        hipEvent_t done = nullptr;  // kernels that read this image finished
    };
    std::mutex mu;
    Slot slot[kRing];
    unsigned next = 0;
    // images go up on their own stream so the copy overlaps whatever the
    // caller's stream is still running (e.g. the previous kernel)
    hipStream_t upload = nullptr;
    hipEvent_t uploaded[kRing] = {};  // GPU-side ordering of an upload before its kernels
    std::vector<uint32_t> masks;      // host-flag calls: packed present masks
    ~MultiWorkspace();
};

// Zeroed scratch (acc, cnt: nobj u32 each) for launch_masked's multi-
// reporter status, a ring so calls in flight on different streams never
// share one.  The kernels leave it zero.
struct StatusScratch {
    static constexpr int kRing = 4;
    struct Slot {
        uint32_t *d = nullptr;  // [2][cap]
        size_t cap = 0;
        hipEvent_t done = nullptr;
    };
    std::mutex mu;
    Slot slot[kRing];
    unsigned next = 0;
    // takes the next slot (waiting for the calls that used it), grows and
    // zeroes it on `stream` when needed; release() records its completion
    hipError_t acquire(size_t nobj, hipStream_t stream, Slot *&s);
    hipError_t release(Slot *s, hipStream_t stream, bool ok);
    ~StatusScratch();
};

// Object o of the layout is coded with plans[plan_of[o]] (a batch of Gets
// with mixed erasure patterns): one launch per (K, R) class of sub-passes,
// each workgroup fetching its object's pass by scalar loads.  d_bad follows
// launch_plan's contract per object.
hipError_t launch_plans_multi(const std::vector<Plan *> &plans, const std::vector<int> &plan_of,
                              const Layout &L, uint32_t *d_bad, hipStream_t stream,
                              MultiWorkspace &ws);

// One object of a variable-size device batch (rsgpu_*_dev_objs): shard i at
// base + i * pitch, pitch >= roundup16(shard_len) (no row's last vector
// reaches past the object's rows).
struct DevObj {
    uint8_t *base;
    size_t shard_len, pitch;
};
// Codes every object of the table with the plan, one launch per sub-pass of
// <= 4 rows whatever the objects' sizes (the table goes up through ws's
// ring).  d_bad[o] follows launch_plan's contract per object.
hipError_t launch_plan_objs(Plan &p, const DevObj *objs, int nobj, uint32_t *d_bad, hipStream_t stream,
                            MultiWorkspace &ws);

// Launches the plan over all objects on `stream`.  d_bad (nobj u32) must be
// zeroed by the caller when the plan has check rows.  Returns hipSuccess or
// the first HIP error.
hipError_t launch_plan(Plan &plan, const Layout &L, uint32_t *d_bad, hipStream_t stream);
// Whether the passes of gf_apply_tri's shapes take it (gf_kernels.hip): 1
// (default) or 0 (the single-input kernel).  Measurement (tools/kbench);
// RSGPU_TRI sets it at load.
void set_tri_mode(int mode);

// Device atlas of every erasure pattern of one operation (gf_masked.h): the
// pattern table over all 2^n present masks, one record per (pattern,
// sub-pass), the records' kernel tables, and the 256-entry coefficient table.
struct AtlasView {
    const int32_t *pat = nullptr;
    const void *recs = nullptr;     // PatRec [slot][nsub]
    const uint32_t *tabs = nullptr; // [slot][nsub][kmax][R][kCoefWords]
    const uint32_t *ctab = nullptr; // [256][8]
    int n = 0;      // shards: masks use bits [0, n)
    int kmax = 0;   // inputs of the widest pattern (decode: n; reconstruct: k)
    int R = 0;      // rows per sub-pass (<= 4)
    int nsub = 0;   // sub-passes
    int kfix = 0;   // inputs when every pattern has the same count (reconstruct: k), else 0
    int kcap = 0;   // inputs of the common pattern (occupancy cap: a healthy Get has k)
};

// Codes every object of the layout with the pattern its device-resident
// present mask selects (rsgpu_*_dev_masks).  status (nullable) receives
// kStatus* per object; acc/cnt (nobj u32 each, all zero, left zero) are needed
// when the atlas has check rows.  nvec <= 128 rows use gf_apply_lanes, longer
// rows gf_apply_masked.
hipError_t launch_masked(const AtlasView &A, const Layout &L, const uint32_t *d_masks, uint32_t *d_status,
                         uint32_t *acc, uint32_t *cnt, hipStream_t stream);

}  // namespace rsgpu
