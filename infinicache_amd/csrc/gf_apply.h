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
#include <cstddef>
#include <cstdint>
#include <mutex>
#include <vector>

#include <hip/hip_runtime_api.h>

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
    // device copies for the generic (K > 16) kernel; uploaded once, then
    // immutable (safe for concurrent launches)
    uint32_t *d_tab = nullptr;     // [K][R][kCoefWords] (input-major)
    uint32_t *d_in_row = nullptr;  // [K]
    std::once_flag dev_once;
    hipError_t dev_err = hipSuccess;
    // serialized Pass images for mixed-pattern launches, per (pitch, first row)
    std::mutex img_mu;
    std::vector<std::pair<std::pair<size_t, int>, std::vector<uint8_t>>> pass_imgs;
    void build_tables();
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
    ~MultiWorkspace();
};

// Object o of the layout is coded with plans[plan_of[o]] (a batch of Gets
// with mixed erasure patterns): one launch per (K, R) class of sub-passes,
// each workgroup fetching its object's pass by scalar loads.  d_bad follows
// launch_plan's contract per object.
hipError_t launch_plans_multi(const std::vector<Plan *> &plans, const std::vector<int> &plan_of,
                              const Layout &L, uint32_t *d_bad, hipStream_t stream,
                              MultiWorkspace &ws);

// Launches the plan over all objects on `stream`.  d_bad (nobj u32) must be
// zeroed by the caller when the plan has check rows.  Returns hipSuccess or
// the first HIP error.
hipError_t launch_plan(Plan &plan, const Layout &L, uint32_t *d_bad, hipStream_t stream);

}  // namespace rsgpu
