// gf_launch.h — launch policy shared by the pass launchers (gf_kernels.hip,
// gf_masked.hip): workgroup shape, cache policy, occupancy cap, grid order.
#pragma once
#include <algorithm>
#include <cstddef>
#include <cstdint>

#include "gf_apply.h"
#include "gf_device.h"

namespace rsgpu {

// Tuned launch shape of the specialised pass (tools/kbench.hip sweeps on
// MI355X), measured on COLD batches: every timed launch reads a
// batch copy that no launch has touched within the last ~4 GB of traffic, so
// nothing of it is still in the 256 MiB Infinity Cache (KB_ROT=4).  A batch
// that is re-coded back to back instead (the same 1.3 GB every launch) gets
// its parity rewrites absorbed by that cache; that warm rate is not the HBM
// rate and is not what the policy is tuned for.
//   * 256 lanes x one 16-B vector per row (128/512/1024 lanes, 2-4 vectors
//     per lane and walking 2-8 chunks per workgroup are all <= this);
//   * non-temporal (nt) input loads: every input byte is read exactly once;
//   * nt stores: 70.1 vs 67.9 % (sc1) cold on RS(10+2) encode (sc1 wins only
//     warm: 80 vs 70 %, the Infinity Cache absorbing repeated parity writes);
//   * XCD-contiguous workgroup order for every launch: 72.7 vs 70.0 % (linear)
//     cold; splitting each XCD's share into 2-32 interleaved regions loses
//     1-9 points (gf_device.h Order).
constexpr int kBlock = 256;    // lanes per workgroup
constexpr int kUnroll = 1;     // 16-B vectors per lane
constexpr int kLoadAux = 2;    // buffer_load: nt
constexpr int kStoreAux = 2;   // buffer_store: nt
constexpr int kMultiChunks = 1; // chunks per workgroup in the mixed-pattern kernel (kbench: 1 best)
// launches whose objects span more than this use the XCD-contiguous workgroup
// order (gf_device.h Order); 0: every launch
constexpr size_t kXcdSpan = 0;
// Occupancy cap for passes that store rows.  The kernels use no LDS, so a
// dynamic LDS reservation of 1/W of the CU's 160 KiB caps residency at W
// workgroups (4 waves each) per CU.  Fewer concurrent row streams keep DRAM
// pages open longer; the best W keeps about 160 KiB of input loads in flight
// per CU (K rows x 4 KiB per workgroup): W = 40 / K, clamped to [2, 8]
// (tools/kbench KB_SET=occ, cold, r01_kbench_cold_occ_*):
//   encode RS(8+4)   W=4: 75.9 vs 73.2 % full occupancy
//   encode RS(10+2)  W=4: 74.0 vs 72.5 %; ReconstructData RS(10+4) 75.0 vs 73.9 %
//   encode RS(12+4)  W=3: 73.4 vs 68.5 % (W=2: 74.1)
//   encode RS(16+4)  W=2: 77.8 vs 73.7 %;  encode RS(16+2) W=2: 80.1 vs 76.4 %
// Check-only passes (Verify) keep full occupancy: the VALU-bound RS(10+4)
// verify drops from 84.3 to 77.7 % under a cap of 4.
constexpr unsigned store_lds(int K) {
    const int w = K <= 5 ? 8 : (40 / K < 2 ? 2 : 40 / K);
    return 160u * 1024u / (unsigned)w - 256u;
}
constexpr int kMaxK = 16;  // specialised kernels cover K <= 16
constexpr int kMaxR = 4;   // and up to 4 output rows per pass

// 1D launch over nitem items x nchunk workgroups; `span` = bytes the launch's
// objects cover.  Returns the order and sets the grid size.
inline Order make_order(uint32_t nchunk, uint32_t nitem, size_t span, unsigned &grid) {
    Order o{nchunk, nchunk * nitem, 0};
    if (span > kXcdSpan && o.total >= 8) o.xper = (o.total + 7) / 8;
    grid = o.xper ? o.xper * 8 : o.total;
    return o;
}

// items per launch so that the 1D grid stays below 2^31 workgroups
inline int max_items(unsigned nchunk) { return (int)std::max(1u, 0x7ff00000u / std::max(1u, nchunk)); }

// store_row's `part`: bytes of a row's last 16-B vector that may be written
// when the next row starts within it (pitch < 16 * nvec), else 0
inline uint32_t tail_part(size_t pitch, uint32_t nvec) {
    const size_t w = pitch - (size_t)(nvec - 1) * 16;
    return w < 16 ? (uint32_t)w : 0u;
}

// Bytes a row of one object may be written up to (store_row's `part`): the
// row pitch, except in a shard-major layout ([shard][object], obj_stride <
// pitch), where an object's piece of a row is obj_stride bytes and the next
// object's piece (or, for the row's last object, the next row) follows.
inline size_t row_space(const Layout &L) {
    return L.obj_stride > 0 && L.obj_stride < L.pitch ? L.obj_stride : L.pitch;
}

// bytes covered by `no` objects of layout L (one object: its own span)
inline size_t objs_span(const Layout &L, int no, size_t one) {
    return no > 1 ? (size_t)no * L.obj_stride : one;
}

}  // namespace rsgpu
