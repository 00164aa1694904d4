// pieces.hip — shard-major Get batches on whole 128-B lines
// (rsgpu_shardmajor_layout, rsgpu_copy_pieces; include/rsgpu.h).
//
// Every real Get batch is mixed-pattern (the proxy's first-d rule,
// proxy/lambdastore/connection.go:274-306), and a batch of small objects is
// decoded fastest shard-major ([shard][object]: shard i of object o at
// base + i*pitch + o*obj_stride), where the decode kernels stream whole rows.
// How fast depends on where the pieces sit: at a 112-B stride (1 KiB objects,
// S = 103, 16-B aligned) every lost piece a decode rewrites straddles two
// 128-B lines and the decode runs at 41 % of HBM peak; at a 128-B stride each
// piece is one whole line (profiles/r03_pmc_small1k_sm_mixed.json
// and r04_*a128*).  The library chooses that geometry (rsgpu_shardmajor_layout)
// and moves rows between an object-major batch and it on the device
// (rsgpu_copy_pieces), so a caller need not lay the batch out by hand.
//
// The copy is byte work (no GF arithmetic): one workgroup row of lanes per
// (row, 256 vectors) over the object range of a launch, 16-B buffer loads at
// any byte offset (unaligned mode) and stores that write exactly shard_len
// bytes of each piece (store_row: the last vector in 8/4/2/1-B parts).  Lanes
// walk the objects of one row in order, so the shard-major side is read or
// written contiguously.  HBM-bound: 2 x shard_len bytes per piece moved.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

#include "ctx.h"
#include "gf_device.h"

namespace rsgpu {

namespace {

constexpr int kPieceRows = 32;  // rows per launch (masks are 64-bit; launches repeat above 32)

struct PieceArgs {
    const uint8_t *src;
    uint8_t *dst;
    uint32_t src_pitch, dst_pitch;    // row pitches (fit 32 bits per launch, checked on the host)
    uint32_t src_stride, dst_stride;  // object strides
    uint32_t S, nvec, part, nobj;     // piece bytes, 16-B vectors per piece, last-vector bytes (0: 16), objects
    uint32_t src_span, dst_span;      // readable / writable bytes from a row's first piece
    uint32_t row[kPieceRows];         // the rows this launch moves (blockIdx.y indexes them)
};

__global__ __launch_bounds__(256) void copy_pieces_kernel(const PieceArgs a) {
    const uint32_t r = a.row[blockIdx.y];
    const uint32_t id = blockIdx.x * 256u + threadIdx.x;  // (object, vector) of this row
    const uint32_t o = id / a.nvec, v = id - o * a.nvec;
    if (o >= a.nobj) return;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void *)(a.src + (size_t)r * a.src_pitch), (short)0, (int)a.src_span, 0x00020000);
    const __amdgpu_buffer_rsrc_t rd =
        __builtin_amdgcn_make_buffer_rsrc((void *)(a.dst + (size_t)r * a.dst_pitch), (short)0, (int)a.dst_span, 0x00020000);
    const uint32_t voff = o * a.src_stride + v * 16u;
    u32x4 x;
    if (v == a.nvec - 1 && a.part && o == a.nobj - 1) {
        // the launch's last piece ends inside its last 16-B vector, and the
        // range check zeroes every dword that reaches past src_span: byte loads
        x = u32x4{0u, 0u, 0u, 0u};
        for (uint32_t b = 0; b < a.part; ++b) {
            const uint32_t y = __builtin_amdgcn_raw_buffer_load_b8(rs, voff + b, 0, 0);
            const uint32_t sh = 8u * (b & 3u);
            if (b < 4) x[0] |= y << sh;
            else if (b < 8) x[1] |= y << sh;
            else if (b < 12) x[2] |= y << sh;
            else x[3] |= y << sh;
        }
    } else {
        // a piece's last vector may run into the next piece or gap: read,
        // never written (store_row below writes shard_len bytes)
        x = __builtin_amdgcn_raw_buffer_load_b128(rs, voff, 0, 0);
    }
    store_row<0>(x, rd, o * a.dst_stride + v * 16u, 0, v == a.nvec - 1 ? a.part : 0u);
}

}  // namespace

}  // namespace rsgpu

extern "C" {

int rsgpu_shardmajor_layout(size_t shard_len, int nobj, size_t *obj_stride, size_t *pitch) {
    if (!obj_stride || !pitch || nobj < 0) return RSGPU_ERR_INVALID_ARG;
    if (shard_len == 0) return RSGPU_ERR_SHARD_NO_DATA;
    // whole 128-B lines per piece when the gap stays narrow enough for the
    // encode to code the batch as one object (launch_plan: a gap of at most
    // shard_len / 4), else 16-B aligned pieces
    const size_t s128 = round_up(shard_len, 128), s16 = round_up(shard_len, 16);
    const size_t stride = (s128 - shard_len) * 4 <= shard_len ? s128 : s16;
    const size_t p = round_up(std::max<size_t>(1, (size_t)nobj) * stride, 256);
    // the coding calls require (data+parity) * pitch < 4 GiB (they check it);
    // here only a pitch no code of >= 2 shards can use is refused
    if (p >= ((size_t)1 << 31)) return RSGPU_ERR_INVALID_ARG;
    *obj_stride = stride;
    *pitch = p;
    return RSGPU_OK;
}

int rsgpu_copy_pieces(rsgpu_ctx *ctx, const void *d_src, size_t src_pitch, size_t src_obj_stride, void *d_dst,
                      size_t dst_pitch, size_t dst_obj_stride, size_t shard_len, int nobj, uint64_t rows,
                      void *stream) {
    using namespace rsgpu;
    if (!ctx || !d_src || !d_dst || nobj < 0) return RSGPU_ERR_INVALID_ARG;
    if (ctx->multi()) {
        rsgpu_ctx *c = ctx->sub_for(d_dst);
        if (!c) return RSGPU_ERR_INVALID_ARG;
        ctx = c;
    }
    if (shard_len == 0) return RSGPU_ERR_SHARD_NO_DATA;
    if (ctx->n < 64 && (rows >> ctx->n) != 0) return RSGPU_ERR_INVALID_ARG;
    // pieces of one layout never overlap: src_obj_stride / dst_obj_stride >=
    // shard_len when nobj > 1
    if (nobj > 1 && (src_obj_stride < shard_len || dst_obj_stride < shard_len)) return RSGPU_ERR_INVALID_ARG;
    std::vector<uint32_t> list;
    for (int i = 0; i < ctx->n && i < 64; ++i)
        if ((rows >> i) & 1) list.push_back((uint32_t)i);
    const size_t maxrow = list.empty() ? 0 : list.back();
    // ... and neither do its rows (check_layout's rule, over the rows that
    // move): object-major, each object's rows 0..maxrow inside its stride;
    // shard-major, each row holding every object's piece.  Workgroups write
    // pieces concurrently, so an overlapping destination would be silent,
    // nondeterministic corruption; a malformed source is refused
    // the same way.
    auto layout_ok = [&](size_t pitch, size_t stride) {
        if (list.size() > 1 && pitch < shard_len) return false;
        if (nobj > 1 && list.size() > 0 && stride < (maxrow + 1) * pitch &&
            !(stride >= shard_len && pitch >= (size_t)(nobj - 1) * stride + shard_len))
            return false;
        return true;
    };
    if (!layout_ok(src_pitch, src_obj_stride) || !layout_ok(dst_pitch, dst_obj_stride)) return RSGPU_ERR_INVALID_ARG;
    DeviceGuard dg_;
    int e = ctx->use_device(dg_);
    if (e) return e;
    if (nobj == 0 || rows == 0) return RSGPU_OK;
    if (maxrow * std::max(src_pitch, dst_pitch) >= ((size_t)1 << 32)) return RSGPU_ERR_INVALID_ARG;
    PieceArgs a{};
    a.src_pitch = (uint32_t)src_pitch;
    a.dst_pitch = (uint32_t)dst_pitch;
    a.src_stride = (uint32_t)src_obj_stride;
    a.dst_stride = (uint32_t)dst_obj_stride;
    a.S = (uint32_t)shard_len;
    a.nvec = (uint32_t)((shard_len + 15) / 16);
    a.part = (uint32_t)(shard_len % 16);
    // objects per launch: every offset within a row (object * stride + 16 *
    // vector) and every lane id fit 31 bits
    const size_t stride_max = std::max<size_t>({src_obj_stride, dst_obj_stride, 16});
    const size_t per = std::max<size_t>(1, std::min<size_t>(((size_t)1 << 31) / stride_max,
                                                          ((size_t)1 << 31) / a.nvec) - 1);
    if (src_obj_stride >= ((size_t)1 << 31) || dst_obj_stride >= ((size_t)1 << 31) || shard_len >= ((size_t)1 << 31))
        return RSGPU_ERR_INVALID_ARG;
    const hipStream_t st = (hipStream_t)stream;
    for (size_t o0 = 0; o0 < (size_t)nobj; o0 += per) {
        const size_t no = std::min(per, (size_t)nobj - o0);
        a.src = (const uint8_t *)d_src + o0 * src_obj_stride;
        a.dst = (uint8_t *)d_dst + o0 * dst_obj_stride;
        a.nobj = (uint32_t)no;
        a.src_span = (uint32_t)((no - 1) * src_obj_stride + shard_len);
        a.dst_span = (uint32_t)((no - 1) * dst_obj_stride + shard_len);
        const unsigned gx = (unsigned)((no * a.nvec + 255) / 256);
        for (size_t r0 = 0; r0 < list.size(); r0 += kPieceRows) {
            const size_t nr = std::min<size_t>(kPieceRows, list.size() - r0);
            for (size_t j = 0; j < nr; ++j) a.row[j] = list[r0 + j];
            hipLaunchKernelGGL(copy_pieces_kernel, dim3(gx, (unsigned)nr), dim3(256), 0, st, a);
            const hipError_t he = hipGetLastError();
            if (he != hipSuccess) return hip_fail(he, "copy_pieces");
        }
    }
    return RSGPU_OK;
}

}  // extern "C"
