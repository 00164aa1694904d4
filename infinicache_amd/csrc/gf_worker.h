// gf_worker.h — the resident per-object coder (rsgpu_worker_start,
// include/rsgpu.h): shared host/device layout of its mailboxes and its
// launch arguments.
//
// The reference codes ONE object per EcSet / EcGet call (client/ecRedis.go:96,
// :173; its example object is 1 KiB, client/example/main.go:15,26).  On the
// stream path every such call pays a kernel launch and a stream
// synchronisation (>= 10.8 us for an empty kernel on MI355X,
// profiles/r03_mailbox_probe_hostpoll.txt), more than the coding itself.  The
// worker is one launch of `nslots` workgroups that stay resident: workgroup w
// polls mailbox w in coherent pinned host memory, codes the object the
// request names (reading its rows from, and writing them to, pinned host
// memory over PCIe) and publishes a response word the caller spins on.
//
// Request: one 64-B line of eight 8-B granules {payload, tag}.  The caller
// writes every granule with one 8-B store, tag = the slot's next request
// number; the worker accepts the line only when all eight tags carry that
// number, so a read that raced the caller's stores is simply polled again.
#pragma once
#include <cstdint>

namespace rsgpu {

enum WorkerOp : uint32_t {
    kWopEncode = 0,        // Encode: parity rows <- M[k:] x data rows
    kWopEncodeVerify = 1,  // Encode, then Verify on the parity rows as stored (read back)
    kWopVerify = 2,        // Verify: check rows over all n rows
    kWopReconstruct = 3,   // atlas mode kAtlasReconstruct
    kWopReconstructData = 4,
    kWopDecode = 5,        // fused Client.decode (atlas mode kAtlasDecode)
};

// granule payloads of a request line; kWfSum checks the other seven.
//   kWfOp:       operation (bits 0-7) | present mask << 8 (n <= 16 shards)
//   kWfShardLen: bytes coded per row
//   kWfPitch:    bytes between rows (Split's layout: the shard length; a
//                column slice of a larger object: that object's shard length)
enum WorkerField { kWfOp = 0, kWfShardLen = 1, kWfPitch = 2, kWfSum = 3, kWfInLo = 4, kWfInHi = 5, kWfOutLo = 6,
                   kWfOutHi = 7 };
__host__ __device__ inline uint32_t worker_opmask(uint32_t op, uint32_t mask) { return (op & 0xffu) | (mask << 8); }

// The request line's check word.  Every granule is one aligned 8-B store,
// which the worker accepts only once its tag is current; the check word
// also catches a payload word that arrived apart from its tag (the VRAM
// transport's lines are written through the write-combining BAR mapping,
// whose flush granularity the library does not control): the worker polls
// again until the sum matches.
__host__ __device__ inline uint32_t worker_req_sum(const uint32_t *p) {
    auto rotl = [](uint32_t x, int r) { return (x << r) | (x >> (32 - r)); };
    uint32_t h = 0x5bd1e995u ^ (p[kWfOp] * 0x9E3779B1u);
    h ^= rotl(p[kWfShardLen], 7) ^ rotl(p[kWfPitch], 13) ^ p[kWfInLo] ^ rotl(p[kWfInHi], 3);
    h ^= rotl(p[kWfOutLo], 17) ^ rotl(p[kWfOutHi], 23);
    return h * 0x85EBCA6Bu ^ (h >> 15);
}

struct alignas(64) WorkerReq {
    uint64_t g[8];  // low 32 bits: payload (WorkerField), high 32 bits: tag (request number)
};
struct alignas(64) WorkerResp {
    uint64_t done;     // low: last request number served, high: its status (0 ok, 1 mismatch)
    uint32_t exited;   // the launch generation whose workgroup left this slot
    uint32_t started;  // the launch generation whose workgroup polls this slot (written before its first poll)
    uint32_t pad[12];  // [0..4]: trace stamps (RSGPU_WORKER_TRACE)
};
struct alignas(64) WorkerSlot {
    WorkerReq req;
    WorkerResp resp;
};
static_assert(sizeof(WorkerSlot) == 128, "one line per direction");

constexpr uint32_t kWorkerMaxN = 16;  // codes of <= 16 shards (PatRec records)

struct WorkerArgs {
    WorkerSlot *slots;          // device view of the host mailboxes (responses; host transport: requests too)
    WorkerReq *vreq;            // VRAM transport: the request lines in fine-grained VRAM (else null)
    uint32_t *vmark;            // VRAM transport: start marks, 64 B apart (else resp.started)
    const int32_t *pat[3];      // atlases by mode (kAtlasReconstruct, kAtlasData, kAtlasDecode)
    const void *recs[3];        // PatRec [slot][nsub]
    const uint32_t *tabs[3];    // [slot][nsub][tk][tr][kTabWords] v_perm tables
    uint32_t nsub[3], tk[3], tr[3];
    const void *enc_rec;        // Encode's records [enc_nsub]
    const void *ver_rec;        // Verify's records [ver_nsub]
    const uint32_t *enc_tab, *ver_tab;  // their tables [nsub][k or n][enc_r / ver_r][kTabWords]
    uint32_t enc_nsub, ver_nsub, enc_r, ver_r;
    const uint32_t *ctab;       // [256][kCtabStride] coefficient tables (unused by the kernel)
    uint64_t *activity;         // device words: [0] last time any workgroup served a request, [1] closing
    uint64_t idle_ticks;        // exit after this long without requests (s_memrealtime, 100 MHz)
    uint32_t gen;               // launch generation (written to resp.exited on exit)
    uint32_t n, nmask, k;
    uint32_t trace;             // write device stamps into resp.pad (RSGPU_WORKER_TRACE)
};

}  // namespace rsgpu
