/*
 * rsgpu.h — C ABI of the MI355X-native Reed-Solomon (GF(2^8)) codec that
 * replaces the InfiniCache client's erasure-coding hot path.
 *
 * Interface being replaced: the Go interface reedsolomon.Encoder
 * (github.com/klauspost/reedsolomon v1.9.3, /root/reference/go.mod:16) held in
 * Client.EC (/root/reference/client/client.go:38), built by NewEncoder
 * (/root/reference/client/ec.go:14-24) and called from exactly
 * /root/reference/client/ecRedis.go:384 (Split), :390 (Encode), :395/:406/:420
 * (Verify), :415 (Reconstruct), :430 (Join).  The 7-method contract is mirrored
 * by DummyEncoder at /root/reference/client/ec.go:30-121.
 *
 * Split/Join are host slicing and stay on the caller's side (Go shim / the
 * Python host mirror in infinicache_amd/ec.py); every byte of GF arithmetic
 * goes through the functions below onto hand-written HIP kernels for gfx950.
 * There is no CPU compute fallback: without a usable device every compute
 * entry point returns RSGPU_ERR_NO_DEVICE (argument validation, which follows
 * the upstream error precedence, still runs first).
 *
 * Conventions
 *   - return 0 on success, a negative RSGPU_ERR_* code otherwise;
 *   - shard "present" == non-zero length (Go: len(shard) != 0; nil == empty);
 *   - the library never retains a caller pointer after a call returns; host
 *     calls are synchronous (all device work done, outputs written);
 *   - contexts are safe for concurrent use from several threads.
 */
#ifndef RSGPU_H
#define RSGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- error codes: 1:1 onto the upstream Go error values ---------------- */
#define RSGPU_OK 0
#define RSGPU_ERR_INV_SHARD_NUM -1        /* reedsolomon.ErrInvShardNum      */
#define RSGPU_ERR_MAX_SHARD_NUM -2        /* reedsolomon.ErrMaxShardNum      */
#define RSGPU_ERR_TOO_FEW_SHARDS -3       /* reedsolomon.ErrTooFewShards     */
#define RSGPU_ERR_SHARD_NO_DATA -4        /* reedsolomon.ErrShardNoData      */
#define RSGPU_ERR_SHARD_SIZE -5           /* reedsolomon.ErrShardSize        */
#define RSGPU_ERR_SINGULAR -6             /* reedsolomon errSingular         */
#define RSGPU_ERR_SHORT_DATA -7           /* reedsolomon.ErrShortData        */
#define RSGPU_ERR_RECONSTRUCT_REQUIRED -8 /* reedsolomon.ErrReconstructRequired */
#define RSGPU_ERR_INVALID_INPUT -9        /* reedsolomon.ErrInvalidInput     */
#define RSGPU_ERR_NOT_IMPLEMENTED -10     /* client.ErrNotImplemented (ec.go:10-12) */
/* library-level failures (no Go counterpart) */
#define RSGPU_ERR_INVALID_ARG -20         /* NULL pointer, bad layout/alignment */
#define RSGPU_ERR_NO_DEVICE -21           /* no HIP device / device id out of range */
#define RSGPU_ERR_HIP -22                 /* a HIP runtime call failed */
#define RSGPU_ERR_NOMEM -23               /* host or device allocation failed */

/* ---- rsgpu_create flags ------------------------------------------------ */
#define RSGPU_MATRIX_VANDERMONDE 0u /* default: upstream buildMatrix          */
#define RSGPU_MATRIX_CAUCHY 1u      /* upstream WithCauchyMatrix()            */
#define RSGPU_MATRIX_PAR1 2u        /* upstream WithPAR1Matrix()              */
#define RSGPU_MATRIX_MASK 3u

typedef struct rsgpu_ctx rsgpu_ctx;

/* rsgpu_create's `device`: every visible gfx950 device (a multi-device
 * context, see rsgpu_create_multi); with none visible, a context on device 0
 * whose compute calls return RSGPU_ERR_NO_DEVICE. */
#define RSGPU_ALL_DEVICES (-1)

/* Replaces reedsolomon.New(dataShards, parityShards, opts...) as called at
 * /root/reference/client/ec.go:19.  Rejects data<=0 || parity<=0
 * (RSGPU_ERR_INV_SHARD_NUM) and data+parity > 256 (RSGPU_ERR_MAX_SHARD_NUM).
 * Builds the coding matrix on the host; device resources are created lazily
 * on the first compute call on `device`.  *out is NULL on error. */
int rsgpu_create(int data_shards, int parity_shards, int device, unsigned flags, rsgpu_ctx **out);
void rsgpu_destroy(rsgpu_ctx *ctx);

/* One context over several GPUs of this process (the Go client is one
 * process, client/client.go:47-59; its EcSet/EcGet callers share Client.EC).
 * An object's shards never leave one GPU: per-object host calls go to the
 * devices round-robin, batch host calls send object o to devices[o % ndev]
 * and run the devices' pipelines in parallel (one PCIe link each),
 * device-resident calls run on the device that owns d_base.  A device may be
 * listed more than once: every entry is an independent single-device context
 * (its own streams, staging slots and batch pipeline, e.g. two pipelines
 * feeding one GPU), and device-resident calls on memory of a device listed
 * several times go to its entries in turn. */
int rsgpu_create_multi(int data_shards, int parity_shards, const int *devices, int ndev, unsigned flags,
                       rsgpu_ctx **out);
/* The context's devices, one per entry of its device list (up to cap written
 * to out); returns their number. */
int rsgpu_devices(const rsgpu_ctx *ctx, int *out, int cap);
/* Per entry of rsgpu_devices: the number of compute calls that entry has run
 * on its device so far (batch calls count once per entry they reached).
 * Returns the number of entries.  Lets a caller see how its work spread. */
int rsgpu_device_calls(const rsgpu_ctx *ctx, uint64_t *out, int cap);

int rsgpu_data_shards(const rsgpu_ctx *ctx);
int rsgpu_parity_shards(const rsgpu_ctx *ctx);
/* Copies the (data+parity) x data coding matrix, row-major, into out. */
int rsgpu_matrix(const rsgpu_ctx *ctx, uint8_t *out);
const char *rsgpu_strerror(int code);
/* Number of visible HIP devices (0 when none); never fails. */
int rsgpu_device_count(void);
/* 1 if the library's gfx950 code object can run on `device`, else 0. */
int rsgpu_device_ok(int device);

/* ---- per-object host-memory API (what the Go shim forwards to) ---------- */
/* shards[i]: caller-owned host buffer of lens[i] bytes; lens[i] == 0 marks a
 * nil/empty shard.  nshards must equal data+parity (else TOO_FEW_SHARDS).
 * Shards of any length, as upstream: an object whose staged rows would pass
 * 1 GiB is coded in column slabs (each byte column is independent), so the
 * 4 GiB a device pass addresses is no limit here. */

/* Encode (upstream Encode; ecRedis.go:390): checkShards(nilok=false), then
 * shards[k..k+p) = parity.  All shards must be allocated (len == size). */
int rsgpu_encode(rsgpu_ctx *ctx, uint8_t *const *shards, const size_t *lens, int nshards);

/* Verify (upstream Verify; ecRedis.go:395,406,420): *ok = 1 iff every parity
 * shard equals the parity recomputed from the data shards.  Any nil shard ->
 * (*ok = 0, RSGPU_ERR_SHARD_SIZE) with no device work, as upstream. */
int rsgpu_verify(rsgpu_ctx *ctx, const uint8_t *const *shards, const size_t *lens, int nshards,
                 int *ok);

/* Client.encode's Encode -> Verify pair (ecRedis.go:390-395), fused: the data
 * shards go to the device once, Encode's pass writes the parity shards back
 * into the caller's buffers, and Verify's pass then re-checks every parity
 * shard against the data on the same device image (the bytes just copied
 * back) -> *ok.  Argument checks and errors are Encode's.  Saves Verify's
 * second upload of all data+parity shards. */
int rsgpu_encode_verify(rsgpu_ctx *ctx, uint8_t *const *shards, const size_t *lens, int nshards,
                        int *ok);

/* Reconstruct / ReconstructData (upstream reconstruct(shards, dataOnly);
 * ecRedis.go:415).  lens[i] == 0 marks shard i missing; for every missing
 * shard the caller passes a writable buffer of the common shard size in
 * shards[i] (upstream re-uses cap >= size, else allocates — the Go shim does
 * that allocation before the call).  Survivors are the first `data` present
 * shards in index order; inverses are cached per erasure pattern (upstream
 * inversionTree).  data_only = 1 leaves missing parity shards untouched. */
int rsgpu_reconstruct(rsgpu_ctx *ctx, uint8_t *const *shards, const size_t *lens, int nshards,
                      int data_only);

/* Fused Client.decode (ecRedis.go:404-427: Reconstruct, then Verify) in ONE
 * device pass: reconstructs every missing shard in place and sets *ok to the
 * result the upstream Verify-after-Reconstruct would return.  With every
 * shard present it is Client.decode's first Verify (*ok = its result). */
int rsgpu_decode(rsgpu_ctx *ctx, uint8_t *const *shards, const size_t *lens, int nshards, int *ok);

/* Update (upstream Update): for each non-nil newdata[c] (new_lens[c] != 0):
 * shards[c] ^= newdata[c] (the old buffer becomes the delta, as upstream) and
 * parity ^= M[.,c] * delta.  nnew must equal data. */
int rsgpu_update(rsgpu_ctx *ctx, uint8_t *const *shards, const size_t *lens, int nshards,
                 const uint8_t *const *newdata, const size_t *new_lens, int nnew);

/* ---- resident worker: low-latency per-object calls -----------------------
 * One EcSet / EcGet codes ONE object (ecRedis.go:96, :173; the example object
 * is 1 KiB, client/example/main.go:15,26).  On the stream path each such call
 * costs a kernel launch plus a stream synchronisation (>= 10.8 us on MI355X
 * for an empty kernel).  rsgpu_worker_start makes the per-object calls above
 * (rsgpu_encode, rsgpu_encode_verify, rsgpu_verify, rsgpu_reconstruct,
 * rsgpu_decode and their *_image forms) go to a resident kernel instead:
 * nslots workgroups, each polling its own request mailbox in pinned host
 * memory; a call posts one 64-B request line and spins on the response word.
 * The object's rows are read and written over PCIe in place when they form
 * one Split image in memory from rsgpu_host_alloc, else through the mailbox's
 * pinned image (memcpy).  Objects with shard_len > max_shard (up to 64 KiB)
 * whose rows form one pinned Split image go to several free mailboxes at once,
 * each coding a column slice of every row in place (128-640 KiB objects:
 * 1.1-1.4x faster than the stream path); other buffers with shard_len up to
 * 16 KiB go as slices staged through the mailboxes' images.  Larger objects,
 * codes of more than 16 shards, and calls that find too few mailboxes free
 * take the stream path.
 * Results, checks and errors are exactly those of the stream path.
 *   nslots     mailboxes = resident workgroups (1..64; 0: 8)
 *   idle_us    the kernel leaves after this long without any request (0: 50 ms)
 *              and the next call relaunches it
 *   max_shard  the largest shard_len served (0: 4 KiB; the worker is ahead of the
 *              stream path up to ~40 KB objects and level with it at 64 KiB)
 * Calling it again restarts the worker with the new settings.  Multi-device
 * contexts: one worker per entry (a start that fails on one entry stops the
 * others).  Requires data+parity <= 16 (RSGPU_ERR_NOT_IMPLEMENTED otherwise).
 * Beside a resident kernel (DESIGN.md §5 "The worker beside the rest of the
 * library"): it runs on a non-blocking stream of its own hardware queue, so
 * other streams and the null stream never wait for it; the library defers its
 * own device / pinned frees while a worker runs (hipFree and hipHostFree wait
 * for every kernel of the device) and parks every worker around
 * rsgpu_host_free / rsgpu_host_unregister; a caller's own hipDeviceSynchronize,
 * hipFree or hipHostFree still waits until the worker idles out.  A request
 * whose workgroup has not started within RSGPU_WORKER_TIMEOUT_US (200 ms) is
 * taken back and the call takes the stream path.  On large-BAR devices the
 * request lines and the input rows go through fine-grained VRAM the CPU
 * writes through the BAR (RSGPU_WORKER_TRANSPORT=host keeps them in pinned
 * host memory); outputs and responses are written to host memory. */
int rsgpu_worker_start(rsgpu_ctx *ctx, int nslots, unsigned idle_us, size_t max_shard);
/* Stops the worker (waits for calls in flight; calls arriving meanwhile take
 * the stream path); the per-object calls go back to the stream path.
 * rsgpu_destroy stops it too. */
int rsgpu_worker_stop(rsgpu_ctx *ctx);
/* Calls the worker served, calls it declined (too few mailboxes free, an
 * object past max_shard it cannot slice, a request taken back at its
 * deadline: they took the stream path), and kernel launches so far (the
 * first call after an idle exit relaunches it); summed over a multi-device
 * context's entries.  Any pointer may be NULL. */
int rsgpu_worker_stats(const rsgpu_ctx *ctx, uint64_t *served, uint64_t *declined, uint64_t *launches);

/* ---- per-object calls on one contiguous image ----------------------------
 * Shard i of the object is base[i*shard_len, (i+1)*shard_len): Split's layout
 * (ecRedis.go:384 — Split returns consecutive slices of one backing array).
 * One pointer crosses the boundary, so a cgo caller passes the Split backing
 * array itself (Go memory holding no Go pointers: legal under cgo's rules), or
 * a C-owned pinned image it copied gathered shards into (EcGet's separate
 * buffers, ecRedis.go:161-170).  present: bit i set = shard i holds data
 * (the others are missing and get written); data+parity <= 64.  Semantics,
 * checks and errors are those of the pointer-table calls above. */
int rsgpu_encode_image(rsgpu_ctx *ctx, uint8_t *base, size_t shard_len, int nshards);
int rsgpu_encode_verify_image(rsgpu_ctx *ctx, uint8_t *base, size_t shard_len, int nshards, int *ok);
int rsgpu_verify_image(rsgpu_ctx *ctx, const uint8_t *base, size_t shard_len, int nshards, int *ok);
int rsgpu_reconstruct_image(rsgpu_ctx *ctx, uint8_t *base, size_t shard_len, int nshards, uint64_t present,
                            int data_only);
int rsgpu_decode_image(rsgpu_ctx *ctx, uint8_t *base, size_t shard_len, int nshards, uint64_t present, int *ok);

/* ---- batched device-resident API (HBM in, HBM out) ---------------------
 * Layout: shard i of object o lives at d_base + o*obj_stride + i*pitch, for
 * i in [0, data+parity), in either orientation:
 *   object-major ([object][shard]): obj_stride >= (data+parity)*pitch when
 *     nobj > 1, pitch >= shard_len;
 *   shard-major ([shard][object], each shard row holds every object's piece):
 *     shard_len <= obj_stride and pitch >= (nobj-1)*obj_stride + shard_len.
 *     A batch whose gaps between pieces are narrow (obj_stride <=
 *     roundup16(shard_len), or a gap of at most shard_len/4) is coded as one
 *     object whose shard is the whole row: the gap bytes are pad bytes and
 *     are overwritten in written rows, as are the row's bytes up to
 *     roundup16 of its last piece's end when the pitch holds them.
 * Any alignment (16-B aligned d_base, pitch and obj_stride are the fast path
 * and are required by the *_dev_masks calls).  Object size: the uniform
 * calls (rsgpu_{encode,verify,reconstruct,decode}_dev) take objects whose
 * rows span 4 GiB or more too, coded in column slabs through a scratch image
 * (two extra device copies per slab); the mixed-pattern calls require
 * (data+parity)*pitch < 4 GiB.
 * Kernels read whole 16-B vectors and write them where the layout allows:
 * written rows' bytes in [shard_len, min(space, roundup16(shard_len))), space
 * = the pitch (object-major) or obj_stride (shard-major), are overwritten
 * with the coding of the input rows' pad bytes (zero when those are zero);
 * with less space (e.g. pitch = shard_len, byte-packed rows) nothing past
 * shard_len is written.  `stream` is a hipStream_t (NULL = default stream);
 * calls are asynchronous on it and make no host<->device synchronisation.
 * HIP graphs: once a first call has built the code's plans (and, for the
 * *_dev_masks calls, the pattern atlas), rsgpu_{encode,verify,reconstruct,
 * decode}_dev and rsgpu_*_dev_masks issue only stream-ordered work and may be
 * captured into a graph and replayed (tests/test_gpu_graphs.py). */

/* Encode nobj objects: rows [k, k+p) <- M[k:] x rows [0, k). */
int rsgpu_encode_dev(rsgpu_ctx *ctx, void *d_base, size_t shard_len, size_t pitch,
                     size_t obj_stride, int nobj, void *stream);

/* Verify nobj objects: d_bad[o] (device, uint32) is set to 1 when object o's
 * parity mismatches, 0 otherwise. */
int rsgpu_verify_dev(rsgpu_ctx *ctx, const void *d_base, size_t shard_len, size_t pitch,
                     size_t obj_stride, int nobj, uint32_t *d_bad, void *stream);

/* Reconstruct nobj objects sharing one erasure pattern: present[i] (host,
 * data+parity bytes) != 0 marks row i present; missing rows are written in
 * place (parity rows too unless data_only). */
int rsgpu_reconstruct_dev(rsgpu_ctx *ctx, void *d_base, const uint8_t *present, size_t shard_len,
                          size_t pitch, size_t obj_stride, int nobj, int data_only, void *stream);

/* Fused decode (Reconstruct + Verify) of nobj objects sharing one pattern;
 * d_bad[o] = 1 when upstream's Verify-after-Reconstruct would fail for o. */
int rsgpu_decode_dev(rsgpu_ctx *ctx, void *d_base, const uint8_t *present, size_t shard_len,
                     size_t pitch, size_t obj_stride, int nobj, uint32_t *d_bad, void *stream);

/* Mixed erasure patterns (a batch of Gets, each with its own first-d
 * subset): present[o*(data+parity) + i] != 0 marks row i of object o present.
 * One launch per (K, R) class; each workgroup fetches its object's pass
 * (cached per pattern) through scalar loads.  Same per-object semantics as
 * rsgpu_reconstruct_dev / rsgpu_decode_dev (objects with every shard present
 * are skipped by reconstruct and verified by decode). */
int rsgpu_reconstruct_dev_multi(rsgpu_ctx *ctx, void *d_base, const uint8_t *present,
                                size_t shard_len, size_t pitch, size_t obj_stride, int nobj,
                                int data_only, void *stream);
int rsgpu_decode_dev_multi(rsgpu_ctx *ctx, void *d_base, const uint8_t *present, size_t shard_len,
                           size_t pitch, size_t obj_stride, int nobj, uint32_t *d_bad, void *stream);

/* Mixed erasure patterns with the arrival bitmaps already in HBM:
 * d_masks[o] (device, uint32) has bit i set when shard i of object o arrived
 * (bits >= data+parity ignored).  The pattern -> coefficient resolution runs
 * on the device against a per-context atlas of every erasure pattern, built
 * and uploaded on the first call: no per-call host planning, upload or host
 * synchronisation.  Codes of 17-32 shards (and codes whose atlas would pass
 * its size bound, e.g. data 2 + parity 14) have no atlas: the masks are read
 * back (one synchronisation of `stream`), grouped by pattern on the host and
 * coded by the host-planned mixed-pattern launches, with the same statuses.
 * More than 32 shards: RSGPU_ERR_NOT_IMPLEMENTED (masks are 32-bit words; the
 * host-flag *_dev_multi calls cover those codes).
 * d_status[o] (device uint32; optional for reconstruct) receives, per object:
 *   0  done (decode: upstream's Verify-after-Reconstruct would pass),
 *   1  decode only: that Verify would fail (ecRedis.go:420-426),
 *   2  fewer than data shards present (upstream ErrTooFewShards): untouched,
 *   3  survivors' matrix singular (upstream errSingular; non-MDS matrices): untouched.
 * Same per-object semantics as rsgpu_decode_dev / rsgpu_reconstruct_dev
 * (survivors = first data present shards in index order, as upstream). */
int rsgpu_decode_dev_masks(rsgpu_ctx *ctx, void *d_base, const uint32_t *d_masks, size_t shard_len,
                           size_t pitch, size_t obj_stride, int nobj, uint32_t *d_status, void *stream);
int rsgpu_reconstruct_dev_masks(rsgpu_ctx *ctx, void *d_base, const uint32_t *d_masks, size_t shard_len,
                                size_t pitch, size_t obj_stride, int nobj, int data_only,
                                uint32_t *d_status, void *stream);

/* ---- shard-major Get batches on whole lines ------------------------------
 * A Get batch of small objects decodes fastest shard-major through the
 * *_dev_masks calls with every piece on whole 128-B lines: at a 112-B stride
 * (1 KiB objects, shard_len 103) each rebuilt piece straddles two lines and
 * the decode runs at 41 % of HBM peak, at a 128-B stride it rewrites whole
 * lines.  (Replaces hand-laid batches behind
 * proxy/lambdastore/connection.go:274-306: every Get batch is mixed-pattern.)
 * rsgpu_shardmajor_layout returns that geometry for nobj pieces of shard_len
 * bytes: obj_stride = shard_len rounded up to 128 when the gap is at most
 * shard_len/4 (the encode still codes the batch as one object), else to 16;
 * pitch = nobj*obj_stride rounded up to 256. */
int rsgpu_shardmajor_layout(size_t shard_len, int nobj, size_t *obj_stride, size_t *pitch);
/* Device copy of the pieces of rows `rows` (bit i: row i; i < data+parity):
 * for every object o < nobj and such row i, shard_len bytes from
 * d_src + i*src_pitch + o*src_obj_stride to d_dst + i*dst_pitch +
 * o*dst_obj_stride, exactly (nothing else is written).  Either side may be
 * object-major or shard-major (the *_dev layouts above), at any alignment;
 * source and destination must not overlap.  Moves a batch into the
 * rsgpu_shardmajor_layout geometry before a *_dev_masks call (the rows that
 * arrived) and the rebuilt rows back after it.  Asynchronous on `stream`. */
int rsgpu_copy_pieces(rsgpu_ctx *ctx, const void *d_src, size_t src_pitch, size_t src_obj_stride, void *d_dst,
                      size_t dst_pitch, size_t dst_obj_stride, size_t shard_len, int nobj, uint64_t rows,
                      void *stream);

/* ---- variable-size device-resident batches ------------------------------
 * Objects of ANY sizes in one launch per pass (config 5's objects range from
 * 4 KiB to 100 MiB, client/ecRedis.go:96): objs[o] (a host array) describes
 * object o, shard i at base + i*pitch with pitch >= shard_len rounded up to
 * 16 (so no row's last 16-B vector reaches past the object's data+parity
 * rows); (data+parity)*pitch < 4 GiB.  Every object in device memory of one
 * device.  The table is uploaded by the library (a pinned ring, no per-call
 * allocation); the calls are asynchronous on `stream` like the *_dev calls,
 * with the same per-object semantics; d_bad[o] refers to objs[o]. */
typedef struct rsgpu_dev_obj {
    void *base;       /* device address of shard 0 of the object */
    size_t shard_len; /* bytes per shard of this object */
    size_t pitch;     /* bytes between its shard rows */
} rsgpu_dev_obj;

int rsgpu_encode_dev_objs(rsgpu_ctx *ctx, const rsgpu_dev_obj *objs, int nobj, void *stream);
int rsgpu_verify_dev_objs(rsgpu_ctx *ctx, const rsgpu_dev_obj *objs, int nobj, uint32_t *d_bad, void *stream);
/* one erasure pattern for every object: present[i] != 0 marks row i present */
int rsgpu_reconstruct_dev_objs(rsgpu_ctx *ctx, const rsgpu_dev_obj *objs, int nobj, const uint8_t *present,
                               int data_only, void *stream);
int rsgpu_decode_dev_objs(rsgpu_ctx *ctx, const rsgpu_dev_obj *objs, int nobj, const uint8_t *present,
                          uint32_t *d_bad, void *stream);

/* ---- batched host-memory API (pipelined H2D -> kernel -> D2H) ----------
 * The path starts and ends in host memory (ecRedis.go:96 Set buffer,
 * ecRedis.go:161-170 gathered Get buffers).  These calls stream a batch of
 * objects through the GPU over a ring of device slots / HIP streams so the
 * copies of one object overlap the kernel of another; they return when every
 * output is in host memory.  Host buffers should be pinned
 * (rsgpu_host_register / rsgpu_host_alloc) for the copies to run async.
 * Objects whose data+parity rows pass 1 GiB go through the per-object path
 * above (column slabs) in the same call. */

/* objs[o]: the Split() backing array of object o — data+parity rows of
 * shard_lens[o] bytes each, contiguous (pitch = shard length).  Parity rows
 * are written in place (Encode, ecRedis.go:390). */
int rsgpu_encode_batch(rsgpu_ctx *ctx, uint8_t *const *objs, const size_t *shard_lens, int nobj);

/* shards[o*(data+parity) + i]: buffer of shard i of object o (every entry
 * non-NULL: missing ones receive the reconstruction), present[same index] != 0
 * marks shards that arrived.  Fused Client.decode per object (ecRedis.go:404-
 * 427): missing shards written, ok[o] = Verify-after-Reconstruct result. */
int rsgpu_decode_batch(rsgpu_ctx *ctx, uint8_t *const *shards, const uint8_t *present,
                       const size_t *shard_lens, int nobj, int *ok);

/* Pinned host memory helpers (hipHostRegister / hipHostMalloc; alloc takes
 * Mapped | Coherent pages, RSGPU_HOST_ALLOC=default the runtime's default
 * kind).  hipHostFree / hipHostUnregister wait for every kernel of the
 * device, a resident worker's too: with no worker kernel resident they run at
 * once; otherwise unregister parks the workers around the call and free is
 * deferred to the next moment no worker kernel is resident (at most 256 MiB
 * held; past that it parks the workers too). */
int rsgpu_host_register(void *p, size_t len);
int rsgpu_host_unregister(void *p);
int rsgpu_host_alloc(size_t len, void **out);
int rsgpu_host_free(void *p);

/* ---- diagnostics and test knobs ------------------------------------------
 * Library buffers whose free is being held back because a worker kernel is
 * resident (count, bytes) and the number of frees ever held back. */
int rsgpu_retired_stats(size_t *count, size_t *bytes, uint64_t *deferred);
/* Staged bytes per object above which the per-object host calls code in
 * column slabs (default 1 GiB; RSGPU_SLAB_BYTES at first use).  bytes < 4096
 * restores the default.  Process-wide; set it while no call is in flight. */
int rsgpu_set_slab_bytes(size_t bytes);

#ifdef __cplusplus
}
#endif
#endif /* RSGPU_H */
