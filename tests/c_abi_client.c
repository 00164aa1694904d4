/* c_abi_client.c — a plain-C consumer of include/rsgpu.h, exercising the
 * boundary the way the cgo shim would: create, per-object
 * Encode / Verify / Reconstruct / decode with caller-owned host buffers,
 * error codes.  Built by tests/test_c_abi.py with gcc against librsgpu.so and
 * the CPU oracle (oracle/liboracle.so, the checker).
 *
 *   ./c_abi_client host      # no device needed: create/matrix/error paths
 *   ./c_abi_client gpu       # + compute, checked byte-for-byte vs the oracle
 * Exit code 0 = pass. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "rsgpu.h"

/* oracle entry points (oracle/rs_oracle.c) */
int orc_build_matrix(int k, int p, int kind, uint8_t *out);
int orc_encode(int k, int p, int kind, uint8_t *const *shards, const size_t *lens, int nshards);

#define CHECK(c)                                                         \
    do {                                                                 \
        if (!(c)) {                                                      \
            fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
            return 1;                                                    \
        }                                                                \
    } while (0)

static uint64_t rng = 0x1F1C;
static uint8_t rnd8(void) {
    rng = rng * 6364136223846793005ull + 1442695040888963407ull;
    return (uint8_t)(rng >> 56);
}

static int host_checks(void) {
    rsgpu_ctx *ctx = NULL;
    CHECK(rsgpu_create(0, 2, 0, 0, &ctx) == RSGPU_ERR_INV_SHARD_NUM && ctx == NULL);
    CHECK(rsgpu_create(200, 57, 0, 0, &ctx) == RSGPU_ERR_MAX_SHARD_NUM);
    CHECK(rsgpu_create(10, 2, 0, 99, &ctx) == RSGPU_ERR_INVALID_ARG);
    CHECK(rsgpu_create(10, 2, 0, RSGPU_MATRIX_VANDERMONDE, &ctx) == RSGPU_OK && ctx);
    CHECK(rsgpu_data_shards(ctx) == 10 && rsgpu_parity_shards(ctx) == 2);
    uint8_t m[12 * 10], want[12 * 10];
    CHECK(rsgpu_matrix(ctx, m) == RSGPU_OK);
    CHECK(orc_build_matrix(10, 2, 0, want) == 0);
    CHECK(memcmp(m, want, sizeof m) == 0);
    /* upstream error precedence, no device needed */
    uint8_t a[8] = {0};
    uint8_t *sh[12];
    size_t lens[12];
    for (int i = 0; i < 12; i++) { sh[i] = a; lens[i] = 8; }
    CHECK(rsgpu_encode(ctx, sh, lens, 11) == RSGPU_ERR_TOO_FEW_SHARDS);
    lens[11] = 0;
    CHECK(rsgpu_encode(ctx, sh, lens, 12) == RSGPU_ERR_SHARD_SIZE);
    int ok = 7;
    CHECK(rsgpu_verify(ctx, (const uint8_t *const *)sh, lens, 12, &ok) == RSGPU_ERR_SHARD_SIZE && ok == 0);
    for (int i = 0; i < 12; i++) lens[i] = 0;
    CHECK(rsgpu_encode(ctx, sh, lens, 12) == RSGPU_ERR_SHARD_NO_DATA);
    for (int i = 0; i < 12; i++) lens[i] = i < 9 ? 8 : 0;
    CHECK(rsgpu_reconstruct(ctx, sh, lens, 12, 0) == RSGPU_ERR_TOO_FEW_SHARDS);
    CHECK(strlen(rsgpu_strerror(RSGPU_ERR_SHARD_SIZE)) > 0);
    /* the image calls: one base pointer, same checks */
    CHECK(rsgpu_encode_image(ctx, a, 8, 11) == RSGPU_ERR_TOO_FEW_SHARDS);
    CHECK(rsgpu_encode_image(ctx, NULL, 8, 12) == RSGPU_ERR_INVALID_ARG);
    CHECK(rsgpu_reconstruct_image(ctx, a, 8, 12, 0x1ff, 0) == RSGPU_ERR_TOO_FEW_SHARDS);
    CHECK(rsgpu_encode_image(ctx, a, 0, 12) == RSGPU_ERR_SHARD_NO_DATA);
    rsgpu_destroy(ctx);
    int devs[2] = {0, 0};
    uint64_t calls[2] = {7, 7};
    /* a device listed twice: two independent entries, no calls yet */
    CHECK(rsgpu_create_multi(10, 2, devs, 2, 0, &ctx) == RSGPU_OK && rsgpu_devices(ctx, devs, 2) == 2);
    CHECK(rsgpu_device_calls(ctx, calls, 2) == 2 && calls[0] == 0 && calls[1] == 0);
    rsgpu_destroy(ctx);
    CHECK(rsgpu_create_multi(10, 2, NULL, 2, 0, &ctx) == RSGPU_ERR_INVALID_ARG && ctx == NULL);
    CHECK(rsgpu_create(10, 2, RSGPU_ALL_DEVICES, 0, &ctx) == RSGPU_OK && rsgpu_devices(ctx, devs, 2) >= 1);
    rsgpu_destroy(ctx);
    printf("host checks ok (devices: %d)\n", rsgpu_device_count());
    return 0;
}

static int gpu_checks(void) {
    const int k = 10, p = 4, n = 14;
    const size_t S = 104858;  /* 1 MiB object / 10, as Split makes it */
    rsgpu_ctx *ctx;
    CHECK(rsgpu_create(k, p, 0, 0, &ctx) == RSGPU_OK);
    CHECK(rsgpu_device_ok(0) == 1);
    uint8_t *mine[14], *ref[14];
    size_t lens[14];
    for (int i = 0; i < n; i++) {
        mine[i] = malloc(S);
        ref[i] = malloc(S);
        lens[i] = S;
        for (size_t j = 0; j < S; j++) mine[i][j] = ref[i][j] = i < k ? rnd8() : 0;
    }
    CHECK(rsgpu_encode(ctx, mine, lens, n) == RSGPU_OK);
    CHECK(orc_encode(k, p, 0, ref, lens, n) == 0);
    for (int i = k; i < n; i++) CHECK(memcmp(mine[i], ref[i], S) == 0);
    int ok = 0;
    CHECK(rsgpu_verify(ctx, (const uint8_t *const *)mine, lens, n, &ok) == RSGPU_OK && ok == 1);
    mine[12][S - 1] ^= 1;
    CHECK(rsgpu_verify(ctx, (const uint8_t *const *)mine, lens, n, &ok) == RSGPU_OK && ok == 0);
    mine[12][S - 1] ^= 1;
    /* lose data 0, 7 and parity 11: buffers supplied by the caller, len 0 */
    int lost[3] = {0, 7, 11};
    for (int j = 0; j < 3; j++) { memset(mine[lost[j]], 0xEE, S); lens[lost[j]] = 0; }
    CHECK(rsgpu_reconstruct(ctx, mine, lens, n, 0) == RSGPU_OK);
    for (int i = 0; i < n; i++) CHECK(memcmp(mine[i], ref[i], S) == 0);
    /* fused Client.decode with one extra present shard corrupted */
    for (int i = 0; i < n; i++) lens[i] = S;
    lens[3] = 0;
    memset(mine[3], 0, S);
    mine[13][5] ^= 0x10;  /* 13 present: survivors 0..12 except 3, extra = 13 */
    CHECK(rsgpu_decode(ctx, mine, lens, n, &ok) == RSGPU_OK && ok == 0);
    CHECK(memcmp(mine[3], ref[3], S) == 0);
    /* pinned Split buffer (rsgpu_host_alloc): direct DMA both ways; lost
     * shards keep their pinned buffers with len 0, as the cgo shim passes a
     * slice with capacity */
    uint8_t *pb = NULL;
    CHECK(rsgpu_host_alloc(n * S, (void **)&pb) == RSGPU_OK && pb);
    uint8_t *ps[14];
    for (int i = 0; i < n; i++) {
        ps[i] = pb + i * S;
        memcpy(ps[i], i < k ? ref[i] : mine[0], S);
        if (i >= k) memset(ps[i], 0, S);
        lens[i] = S;
    }
    CHECK(rsgpu_encode(ctx, ps, lens, n) == RSGPU_OK);
    for (int i = k; i < n; i++) CHECK(memcmp(ps[i], ref[i], S) == 0);
    CHECK(rsgpu_verify(ctx, (const uint8_t *const *)ps, lens, n, &ok) == RSGPU_OK && ok == 1);
    /* Client.encode fused: Encode then Verify in one device round trip */
    for (int i = k; i < n; i++) memset(ps[i], 0x11, S);
    ok = 0;
    CHECK(rsgpu_encode_verify(ctx, ps, lens, n, &ok) == RSGPU_OK && ok == 1);
    for (int i = k; i < n; i++) CHECK(memcmp(ps[i], ref[i], S) == 0);
    int plost[4] = {2, 3, 9, 12};
    for (int j = 0; j < 4; j++) { memset(ps[plost[j]], 0x77, S); lens[plost[j]] = 0; }
    CHECK(rsgpu_reconstruct(ctx, ps, lens, n, 0) == RSGPU_OK);
    for (int i = 0; i < n; i++) CHECK(memcmp(ps[i], ref[i], S) == 0);
    for (int i = 0; i < n; i++) lens[i] = S;
    lens[6] = lens[7] = 0;
    memset(ps[6], 0, S);
    memset(ps[7], 0, S);
    CHECK(rsgpu_decode(ctx, ps, lens, n, &ok) == RSGPU_OK && ok == 1);
    CHECK(memcmp(ps[6], ref[6], S) == 0 && memcmp(ps[7], ref[7], S) == 0);
    CHECK(rsgpu_host_free(pb) == RSGPU_OK);
    for (int i = 0; i < n; i++) { free(mine[i]); free(ref[i]); }
    rsgpu_destroy(ctx);
    printf("gpu checks ok (RS(10+4), S=%zu, bit-exact vs oracle, pageable and pinned)\n", S);
    return 0;
}

/* ecredis_replay: client/ecRedis.go:382-432 in its exact call order, through
 * the routes the Go shim (integration/go/client/ec_gpu.go) takes so that only
 * cgo-legal pointers cross:
 *   Client.encode: Split into ONE contiguous array (route i: the *_image
 *   calls take its base), Encode, Verify (false -> error).
 *   Client.decode over EcGet's 12 separate buffers, 2 of them nil (the
 *   proxy's first-d rule): Verify -> (false, ErrShardSize) with no device
 *   work (:406; the shim answers it in Go); Reconstruct through a C-owned
 *   pinned image (route ii), rebuilt shards copied out; Verify -> true, which
 *   upstream stores in stats.Corrupted (true on SUCCESS, :420-426); Join.
 *   Then a Get whose extra present parity shard is corrupted: Reconstruct
 *   succeeds, the second Verify is false -> decode's error path.  The fused
 *   forms (rsgpu_encode_verify_image, rsgpu_decode_image) give the same
 *   booleans and bytes.
 * p = 2: the client's own RS(10+2).  p = 4: BASELINE config 3's RS(10+4) Get
 * (data shard 3 and parity 10 lost: 12 of 14 present, 2 extra shards the
 * second Verify checks; then 13 present with the last shard corrupted). */
static int ecredis_replay(size_t N, int worker, int p) {
    const int k = 10, n = k + p;
    const size_t S = (N + k - 1) / k;
    rsgpu_ctx *ctx;
    CHECK(rsgpu_create(k, p, RSGPU_ALL_DEVICES, 0, &ctx) == RSGPU_OK);
    /* the resident worker serves the same calls (rsgpu_worker_start) */
    if (worker) CHECK(rsgpu_worker_start(ctx, 4, 0, 0) == RSGPU_OK);
    uint8_t *obj = malloc(N);
    for (size_t j = 0; j < N; j++) obj[j] = rnd8();
    /* ---- Client.encode (ecRedis.go:382-402) */
    uint8_t *split = calloc(n, S); /* Split: perShard = ceil(N/k), zero pad */
    memcpy(split, obj, N);
    CHECK(rsgpu_encode_image(ctx, split, S, n) == RSGPU_OK);
    int ok = 0;
    CHECK(rsgpu_verify_image(ctx, split, S, n, &ok) == RSGPU_OK && ok == 1);
    uint8_t *ref[16];
    size_t lens[16];
    for (int i = 0; i < n; i++) {
        ref[i] = malloc(S);
        memcpy(ref[i], split + i * S, S);
        lens[i] = S;
    }
    for (int i = k; i < n; i++) memset(ref[i], 0, S);
    CHECK(orc_encode(k, p, 0, ref, lens, n) == 0);
    for (int i = k; i < n; i++) CHECK(memcmp(ref[i], split + i * S, S) == 0);
    uint8_t *split2 = calloc(n, S);
    memcpy(split2, obj, N);
    CHECK(rsgpu_encode_verify_image(ctx, split2, S, n, &ok) == RSGPU_OK && ok == 1);
    CHECK(memcmp(split, split2, n * S) == 0);
    /* ---- Client.decode (ecRedis.go:404-432): 12 separate Get buffers */
    for (int trial = 0; trial < 2; trial++) {
        const int lost[2] = {3, 10};
        uint8_t *got[16];
        for (int i = 0; i < n; i++) {
            got[i] = (i == lost[0] || i == lost[1]) ? NULL : malloc(S);
            lens[i] = got[i] ? S : 0;
            if (got[i]) memcpy(got[i], split + i * S, S);
        }
        if (trial == 1) {  /* shard 10 arrives too; the last extra shard (n - 1) is corrupted */
            got[10] = malloc(S);
            memcpy(got[10], split + 10 * S, S);
            lens[10] = S;
            got[n - 1][S / 2] ^= 0x20;
        }
        /* stats.AllGood, _ = Verify(data): nil shards -> (false, ErrShardSize) */
        ok = 7;
        CHECK(rsgpu_verify(ctx, (const uint8_t *const *)got, lens, n, &ok) == RSGPU_ERR_SHARD_SIZE && ok == 0);
        /* Reconstruct(data): stage the present shards in a C-owned pinned image */
        uint8_t *img = NULL;
        CHECK(rsgpu_host_alloc(n * S, (void **)&img) == RSGPU_OK);
        uint64_t present = 0;
        for (int i = 0; i < n; i++)
            if (lens[i]) {
                memcpy(img + i * S, got[i], S);
                present |= 1ull << i;
            }
        CHECK(rsgpu_reconstruct_image(ctx, img, S, n, present, 0) == RSGPU_OK);
        for (int i = 0; i < n; i++)
            if (!lens[i]) {  /* upstream allocates the missing shard */
                got[i] = malloc(S);
                memcpy(got[i], img + i * S, S);
                lens[i] = S;
            }
        /* stats.Corrupted, err = Verify(data): true on success (:420) */
        int corrupted = 0;
        CHECK(rsgpu_verify(ctx, (const uint8_t *const *)got, lens, n, &corrupted) == RSGPU_OK);
        if (trial == 0) {
            CHECK(corrupted == 1);
            /* Join: the first N bytes of the data shards */
            for (int i = 0; i < k; i++) {
                const size_t off = (size_t)i * S, len = off + S <= N ? S : (off < N ? N - off : 0);
                CHECK(memcmp(got[i], obj + off, len) == 0);
            }
        } else {
            CHECK(corrupted == 0);  /* decode returns the error */
        }
        /* the fused decode gives the same boolean and bytes */
        uint8_t *img2 = NULL;
        CHECK(rsgpu_host_alloc(n * S, (void **)&img2) == RSGPU_OK);
        uint64_t pres2 = 0;
        for (int i = 0; i < n; i++)
            if (i != lost[0] && (i != lost[1] || trial == 1)) {
                memcpy(img2 + i * S, i == n - 1 && trial == 1 ? got[n - 1] : split + i * S, S);
                pres2 |= 1ull << i;
            }
        int fused_ok = 7;
        CHECK(rsgpu_decode_image(ctx, img2, S, n, pres2, &fused_ok) == RSGPU_OK);
        CHECK(fused_ok == corrupted);
        CHECK(memcmp(img2 + lost[0] * S, split + lost[0] * S, S) == 0);
        CHECK(rsgpu_host_free(img) == RSGPU_OK && rsgpu_host_free(img2) == RSGPU_OK);
        for (int i = 0; i < n; i++) free(got[i]);
    }
    for (int i = 0; i < n; i++) free(ref[i]);
    free(split);
    free(split2);
    free(obj);
    if (worker) {
        uint64_t served = 0, declined = 0, launches = 0;
        CHECK(rsgpu_worker_stats(ctx, &served, &declined, &launches) == RSGPU_OK);
        CHECK(served >= 9 && launches >= 1);  /* 3 encode-side + 3 per Get trial */
        printf("worker: %llu calls served, %llu launches\n", (unsigned long long)served, (unsigned long long)launches);
    }
    rsgpu_destroy(ctx);
    printf("ecredis replay ok (RS(10+%d), %zu-B object%s; Client.encode/decode call order, contiguous and staged "
           "routes)\n", p, N, worker ? ", resident worker" : "");
    return 0;
}

/* A host that exits with the resident worker still running and without
 * rsgpu_destroy (a Go client process simply ends): the library's exit guard
 * must stop the worker before the HIP runtime tears down.  With
 * RSGPU_WORKER_TRACE set, worker_stop's trace line on stderr shows that it
 * ran at exit. */
static int exit_with_worker(void) {
    const int k = 10, n = 12;
    const size_t S = 103;
    rsgpu_ctx *ctx = NULL;
    CHECK(rsgpu_create(k, 2, 0, 0, &ctx) == RSGPU_OK);
    CHECK(rsgpu_worker_start(ctx, 2, 10000000u, 0) == RSGPU_OK); /* 10 s idle: running at exit */
    uint8_t *buf[12], *ref[12];
    size_t lens[12];
    for (int i = 0; i < n; i++) {
        buf[i] = calloc(S, 1);
        ref[i] = calloc(S, 1);
        lens[i] = S;
        for (size_t j = 0; i < k && j < S; j++) buf[i][j] = ref[i][j] = rnd8();
    }
    int ok = 0;
    CHECK(rsgpu_encode_verify(ctx, buf, lens, n, &ok) == RSGPU_OK && ok == 1);
    CHECK(orc_encode(k, 2, 0, ref, lens, n) == 0);
    for (int i = 0; i < n; i++) CHECK(memcmp(buf[i], ref[i], S) == 0);
    uint64_t served = 0;
    CHECK(rsgpu_worker_stats(ctx, &served, NULL, NULL) == RSGPU_OK && served == 1);
    printf("exit with the worker running\n");
    fflush(stdout);
    return 0; /* no rsgpu_worker_stop, no rsgpu_destroy */
}

int main(int argc, char **argv) {
    if (argc > 1 && strcmp(argv[1], "exit_with_worker") == 0) return exit_with_worker();
    if (host_checks()) return 1;
    if (argc > 1 && strcmp(argv[1], "gpu") == 0)
        return gpu_checks() || ecredis_replay(1 << 20, 0, 2) || ecredis_replay(1024, 1, 2) ||
               ecredis_replay(4 << 20, 0, 4);
    return 0;
}
