/* c_abi_stress.c — many threads on one context, every per-object route at
 * once, checked byte for byte: the host-side concurrency of the library
 * (staging slots that grow, the resident worker's mailboxes and column
 * slices, the reader epochs that park workers around rsgpu_host_free, the
 * host copy pool) under ThreadSanitizer or ASan/UBSan, with the kernels
 * running.  Built by tests/test_sanitize.py against tools/san/librsgpu_{t,}san.so.
 *
 * The Go client this stands in for runs one goroutine per EcSet / EcGet
 * (client/ecRedis.go:96, :173), so concurrent Client.encode / Client.decode
 * calls on one encoder (client/ec.go:14-24, one per Client) are its normal
 * load.  Each thread loops: pick a route, fill a random object, fused
 * encode+verify (Client.encode, ecRedis.go:390-395), compare parity with the
 * CPU oracle (orc_encode), drop up to `parity` random shards, fused decode
 * (Client.decode, ecRedis.go:404-427), compare every rebuilt row.
 *
 *   c_abi_stress <threads> <seconds> [seed [data parity [matrix kind]]]
 *
 * Routes (RS(10+2) unless given, worker on with 16 mailboxes, max_shard 4 KiB;
 * object sizes below are for RS(10+2), the shard lengths are the same for
 * every code):
 *   0  1 KiB object, pageable pointer table     -> worker, mailbox image
 *   1  1 KiB object, pinned Split image         -> worker, in place
 *   2  100 KiB object, pinned Split image       -> worker column slices in place
 *   3  100 KiB object, pageable pointer table   -> worker slices staged
 *   4  2-6 MiB object, pageable pointer table   -> stream path, slots grow
 *   5  13-17 MiB object, pageable               -> stream path + host copy pool
 *   6  pinned image allocated and freed per call -> parks the worker (host_free)
 * Routes 1 and 2 reuse one pinned image per thread (grown when too small), as
 * a client that keeps its buffers does; route 6 is the rare caller that frees.
 * The CPU oracle is test infrastructure (the checker), never the thing run. */
#define _POSIX_C_SOURCE 199309L
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "rsgpu.h"

int orc_encode(int k, int p, int kind, uint8_t *const *shards, const size_t *lens, int nshards);

enum { MAXN = 16, ROUTES = 7 };
static int K = 10, P = 2, N = 12; /* the code (argv 4, 5): data + parity <= 16 */
static unsigned KIND = RSGPU_MATRIX_VANDERMONDE; /* argv 6: 0 Vandermonde, 1 Cauchy */

static rsgpu_ctx *ctx;
static double deadline;
static uint64_t seed0 = 1;
static long counts[ROUTES];
static pthread_mutex_t count_mu = PTHREAD_MUTEX_INITIALIZER;

static double now_s(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + t.tv_nsec * 1e-9;
}

static uint64_t next(uint64_t *s) {
    *s ^= *s << 13;
    *s ^= *s >> 7;
    *s ^= *s << 17;
    return *s;
}

#define FAIL(...)                                                      \
    do {                                                               \
        fprintf(stderr, "route %d S=%zu: ", route, S);                \
        fprintf(stderr, __VA_ARGS__);                                  \
        fprintf(stderr, "\n");                                         \
        return 1;                                                      \
    } while (0)

/* one Client.encode + Client.decode round on the rows rows[0..N) of S bytes */
static int one_object(int route, size_t S, uint8_t **rows, int image, uint64_t *rng) {
    size_t lens[MAXN];
    uint8_t *ref[MAXN];
    for (int i = 0; i < N; i++) {
        lens[i] = S;
        ref[i] = malloc(S ? S : 1);
        if (!ref[i]) FAIL("malloc");
    }
    for (int i = 0; i < K; i++) {
        uint64_t x = next(rng);
        for (size_t j = 0; j < S; j++) {
            x = x * 6364136223846793005ull + 1442695040888963407ull;
            rows[i][j] = ref[i][j] = (uint8_t)(x >> 56);
        }
    }
    for (int i = K; i < N; i++) memset(rows[i], 0xEE, S), memset(ref[i], 0, S);
    int ok = 7, rc;
    rc = image ? rsgpu_encode_verify_image(ctx, rows[0], S, N, &ok) : rsgpu_encode_verify(ctx, rows, lens, N, &ok);
    if (rc != RSGPU_OK || ok != 1) FAIL("encode_verify rc=%d ok=%d", rc, ok);
    if (orc_encode(K, P, (int)KIND, ref, lens, N)) FAIL("oracle");
    for (int i = K; i < N; i++)
        if (memcmp(rows[i], ref[i], S)) FAIL("parity row %d differs from the oracle", i);
    /* drop up to P shards, scribble over them, decode */
    uint64_t present = (1ull << N) - 1;
    const int drop = (int)(next(rng) % (P + 1));
    for (int d = 0; d < drop; d++) {
        const int i = (int)(next(rng) % N);
        present &= ~(1ull << i);
        memset(rows[i], 0x5A, S);
    }
    for (int i = 0; i < N; i++) lens[i] = (present >> i & 1) ? S : 0;
    ok = 7;
    rc = image ? rsgpu_decode_image(ctx, rows[0], S, N, present, &ok) : rsgpu_decode(ctx, rows, lens, N, &ok);
    if (rc != RSGPU_OK || ok != 1) FAIL("decode rc=%d ok=%d present=%llx", rc, ok, (unsigned long long)present);
    for (int i = 0; i < N; i++)
        if (memcmp(rows[i], ref[i], S)) FAIL("row %d wrong after decode (present %llx)", i, (unsigned long long)present);
    for (int i = 0; i < N; i++) free(ref[i]);
    return 0;
}

static int one_round(int route, uint64_t *rng, uint8_t **img, size_t *img_cap) {
    size_t S;
    switch (route) {
        case 0: case 1: S = 103; break;                                   /* 1 KiB object */
        case 2: case 3: S = 10240 + (next(rng) % 64) * 16; break;          /* ~100 KiB */
        case 4: S = (200u << 10) + (size_t)(next(rng) % (400u << 10)); break;    /* 2-6 MiB */
        case 5: S = (1300u << 10) + (size_t)(next(rng) % (400u << 10)); break;   /* 13-17 MiB */
        default: S = 1 + (size_t)(next(rng) % 4096); break;
    }
    uint8_t *rows[MAXN];
    int rc;
    if (route == 1 || route == 2) {  /* the thread's own pinned image, kept across calls */
        if (*img_cap < N * S) {
            if (*img && rsgpu_host_free(*img) != RSGPU_OK) FAIL("host_free");
            *img = NULL;
            if (rsgpu_host_alloc(N * S, (void **)img) != RSGPU_OK) FAIL("host_alloc");
            *img_cap = N * S;
        }
        for (int i = 0; i < N; i++) rows[i] = *img + i * S;
        rc = one_object(route, S, rows, 1, rng);
    } else if (route == 6) {
        /* allocated and freed around the call: rsgpu_host_free parks the worker */
        uint8_t *tmp = NULL;
        if (rsgpu_host_alloc(N * S, (void **)&tmp) != RSGPU_OK) FAIL("host_alloc");
        for (int i = 0; i < N; i++) rows[i] = tmp + i * S;
        rc = one_object(route, S, rows, 1, rng);
        if (rsgpu_host_free(tmp) != RSGPU_OK) FAIL("host_free");
    } else {
        for (int i = 0; i < N; i++) rows[i] = malloc(S);
        rc = one_object(route, S, rows, 0, rng);
        for (int i = 0; i < N; i++) free(rows[i]);
    }
    return rc;
}

static void *thread_main(void *arg) {
    const long id = (long)arg;
    uint64_t rng = seed0 * 0x9E3779B97F4A7C15ull + (uint64_t)id * 7919 + 1;
    long mine[ROUTES] = {0};
    long rc = 0;
    uint8_t *img = NULL;
    size_t img_cap = 0;
    while (!rc && now_s() < deadline) {
        /* the large routes are rare: they dominate the bytes */
        const uint64_t r = next(&rng) % 40;
        const int route = r < 12 ? 0 : r < 22 ? 1 : r < 29 ? 2 : r < 35 ? 3 : r < 38 ? 4 : r < 39 ? 5 : 6;
        rc = one_round(route, &rng, &img, &img_cap);
        mine[route]++;
    }
    if (img) rsgpu_host_free(img);
    pthread_mutex_lock(&count_mu);
    for (int i = 0; i < ROUTES; i++) counts[i] += mine[i];
    pthread_mutex_unlock(&count_mu);
    return (void *)rc;
}

int main(int argc, char **argv) {
    const int threads = argc > 1 ? atoi(argv[1]) : 8;
    const double seconds = argc > 2 ? atof(argv[2]) : 10;
    if (argc > 3) seed0 = strtoull(argv[3], NULL, 10);
    if (argc > 5) {
        K = atoi(argv[4]);
        P = atoi(argv[5]);
        N = K + P;
        if (K < 1 || P < 1 || N > MAXN) return fprintf(stderr, "code must have 1 <= data, parity and data+parity <= 16\n"), 2;
    }
    /* PAR1 is not MDS (some erasure patterns are singular): not a stress kind */
    if (argc > 6) KIND = (unsigned)atoi(argv[6]);
    if (KIND > RSGPU_MATRIX_CAUCHY) return fprintf(stderr, "matrix kind must be 0 or 1\n"), 2;
    if (rsgpu_create(K, P, 0, KIND, &ctx) != RSGPU_OK) return fprintf(stderr, "create failed\n"), 1;
    if (rsgpu_worker_start(ctx, 16, 0, 0) != RSGPU_OK) return fprintf(stderr, "worker_start failed\n"), 1;
    deadline = now_s() + seconds;
    pthread_t th[64];
    const int nt = threads < 1 ? 1 : threads > 64 ? 64 : threads;
    for (long i = 0; i < nt; i++) pthread_create(&th[i], NULL, thread_main, (void *)i);
    /* the frees the library holds back while the worker kernel is resident
     * (devmem.cpp) stay bounded: 256 MiB plus what one call can retire */
    size_t peak = 0, cnt = 0, bytes = 0;
    uint64_t deferred = 0;
    while (now_s() < deadline) {
        rsgpu_retired_stats(&cnt, &bytes, &deferred);
        if (bytes > peak) peak = bytes;
        const struct timespec ts = {0, 5000000};
        nanosleep(&ts, NULL);
    }
    long bad = 0;
    for (int i = 0; i < nt; i++) {
        void *r;
        pthread_join(th[i], &r);
        bad |= (long)r;
    }
    uint64_t served = 0, declined = 0, launches = 0;
    rsgpu_worker_stats(ctx, &served, &declined, &launches);
    rsgpu_destroy(ctx);
    rsgpu_retired_stats(&cnt, &bytes, &deferred);
    printf("retired: peak %.1f MiB held, %llu frees held back in all, %zu held after destroy\n",
           peak / 1048576.0, (unsigned long long)deferred, cnt);
    if (peak > ((size_t)320 << 20) || cnt != 0) {
        fprintf(stderr, "held-back frees unbounded or left over after the worker stopped\n");
        bad = 1;
    }
    long total = 0;
    for (int i = 0; i < ROUTES; i++) total += counts[i];
    printf("stress: RS(%d+%d)%s, %d threads, %.0f s, %ld objects (routes:", K, P, KIND ? " Cauchy" : "", nt, seconds,
           total);
    for (int i = 0; i < ROUTES; i++) printf(" %ld", counts[i]);
    printf("), worker served %llu declined %llu launches %llu: %s\n", (unsigned long long)served,
           (unsigned long long)declined, (unsigned long long)launches, bad ? "FAILED" : "all bit-exact");
    fflush(stdout);
#if defined(__has_feature)
#if __has_feature(address_sanitizer)
    /* every context is destroyed and no worker runs: under ASan the process
     * ends here, before the HIP runtime's own static destruction, where ASan's
     * device-allocation tracking aborts when its quarantine recycles a device
     * chunk after the runtime has unloaded (a CHECK in
     * sanitizer_allocator_device.h, seen once in round 6 inside libamdhip64's
     * __cxa_finalize; outside this library).  c_abi_client.c keeps the normal
     * exit, including the exit with a resident worker. */
    _exit(bad ? 1 : 0);
#endif
#endif
    return bad ? 1 : 0;
}
