/* lat_bench.c — per-object latency of the host-buffer C ABI, as the cgo shim
 *  drives it for one EcSet / EcGet: Client.encode = Encode +
 * Verify (separate calls, and fused: rsgpu_encode_verify), Client.decode =
 * Reconstruct + Verify (fused, rsgpu_decode), RS(10+2) objects of
 * LAT_BYTES bytes (default 1 MiB; client/example/main.go uses 1 KiB), shards
 * as Split lays them out (one contiguous buffer).
 *
 *   [LAT_BYTES=N] [LAT_WORKER=nslots] ./lat_bench [iters [concurrent_seconds]]
 *
 * LAT_WORKER=nslots: the per-object calls go through the resident worker
 * (rsgpu_worker_start with nslots mailboxes) instead of the stream path;
 * LAT_MAX_SHARD sets its max_shard.
 *
 * Prints p50/p99 in microseconds for pageable (malloc) and pinned
 * (rsgpu_host_alloc) buffers.  No Python in the process. */
#define _POSIX_C_SOURCE 199309L
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>
#include <time.h>

#include "rsgpu.h"

static double now_us(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e6 + t.tv_nsec * 1e-3;
}

static int cmp(const void *a, const void *b) {
    double x = *(const double *)a, y = *(const double *)b;
    return x < y ? -1 : x > y;
}

static size_t obj_bytes(void) {
    const char *e = getenv("LAT_BYTES");
    return e && atol(e) > 0 ? (size_t)atol(e) : (size_t)1 << 20;
}

static double pct(double *v, int n, double p) {
    qsort(v, n, sizeof(double), cmp);
    int i = (int)(p * (n - 1) + 0.5);
    return v[i];
}

/* Concurrent callers (many EcSet/EcGet in flight, as a client serving many
 * requests would issue): T threads, each with its own pinned Split buffer,
 * run fused encode+verify then decode on 1 MiB objects for `secs` seconds;
 * prints the aggregate object rate. */
struct conc_arg {
    rsgpu_ctx *ctx;
    double secs;
    long done;
    int err;
};

static void *conc_worker(void *vp) {
    struct conc_arg *a = (struct conc_arg *)vp;
    const int k = 10, p = 2, n = k + p;
    const size_t nb = obj_bytes(), S = (nb + k - 1) / k;
    uint8_t *buf = NULL;
    if (rsgpu_host_alloc(n * S, (void **)&buf)) { a->err = 1; return NULL; }
    for (size_t i = 0; i < k * S; ++i) buf[i] = (uint8_t)(i * 131 + 7);
    uint8_t *sh[12];
    size_t lens[12];
    for (int i = 0; i < n; ++i) sh[i] = buf + i * S;
    const double t0 = now_us();
    while (now_us() - t0 < a->secs * 1e6) {
        int ok = 0;
        for (int i = 0; i < n; ++i) lens[i] = S;
        if (rsgpu_encode_verify(a->ctx, sh, lens, n, &ok) || !ok) { a->err = 2; break; }
        lens[0] = lens[5] = 0;
        if (rsgpu_decode(a->ctx, sh, lens, n, &ok) || !ok) { a->err = 3; break; }
        a->done += 1;
    }
    rsgpu_host_free(buf);
    return NULL;
}

static int concurrent(rsgpu_ctx *ctx, int threads, double secs) {
    pthread_t th[64];
    struct conc_arg args[64];
    if (threads > 64) threads = 64;
    const double t0 = now_us();
    for (int t = 0; t < threads; ++t) {
        args[t] = (struct conc_arg){ctx, secs, 0, 0};
        pthread_create(&th[t], NULL, conc_worker, &args[t]);
    }
    long done = 0;
    int err = 0;
    for (int t = 0; t < threads; ++t) {
        pthread_join(th[t], NULL);
        done += args[t].done;
        err |= args[t].err;
    }
    const double el = (now_us() - t0) * 1e-6;
    printf("concurrent %2d threads: %7.0f objects/s (encode+verify and decode each), %6.2f GiB/s of object "
           "bytes per op pair%s\n", threads, done / el, 2.0 * done * (double)obj_bytes() / el / (1 << 30),
           err ? "  ERROR" : "");
    return err;
}

int main(int argc, char **argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 200, warm = 10;
    const int k = 10, p = 2, n = k + p;
    const size_t nb = obj_bytes(), S = (nb + k - 1) / k;
    rsgpu_ctx *ctx;
    printf("object %zu B (S = %zu)\n", nb, S);
    if (rsgpu_create(k, p, 0, 0, &ctx)) return 1;
    const char *wenv = getenv("LAT_WORKER");
    if (wenv && atoi(wenv) > 0) {
        /* LAT_MAX_SHARD: the worker's max_shard (default: S past 16 KiB, so
         * one mailbox serves the whole object; 4096 or less sends larger
         * pinned objects to several mailboxes as column slices) */
        const char *ms = getenv("LAT_MAX_SHARD");
        const size_t max_shard = ms ? (size_t)atol(ms) : (S > 16384 ? S : 0);
        const int e = rsgpu_worker_start(ctx, atoi(wenv), 0, max_shard);
        printf("resident worker: %d mailboxes (rc %d)\n", atoi(wenv), e);
        if (e) return 1;
    }
    double *te = malloc(sizeof(double) * iters), *td = malloc(sizeof(double) * iters);
    double *tf = malloc(sizeof(double) * iters);
    for (int pinned = 0; pinned < 2; ++pinned) {
        uint8_t *buf = NULL, *keep = malloc(S);
        if (pinned) {
            if (rsgpu_host_alloc(n * S, (void **)&buf)) return 1;
        } else {
            buf = malloc(n * S);
        }
        uint64_t x = 12345;
        for (size_t i = 0; i < k * S; ++i) {
            x = x * 6364136223846793005ull + 1442695040888963407ull;
            buf[i] = (uint8_t)(x >> 56);
        }
        uint8_t *sh[12];
        size_t lens[12];
        for (int i = 0; i < n; ++i) { sh[i] = buf + i * S; lens[i] = S; }
        for (int it = 0; it < iters + warm; ++it) {
            for (int i = 0; i < n; ++i) lens[i] = S;
            double t0 = now_us();
            int ok = 0;
            if (rsgpu_encode(ctx, sh, lens, n)) return 2;
            if (rsgpu_verify(ctx, (const uint8_t *const *)sh, lens, n, &ok) || !ok) return 3;
            double t1 = now_us();
            memcpy(keep, sh[0], S);
            lens[0] = lens[5] = 0;
            double t2 = now_us();
            if (rsgpu_decode(ctx, sh, lens, n, &ok) || !ok) return 4;
            double t3 = now_us();
            if (memcmp(keep, sh[0], S)) { fprintf(stderr, "decode mismatch\n"); return 5; }
            lens[0] = lens[5] = S;
            double t4 = now_us();  /* the same pair fused (rsgpu_encode_verify) */
            if (rsgpu_encode_verify(ctx, sh, lens, n, &ok) || !ok) return 6;
            double t5 = now_us();
            if (it >= warm) { te[it - warm] = t1 - t0; td[it - warm] = t3 - t2; tf[it - warm] = t5 - t4; }
        }
        printf("%-8s encode+verify p50 %7.1f us  p99 %7.1f us   decode p50 %7.1f us  p99 %7.1f us\n",
               pinned ? "pinned" : "pageable", pct(te, iters, 0.5), pct(te, iters, 0.99), pct(td, iters, 0.5),
               pct(td, iters, 0.99));
        printf("%-8s encode+verify fused (rsgpu_encode_verify) p50 %7.1f us  p99 %7.1f us\n",
               pinned ? "pinned" : "pageable", pct(tf, iters, 0.5), pct(tf, iters, 0.99));
        if (pinned) rsgpu_host_free(buf); else free(buf);
        free(keep);
    }
    int err = 0;
    if (argc > 2)  /* ./lat_bench ITERS CONC_SECONDS: concurrent callers too */
        for (int t = 1; t <= 16; t *= 2) err |= concurrent(ctx, t, atof(argv[2]));
    rsgpu_destroy(ctx);
    return err ? 7 : 0;
}
