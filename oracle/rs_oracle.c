/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C restatement of the Reed-Solomon codec the InfiniCache client uses
 * (github.com/klauspost/reedsolomon v1.9.3, pinned at /root/reference/go.mod:16,
 * go.sum:36-37; the module is NOT vendored in /root/reference and cannot be
 * fetched offline, so this file restates its published algorithm).  Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * the library built from this file, and only as the checker / the timed CPU
 * baseline — never as the product path (infinicache_amd/ + include/rsgpu.h).
 *
 * Pinning: the reference's own tests hold no EC vectors.
 * This restatement is pinned by the upstream module's published known-answer
 * vectors (galois_test.go / matrix_test.go / reedsolomon_test.go, recalled in
 * SURVEY.md §8c) — see tests/test_oracle_kat.py — and cross-checked against an
 * independent numpy restatement (oracle/rs_numpy.py).
 *
 * Call-site semantics follow /root/reference/client/ecRedis.go:382-432
 * (Client.encode / Client.decode) and /root/reference/client/ec.go:14-121.
 *
 * Two kernels are provided:
 *   - scalar table-driven coding (the "galMulSlice(Xor)" generic Go path);
 *   - the upstream SIMD coders restated: AVX2 PSHUFB nibble tables
 *     (galMulAVX2/galMulAVX2Xor) and the AVX-512 multi-output form
 *     (codeSomeShardsAvx512), with the codeSomeShardsP byte-range split on a
 *     persistent thread pool: the CPU baseline bench.py times
 *     (cpu_baseline.kind = "port").
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>
#if defined(__x86_64__)
#include <immintrin.h>
#endif

/* Error codes: same numeric values as include/rsgpu.h (kept independent on
 * purpose so the oracle shares no code with the product). */
#define ORC_OK 0
#define ORC_ERR_INV_SHARD_NUM -1      /* reedsolomon.ErrInvShardNum */
#define ORC_ERR_MAX_SHARD_NUM -2      /* reedsolomon.ErrMaxShardNum */
#define ORC_ERR_TOO_FEW_SHARDS -3     /* reedsolomon.ErrTooFewShards */
#define ORC_ERR_SHARD_NO_DATA -4      /* reedsolomon.ErrShardNoData */
#define ORC_ERR_SHARD_SIZE -5         /* reedsolomon.ErrShardSize */
#define ORC_ERR_SINGULAR -6           /* reedsolomon errSingular */
#define ORC_ERR_SHORT_DATA -7         /* reedsolomon.ErrShortData */
#define ORC_ERR_RECONSTRUCT_REQUIRED -8
#define ORC_ERR_INVALID_INPUT -9      /* reedsolomon.ErrInvalidInput (Update) */

/* ---------------------------------------------------------------- GF(2^8) */
/* upstream galois.go: field polynomial x^8+x^4+x^3+x^2+1 (0x11D), generator 2,
 * logTable/expTable (expTable doubled to 510 entries), mulTable[256][256]. */
static uint8_t EXP[512];
static uint8_t LOG[256];
static uint8_t MUL[256][256];
static uint8_t MUL_LO[256][16]; /* mulTableLow[c][i]  = c*i        */
static uint8_t MUL_HI[256][16]; /* mulTableHigh[c][i] = c*(i << 4) */
static pthread_once_t gf_once = PTHREAD_ONCE_INIT;

static void gf_init_impl(void) {
    unsigned x = 1;
    for (int i = 0; i < 255; i++) {
        EXP[i] = (uint8_t)x;
        LOG[x] = (uint8_t)i;
        x <<= 1;
        if (x & 0x100) x ^= 0x11D;
    }
    for (int i = 255; i < 512; i++) EXP[i] = EXP[i - 255];
    LOG[0] = 0; /* unused, as upstream */
    for (int a = 0; a < 256; a++)
        for (int b = 0; b < 256; b++)
            MUL[a][b] = (a == 0 || b == 0) ? 0 : EXP[LOG[a] + LOG[b]];
    for (int c = 0; c < 256; c++)
        for (int i = 0; i < 16; i++) {
            MUL_LO[c][i] = MUL[c][i];
            MUL_HI[c][i] = MUL[c][i << 4];
        }
}
static void gf_init(void) { pthread_once(&gf_once, gf_init_impl); }

uint8_t orc_gf_mul(uint8_t a, uint8_t b) { gf_init(); return MUL[a][b]; }

/* upstream galDivide: a/b, b != 0 */
uint8_t orc_gf_div(uint8_t a, uint8_t b) {
    gf_init();
    if (a == 0) return 0;
    if (b == 0) return 0; /* upstream panics; callers never divide by zero */
    int l = (int)LOG[a] - (int)LOG[b];
    if (l < 0) l += 255;
    return EXP[l];
}

/* upstream galExp(a, n): a^n, with 0^0 = 1 */
uint8_t orc_gf_exp(uint8_t a, int n) {
    gf_init();
    if (n == 0) return 1;
    if (a == 0) return 0;
    int l = LOG[a] * n;
    while (l >= 255) l -= 255;
    return EXP[l];
}

/* --------------------------------------------------------------- matrices */
/* upstream matrix.go Invert(): Augment(identity) + gaussianElimination. */
int orc_invert(int n, const uint8_t *in, uint8_t *out) {
    gf_init();
    int cols = 2 * n;
    uint8_t *w = (uint8_t *)calloc((size_t)n * cols, 1);
    if (!w) return ORC_ERR_INVALID_INPUT;
    for (int r = 0; r < n; r++) {
        memcpy(w + r * cols, in + r * n, (size_t)n);
        w[r * cols + n + r] = 1;
    }
    for (int r = 0; r < n; r++) {
        if (w[r * cols + r] == 0) {
            for (int rb = r + 1; rb < n; rb++) {
                if (w[rb * cols + r] != 0) {
                    for (int c = 0; c < cols; c++) {
                        uint8_t t = w[r * cols + c];
                        w[r * cols + c] = w[rb * cols + c];
                        w[rb * cols + c] = t;
                    }
                    break;
                }
            }
        }
        if (w[r * cols + r] == 0) { free(w); return ORC_ERR_SINGULAR; }
        if (w[r * cols + r] != 1) {
            uint8_t scale = orc_gf_div(1, w[r * cols + r]);
            for (int c = 0; c < cols; c++) w[r * cols + c] = MUL[w[r * cols + c]][scale];
        }
        for (int rb = r + 1; rb < n; rb++) {
            uint8_t s = w[rb * cols + r];
            if (s) for (int c = 0; c < cols; c++) w[rb * cols + c] ^= MUL[s][w[r * cols + c]];
        }
    }
    for (int d = 0; d < n; d++)
        for (int ra = 0; ra < d; ra++) {
            uint8_t s = w[ra * cols + d];
            if (s) for (int c = 0; c < cols; c++) w[ra * cols + c] ^= MUL[s][w[d * cols + c]];
        }
    for (int r = 0; r < n; r++) memcpy(out + r * n, w + r * cols + n, (size_t)n);
    free(w);
    return ORC_OK;
}

/* Matrix kinds (upstream options): 0 = default (Vandermonde * top^-1,
 * reedsolomon.go buildMatrix), 1 = WithCauchyMatrix (buildMatrixCauchy),
 * 2 = WithPAR1Matrix (buildMatrixPAR1).  out: (k+p) x k row-major. */
int orc_build_matrix(int k, int p, int kind, uint8_t *out) {
    gf_init();
    if (k <= 0 || p <= 0) return ORC_ERR_INV_SHARD_NUM;
    if (k + p > 256) return ORC_ERR_MAX_SHARD_NUM;
    int n = k + p;
    memset(out, 0, (size_t)n * k);
    if (kind == 1) {
        for (int r = 0; r < n; r++)
            for (int c = 0; c < k; c++)
                out[r * k + c] = r < k ? (uint8_t)(r == c) : orc_gf_div(1, (uint8_t)(r ^ c));
        return ORC_OK;
    }
    if (kind == 2) {
        for (int r = 0; r < n; r++)
            for (int c = 0; c < k; c++)
                out[r * k + c] = r < k ? (uint8_t)(r == c) : orc_gf_exp((uint8_t)(c + 1), r - k);
        return ORC_OK;
    }
    uint8_t *vm = (uint8_t *)malloc((size_t)n * k);
    uint8_t *top = (uint8_t *)malloc((size_t)k * k);
    uint8_t *inv = (uint8_t *)malloc((size_t)k * k);
    for (int r = 0; r < n; r++)
        for (int c = 0; c < k; c++) vm[r * k + c] = orc_gf_exp((uint8_t)r, c);
    memcpy(top, vm, (size_t)k * k);
    int e = orc_invert(k, top, inv);
    if (e == ORC_OK) {
        for (int r = 0; r < n; r++)
            for (int c = 0; c < k; c++) {
                uint8_t acc = 0;
                for (int i = 0; i < k; i++) acc ^= MUL[vm[r * k + i]][inv[i * k + c]];
                out[r * k + c] = acc;
            }
    }
    free(vm); free(top); free(inv);
    return e;
}

/* ------------------------------------------------------- scalar GF coding */
/* upstream codeSomeShards generic path: out_r = XOR_c M[r][c] * in_c
 * (galMulSlice for c == 0, galMulSliceXor after). */
static void code_scalar(const uint8_t *const *rows, int nrows,
                        const uint8_t *const *inputs, int ninputs,
                        uint8_t *const *outputs, size_t start, size_t stop) {
    for (int c = 0; c < ninputs; c++) {
        const uint8_t *in = inputs[c];
        for (int r = 0; r < nrows; r++) {
            const uint8_t *t = MUL[rows[r][c]];
            uint8_t *o = outputs[r];
            if (c == 0)
                for (size_t i = start; i < stop; i++) o[i] = t[in[i]];
            else
                for (size_t i = start; i < stop; i++) o[i] ^= t[in[i]];
        }
    }
}

/* Generic apply: outputs[r] = sum_c coef[r*ninputs + c] * inputs[c]. */
void orc_apply(const uint8_t *coef, int nrows, int ninputs,
               const uint8_t *const *inputs, uint8_t *const *outputs, size_t len) {
    gf_init();
    const uint8_t *rows[256];
    for (int r = 0; r < nrows; r++) rows[r] = coef + (size_t)r * ninputs;
    code_scalar(rows, nrows, inputs, ninputs, outputs, 0, len);
}

/* upstream checkShards(shards, nilok): size = first non-empty length. */
static int check_shards(const size_t *lens, int n, int nilok, size_t *size_out) {
    size_t size = 0;
    for (int i = 0; i < n; i++) if (lens[i] != 0) { size = lens[i]; break; }
    if (size == 0) return ORC_ERR_SHARD_NO_DATA;
    for (int i = 0; i < n; i++)
        if (lens[i] != size && (lens[i] != 0 || !nilok)) return ORC_ERR_SHARD_SIZE;
    *size_out = size;
    return ORC_OK;
}

/* Encode (upstream reedsolomon.go Encode): len check, checkShards(false),
 * parity = M[k:] * data.  lens[i] = length of shard i (0 = nil/empty). */
int orc_encode(int k, int p, int kind, uint8_t *const *shards, const size_t *lens, int nshards) {
    gf_init();
    if (nshards != k + p) return ORC_ERR_TOO_FEW_SHARDS;
    size_t size;
    int e = check_shards(lens, nshards, 0, &size);
    if (e) return e;
    uint8_t *m = (uint8_t *)malloc((size_t)(k + p) * k);
    e = orc_build_matrix(k, p, kind, m);
    if (e) { free(m); return e; }
    const uint8_t *rows[256];
    for (int r = 0; r < p; r++) rows[r] = m + (size_t)(k + r) * k;
    code_scalar(rows, p, (const uint8_t *const *)shards, k, shards + k, 0, size);
    free(m);
    return ORC_OK;
}

/* Verify (upstream Verify): same checks, recompute parity into temps,
 * compare.  *ok = 1 when all parity matches. */
int orc_verify(int k, int p, int kind, uint8_t *const *shards, const size_t *lens, int nshards, int *ok) {
    gf_init();
    *ok = 0;
    if (nshards != k + p) return ORC_ERR_TOO_FEW_SHARDS;
    size_t size;
    int e = check_shards(lens, nshards, 0, &size);
    if (e) return e;
    uint8_t *m = (uint8_t *)malloc((size_t)(k + p) * k);
    orc_build_matrix(k, p, kind, m);
    const uint8_t *rows[256] = {0};
    uint8_t *tmp[256] = {0};
    for (int r = 0; r < p; r++) { rows[r] = m + (size_t)(k + r) * k; tmp[r] = (uint8_t *)malloc(size); }
    code_scalar(rows, p, (const uint8_t *const *)shards, k, tmp, 0, size);
    int good = 1;
    for (int r = 0; r < p; r++) { if (memcmp(tmp[r], shards[k + r], size)) good = 0; free(tmp[r]); }
    free(m);
    *ok = good;
    return ORC_OK;
}

/* Reconstruct / ReconstructData (upstream reconstruct(shards, dataOnly)).
 * shards[i] must point at a buffer of the common shard size for every i; the
 * "present" role is given by lens[i] != 0.  Missing shards are written in
 * place (upstream allocates them; the caller pre-allocates here).
 * Survivors = first k present shards in index order. */
int orc_reconstruct(int k, int p, int kind, uint8_t *const *shards, const size_t *lens,
                    int nshards, int data_only) {
    gf_init();
    if (nshards != k + p) return ORC_ERR_TOO_FEW_SHARDS;
    size_t size;
    int e = check_shards(lens, nshards, 1, &size);
    if (e) return e;
    int n = k + p, present = 0;
    for (int i = 0; i < n; i++) present += lens[i] != 0;
    if (present == n) return ORC_OK;
    if (present < k) return ORC_ERR_TOO_FEW_SHARDS;
    uint8_t *m = (uint8_t *)malloc((size_t)n * k);
    orc_build_matrix(k, p, kind, m);
    int valid[256], nv = 0;
    for (int r = 0; r < n && nv < k; r++) if (lens[r] != 0) valid[nv++] = r;
    uint8_t *sub = (uint8_t *)malloc((size_t)k * k), *inv = (uint8_t *)malloc((size_t)k * k);
    for (int i = 0; i < k; i++) memcpy(sub + i * k, m + (size_t)valid[i] * k, (size_t)k);
    e = orc_invert(k, sub, inv);
    if (e) { free(m); free(sub); free(inv); return e; }
    const uint8_t *rows[256], *ins[256];
    uint8_t *outs[256];
    int no = 0;
    for (int i = 0; i < k; i++) ins[i] = shards[valid[i]];
    for (int i = 0; i < k; i++)
        if (lens[i] == 0) { rows[no] = inv + (size_t)i * k; outs[no++] = shards[i]; }
    if (no) code_scalar(rows, no, ins, k, outs, 0, size);
    if (!data_only) {
        no = 0;
        for (int i = k; i < n; i++)
            if (lens[i] == 0) { rows[no] = m + (size_t)i * k; outs[no++] = shards[i]; }
        if (no) code_scalar(rows, no, (const uint8_t *const *)shards, k, outs, 0, size);
    }
    free(m); free(sub); free(inv);
    return ORC_OK;
}

/* Update (upstream Update + updateParityShards): for each non-nil new data
 * shard c: old_c ^= new_c (the old buffer becomes the delta, as upstream),
 * parity_r ^= M[k+r][c] * delta.  new_lens[c] == 0 means nil. */
int orc_update(int k, int p, int kind, uint8_t *const *shards, const size_t *lens, int nshards,
               const uint8_t *const *newdata, const size_t *new_lens, int nnew) {
    gf_init();
    if (nshards != k + p) return ORC_ERR_TOO_FEW_SHARDS;
    if (nnew != k) return ORC_ERR_TOO_FEW_SHARDS;
    size_t size, size2;
    int e = check_shards(lens, nshards, 1, &size);
    if (e) return e;
    e = check_shards(new_lens, nnew, 1, &size2);
    if (e) return e;
    for (int i = 0; i < k; i++) if (new_lens[i] != 0 && lens[i] == 0) return ORC_ERR_INVALID_INPUT;
    for (int i = k; i < nshards; i++) if (lens[i] == 0) return ORC_ERR_INVALID_INPUT;
    uint8_t *m = (uint8_t *)malloc((size_t)(k + p) * k);
    orc_build_matrix(k, p, kind, m);
    for (int c = 0; c < k; c++) {
        if (new_lens[c] == 0) continue;
        uint8_t *old = shards[c];
        for (size_t i = 0; i < size; i++) old[i] ^= newdata[c][i];
        for (int r = 0; r < p; r++) {
            const uint8_t *t = MUL[m[(size_t)(k + r) * k + c]];
            uint8_t *o = shards[k + r];
            for (size_t i = 0; i < size; i++) o[i] ^= t[old[i]];
        }
    }
    free(m);
    return ORC_OK;
}

/* ------------------------------------------ AVX2 CPU baseline (the "port") */
/* upstream galMulAVX2 / galMulAVX2Xor: 32 B per step, low/high nibble PSHUFB
 * lookups into mulTableLow/High[c]; codeSomeShardsP splits the byte range
 * into do = max(len/maxGoroutines, minSplitSize) rounded up to 64 B, one
 * goroutine per range (std pthreads here). */
#if defined(__x86_64__)
__attribute__((target("avx2")))
static void gal_mul_avx2(uint8_t c, const uint8_t *in, uint8_t *out, size_t n, int xor_) {
    const __m128i lo128 = _mm_loadu_si128((const __m128i *)MUL_LO[c]);
    const __m128i hi128 = _mm_loadu_si128((const __m128i *)MUL_HI[c]);
    const __m256i lo = _mm256_broadcastsi128_si256(lo128);
    const __m256i hi = _mm256_broadcastsi128_si256(hi128);
    const __m256i mask = _mm256_set1_epi8(0x0f);
    size_t i = 0;
    for (; i + 32 <= n; i += 32) {
        __m256i x = _mm256_loadu_si256((const __m256i *)(in + i));
        __m256i l = _mm256_and_si256(x, mask);
        __m256i h = _mm256_and_si256(_mm256_srli_epi64(x, 4), mask);
        __m256i v = _mm256_xor_si256(_mm256_shuffle_epi8(lo, l), _mm256_shuffle_epi8(hi, h));
        if (xor_) v = _mm256_xor_si256(v, _mm256_loadu_si256((const __m256i *)(out + i)));
        _mm256_storeu_si256((__m256i *)(out + i), v);
    }
    /* upstream handles the < 32 B tail with the generic table loop */
    for (; i < n; i++) out[i] = xor_ ? (uint8_t)(out[i] ^ MUL[c][in[i]]) : MUL[c][in[i]];
}
#endif

#if defined(__x86_64__)
/* upstream codeSomeShardsAvx512 (galMulAVX512Parallel82/84, used when the CPU
 * has AVX512F+BW, >= 4 inputs and >= 2 outputs): each 64-B block of every
 * input is read once and multiplied into up to 4 output accumulators held in
 * zmm registers (low/high-nibble VPSHUFB tables, as galMulAVX2). */
__attribute__((target("avx512f,avx512bw")))
static void code_range_avx512(const uint8_t *const *rows, int nrows, const uint8_t *const *inputs,
                              int ninputs, uint8_t *const *outputs, size_t start, size_t stop) {
    const __m512i mask = _mm512_set1_epi8(0x0f);
    for (int r0 = 0; r0 < nrows; r0 += 4) {
        const int nr = nrows - r0 < 4 ? nrows - r0 : 4;
        size_t i = start;
        for (; i + 64 <= stop; i += 64) {
            __m512i acc[4] = {_mm512_setzero_si512(), _mm512_setzero_si512(),
                              _mm512_setzero_si512(), _mm512_setzero_si512()};
            for (int c = 0; c < ninputs; c++) {
                const __m512i x = _mm512_loadu_si512((const void *)(inputs[c] + i));
                const __m512i lo = _mm512_and_si512(x, mask);
                const __m512i hi = _mm512_and_si512(_mm512_srli_epi64(x, 4), mask);
                for (int r = 0; r < nr; r++) {
                    const uint8_t cf = rows[r0 + r][c];
                    const __m512i tl = _mm512_broadcast_i32x4(_mm_loadu_si128((const __m128i *)MUL_LO[cf]));
                    const __m512i th = _mm512_broadcast_i32x4(_mm_loadu_si128((const __m128i *)MUL_HI[cf]));
                    acc[r] = _mm512_ternarylogic_epi64(acc[r], _mm512_shuffle_epi8(tl, lo),
                                                       _mm512_shuffle_epi8(th, hi), 0x96);
                }
            }
            for (int r = 0; r < nr; r++) _mm512_storeu_si512((void *)(outputs[r0 + r] + i), acc[r]);
        }
        if (i < stop) {  /* < 64 B tail: generic table loop, as upstream */
            const uint8_t *rr[4];
            for (int r = 0; r < nr; r++) rr[r] = rows[r0 + r];
            code_scalar(rr, nr, inputs, ninputs, outputs + r0, i, stop);
        }
    }
}
#endif

static void code_range_fast(const uint8_t *const *rows, int nrows, const uint8_t *const *inputs,
                            int ninputs, uint8_t *const *outputs, size_t start, size_t stop) {
#if defined(__x86_64__)
    static int isa = -1;
    if (isa < 0)
        isa = (__builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw")) ? 2
              : __builtin_cpu_supports("avx2") ? 1 : 0;
    if (isa == 2 && ninputs >= 4 && nrows >= 2 && !getenv("ORC_NO_AVX512")) {
        code_range_avx512(rows, nrows, inputs, ninputs, outputs, start, stop);
        return;
    }
    if (isa >= 1) {
        for (int c = 0; c < ninputs; c++)
            for (int r = 0; r < nrows; r++)
                gal_mul_avx2(rows[r][c], inputs[c] + start, outputs[r] + start, stop - start, c != 0);
        return;
    }
#endif
    code_scalar(rows, nrows, inputs, ninputs, outputs, start, stop);
}

/* ISA the fast coder uses on this host: "avx512bw", "avx2" or "scalar". */
const char *orc_cpu_isa(void) {
#if defined(__x86_64__)
    if (__builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw") && !getenv("ORC_NO_AVX512"))
        return "avx512bw";
    if (__builtin_cpu_supports("avx2")) return "avx2";
#endif
    return "scalar";
}

/* ---- persistent worker pool (goroutine stand-in): workers spin briefly,
 * then sleep on a condvar; the submitting thread participates. */
typedef struct {
    void (*fn)(void *, int);
    void *arg;
    int ntasks;
    int next, done;   /* atomics */
    int active;       /* workers inside run_tasks (guarded by POOL.mu) */
} task_t;

static struct {
    pthread_mutex_t mu;
    pthread_cond_t cv;
    int nthreads;
    unsigned long gen;
    task_t *task;
    pthread_mutex_t submit;   /* one job at a time */
} POOL = {PTHREAD_MUTEX_INITIALIZER, PTHREAD_COND_INITIALIZER, 0, 0, NULL, PTHREAD_MUTEX_INITIALIZER};

static void run_tasks(task_t *t) {
    for (;;) {
        int i = __atomic_fetch_add(&t->next, 1, __ATOMIC_ACQ_REL);
        if (i >= t->ntasks) break;
        t->fn(t->arg, i);
        __atomic_fetch_add(&t->done, 1, __ATOMIC_ACQ_REL);
    }
}

static void *pool_worker(void *unused) {
    (void)unused;
    unsigned long seen = 0;
    for (;;) {
        task_t *t = NULL;
        for (int spin = 0; spin < 20000; spin++) {
            if (__atomic_load_n(&POOL.gen, __ATOMIC_ACQUIRE) != seen) break;
            __builtin_ia32_pause();
        }
        pthread_mutex_lock(&POOL.mu);
        while (POOL.gen == seen) pthread_cond_wait(&POOL.cv, &POOL.mu);
        seen = POOL.gen;
        t = POOL.task;
        if (t) t->active++;
        pthread_mutex_unlock(&POOL.mu);
        if (t) {
            run_tasks(t);
            pthread_mutex_lock(&POOL.mu);
            t->active--;
            pthread_cond_broadcast(&POOL.cv);
            pthread_mutex_unlock(&POOL.mu);
        }
    }
    return NULL;
}

static void pool_run(void (*fn)(void *, int), void *arg, int ntasks, int nthreads) {
    if (nthreads <= 1 || ntasks <= 1) {
        for (int i = 0; i < ntasks; i++) fn(arg, i);
        return;
    }
    pthread_mutex_lock(&POOL.submit);
    pthread_mutex_lock(&POOL.mu);
    while (POOL.nthreads < nthreads - 1 && POOL.nthreads < 255) {
        pthread_t th;
        pthread_create(&th, NULL, pool_worker, NULL);
        pthread_detach(th);
        POOL.nthreads++;
    }
    task_t t = {fn, arg, ntasks, 0, 0, 0};
    POOL.task = &t;
    __atomic_add_fetch(&POOL.gen, 1, __ATOMIC_RELEASE);
    pthread_cond_broadcast(&POOL.cv);
    pthread_mutex_unlock(&POOL.mu);
    run_tasks(&t);
    while (__atomic_load_n(&t.done, __ATOMIC_ACQUIRE) < ntasks) __builtin_ia32_pause();
    pthread_mutex_lock(&POOL.mu);
    POOL.task = NULL;   /* late wakers see no job */
    while (t.active > 0) pthread_cond_wait(&POOL.cv, &POOL.mu);  /* t lives on this stack */
    pthread_mutex_unlock(&POOL.mu);
    pthread_mutex_unlock(&POOL.submit);
}

typedef struct {
    const uint8_t *const *rows; int nrows;
    const uint8_t *const *inputs; int ninputs;
    uint8_t *const *outputs;
    size_t len, chunk;
} job_t;

static void range_task(void *arg, int idx) {
    job_t *j = (job_t *)arg;
    size_t s = (size_t)idx * j->chunk, e = s + j->chunk;
    if (e > j->len) e = j->len;
    code_range_fast(j->rows, j->nrows, j->inputs, j->ninputs, j->outputs, s, e);
}

/* codeSomeShardsP: byte ranges of do = max(len/maxGoroutines, minSplitSize
 * = 1024) rounded up to 64 B, run on `nthreads` pool threads. */
void orc_code_fast(const uint8_t *coef, int nrows, int ninputs, const uint8_t *const *inputs,
                   uint8_t *const *outputs, size_t len, int nthreads, int max_g) {
    gf_init();
    const uint8_t *rows[256];
    for (int r = 0; r < nrows; r++) rows[r] = coef + (size_t)r * ninputs;
    if (max_g < 1) max_g = 1;
    size_t chunk = len / (size_t)max_g;
    if (chunk < 1024) chunk = 1024;
    chunk = (chunk + 63) & ~(size_t)63;
    job_t j = {rows, nrows, inputs, ninputs, outputs, len, chunk};
    pool_run(range_task, &j, (int)((len + chunk - 1) / chunk), nthreads);
}

/* Batch job: object o's inputs at base + o*obj_stride + in_rows[c]*pitch,
 * outputs at out_rows[r]. */
typedef struct {
    const uint8_t *coef; int nrows, ninputs;
    const int *in_rows, *out_rows;
    uint8_t *base; size_t obj_stride, pitch, len;
} bjob_t;

static void obj_task(void *arg, int o) {
    bjob_t *j = (bjob_t *)arg;
    const uint8_t *rows[256], *ins[256];
    uint8_t *outs[256];
    for (int r = 0; r < j->nrows; r++) rows[r] = j->coef + (size_t)r * j->ninputs;
    uint8_t *ob = j->base + (size_t)o * j->obj_stride;
    for (int c = 0; c < j->ninputs; c++) ins[c] = ob + (size_t)j->in_rows[c] * j->pitch;
    for (int r = 0; r < j->nrows; r++) outs[r] = ob + (size_t)j->out_rows[r] * j->pitch;
    code_range_fast(rows, j->nrows, ins, j->ninputs, outs, 0, j->len);
}

/* Batch CPU baseline, object-parallel: one object per task on `nthreads`
 * pool threads, the fast coder single-threaded inside a task (the throughput
 * form of many concurrent EcSet/EcGet calls). */
void orc_code_batch(const uint8_t *coef, int nrows, int ninputs, const int *in_rows,
                    const int *out_rows, uint8_t *base, size_t obj_stride, size_t pitch,
                    size_t len, int nobj, int nthreads) {
    gf_init();
    bjob_t j = {coef, nrows, ninputs, in_rows, out_rows, base, obj_stride, pitch, len};
    pool_run(obj_task, &j, nobj, nthreads);
}

/* Batch Verify (upstream Verify / checkSomeShards): object o's rows
 * coef x inputs are recomputed block by block into a task-local buffer and
 * compared with its stored rows chk_rows (the parity upstream's Verify
 * re-encodes, or the fused Get's extra parity shards); ok[o] = 1 when every
 * stored row matches.  Object-parallel like orc_code_batch. */
typedef struct {
    const uint8_t *coef; int nrows, ninputs;
    const int *in_rows, *chk_rows;
    const uint8_t *base; size_t obj_stride, pitch, len;
    int *ok;
} vjob_t;

#define ORC_VBLOCK ((size_t)64 << 10)
static void verify_task(void *arg, int o) {
    vjob_t *j = (vjob_t *)arg;
    const uint8_t *rows[256], *ins[256];
    uint8_t *outs[256];
    uint8_t *tmp = (uint8_t *)aligned_alloc(64, ORC_VBLOCK * (size_t)j->nrows);
    for (int r = 0; r < j->nrows; r++) rows[r] = j->coef + (size_t)r * j->ninputs;
    const uint8_t *ob = j->base + (size_t)o * j->obj_stride;
    int good = 1;
    for (size_t s = 0; s < j->len && good; s += ORC_VBLOCK) {
        const size_t n = j->len - s < ORC_VBLOCK ? j->len - s : ORC_VBLOCK;
        for (int c = 0; c < j->ninputs; c++) ins[c] = ob + (size_t)j->in_rows[c] * j->pitch + s;
        for (int r = 0; r < j->nrows; r++) outs[r] = tmp + (size_t)r * ORC_VBLOCK;
        code_range_fast(rows, j->nrows, ins, j->ninputs, outs, 0, n);
        for (int r = 0; r < j->nrows && good; r++)
            if (memcmp(outs[r], ob + (size_t)j->chk_rows[r] * j->pitch + s, n)) good = 0;
    }
    free(tmp);
    j->ok[o] = good;
}

void orc_verify_batch(const uint8_t *coef, int nrows, int ninputs, const int *in_rows,
                      const int *chk_rows, const uint8_t *base, size_t obj_stride, size_t pitch,
                      size_t len, int nobj, int nthreads, int *ok) {
    gf_init();
    vjob_t j = {coef, nrows, ninputs, in_rows, chk_rows, base, obj_stride, pitch, len, ok};
    pool_run(verify_task, &j, nobj, nthreads);
}
