/*
 * oracle/cpu_pool.c -- CPU BASELINE DRIVER.  TEST INFRASTRUCTURE ONLY.
 *
 * Used only by bench.py's cpu_baseline leg (and its CPU test).  It times the
 * CPU path the way SURVEY §8d (ii) asks for: every chromosome piece is
 * transformed (oracle_transform_init, the C restatement of hpp:158-504) and
 * each of its segments compressed with bzip2 -9 -- the reference's own
 * vendored libbz2 1.0.6 (oracle/_ref/libbz2ref.so, ref_bz2_compress) when it
 * is given, else the oracle's restatement -- on a pthread pool, with the
 * pieces taken LARGEST FIRST so the longest stream (chr1) starts at once and
 * the run is not stretched by a late start.  Nothing runs under Python's GIL.
 *
 * cpu_pool_run -> 0, or -1 (allocation / codec failure).  piece_seconds[i]
 * gets the wall time of piece i (transform + bzip2), *seconds the whole run.
 */
#include <dlfcn.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

typedef struct {
    uint64_t name_off, name_len, line_count, text_off, text_len;
} oracle_segment;

size_t oracle_transform_init(const uint8_t* in, size_t n, uint8_t* out, size_t out_cap, oracle_segment* segs,
                             size_t seg_cap, size_t* nseg_out, int64_t init_start, int64_t init_stop);
size_t oracle_bz2_compress(const uint8_t* in, size_t n, int bs100k, uint8_t* out, size_t out_cap);

typedef int (*ref_compress_fn)(const uint8_t*, size_t, int, int, uint8_t*, size_t, size_t*);

typedef struct {
    const uint8_t* data;
    const uint64_t* offs;
    const uint64_t* lens;
    int* order;
    int n;
    int level;
    ref_compress_fn ref;
    volatile int next;
    pthread_mutex_t mu;
    double* piece_seconds;
    uint64_t* piece_out;
    volatile int failed;
} pool_t;

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static int run_piece(pool_t* P, int i)
{
    const uint8_t* in = P->data + P->offs[i];
    size_t n = (size_t)P->lens[i];
    size_t lines = 0;
    for (const uint8_t* p = in; (p = memchr(p, '\n', (size_t)(in + n - p))) != NULL; ++p) ++lines;
    /* a transformed line is at most its input plus a "p<cd>\n" line and a
     * 20-digit delta: 48 bytes per line more than the input bounds it */
    size_t cap = n + 48 * (lines + 1) + 1024;
    uint8_t* text = (uint8_t*)malloc(cap);
    oracle_segment* segs = (oracle_segment*)malloc((lines + 2) * sizeof(oracle_segment));
    if (!text || !segs) { free(text); free(segs); return -1; }
    size_t nseg = 0;
    size_t t = oracle_transform_init(in, n, text, cap, segs, lines + 2, &nseg, 0, 0);
    if (t == (size_t)-1) { free(text); free(segs); return -1; }
    uint64_t out_total = 0;
    for (size_t s = 0; s < nseg; ++s) {
        const uint8_t* src = text + segs[s].text_off;
        size_t len = (size_t)segs[s].text_len;
        size_t ocap = len + len / 50 + 1024;
        uint8_t* out = (uint8_t*)malloc(ocap);
        if (!out) { free(text); free(segs); return -1; }
        size_t olen = 0;
        if (P->ref) {
            if (P->ref(src, len, P->level, 30, out, ocap, &olen) != 0) { free(out); free(text); free(segs); return -1; }
        } else {
            olen = oracle_bz2_compress(src, len, P->level, out, ocap);
            if (olen == (size_t)-1) { free(out); free(text); free(segs); return -1; }
        }
        out_total += olen;
        free(out);
    }
    P->piece_out[i] = out_total;
    free(text);
    free(segs);
    return 0;
}

static void* worker(void* arg)
{
    pool_t* P = (pool_t*)arg;
    for (;;) {
        pthread_mutex_lock(&P->mu);
        int k = P->next < P->n ? P->next++ : -1;
        pthread_mutex_unlock(&P->mu);
        if (k < 0 || P->failed) return NULL;
        int i = P->order[k];
        double t0 = now_s();
        if (run_piece(P, i) != 0) P->failed = 1;
        P->piece_seconds[i] = now_s() - t0;
    }
}

static const uint64_t* g_sort_lens;
static int by_len_desc(const void* a, const void* b)
{
    uint64_t x = g_sort_lens[*(const int*)a], y = g_sort_lens[*(const int*)b];
    return x < y ? 1 : (x > y ? -1 : (*(const int*)a - *(const int*)b));
}

int cpu_pool_run(const uint8_t* data, const uint64_t* offs, const uint64_t* lens, int n, int threads, int level,
                 const char* ref_so, double* seconds, double* piece_seconds, uint64_t* piece_out)
{
    pool_t P;
    memset(&P, 0, sizeof(P));
    P.data = data;
    P.offs = offs;
    P.lens = lens;
    P.n = n;
    P.level = level;
    P.piece_seconds = piece_seconds;
    P.piece_out = piece_out;
    pthread_mutex_init(&P.mu, NULL);
    if (ref_so && ref_so[0]) {
        void* h = dlopen(ref_so, RTLD_NOW | RTLD_LOCAL);
        if (!h) return -1;
        P.ref = (ref_compress_fn)dlsym(h, "ref_bz2_compress");
        if (!P.ref) return -1;
    }
    P.order = (int*)malloc((size_t)(n > 0 ? n : 1) * sizeof(int));
    if (!P.order) return -1;
    for (int i = 0; i < n; ++i) P.order[i] = i;
    g_sort_lens = lens;
    qsort(P.order, (size_t)n, sizeof(int), by_len_desc);
    if (threads < 1) threads = 1;
    pthread_t* th = (pthread_t*)malloc((size_t)threads * sizeof(pthread_t));
    if (!th) {
        free(P.order);
        pthread_mutex_destroy(&P.mu);
        return -1;
    }
    double t0 = now_s();
    int started = 0;
    for (int k = 0; k < threads; ++k) {   /* only created handles are kept (and joined) */
        pthread_t t;
        if (pthread_create(&t, NULL, worker, &P) != 0) break;
        th[started++] = t;
    }
    for (int k = 0; k < started; ++k) pthread_join(th[k], NULL);
    *seconds = now_s() - t0;
    free(th);
    free(P.order);
    pthread_mutex_destroy(&P.mu);
    return (P.failed || started == 0) ? -1 : 0;
}
