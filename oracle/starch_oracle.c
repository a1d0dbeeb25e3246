/*
 * oracle/starch_oracle.c -- CPU ORACLE.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this file's shared object (oracle/_build/libstarch_oracle.so).  The product
 * path (starch_amd/, the C-ABI library, the starch3 CLI) never links or calls it.
 *
 * It is a plain-C restatement, written from the behaviour of the reference, of
 *   (1) the Starch coordinate transform of include/starch3api.hpp (hpp:201-345
 *       tokenizer, hpp:428-504 transform, hpp:347-407 segmentation), with the
 *       normative quirks listed in SURVEY.md Appendix A;
 *   (2) the bzip2-1.0.6 -9 compressor that the reference vendors
 *       (third-party/bzip2-1.0.6.tar.gz, members cited as bz:<file>:<line>):
 *       RLE1 + block cut (bz:bzlib.c:224-338, 369-412), CRC (bz:bzlib_private.h:
 *       155-172), block sort = fallbackSort (bz:blocksort.c:30-329, used for every
 *       block: it yields the unique order for non-periodic blocks and the exact
 *       reference tie order for periodic ones, where mainSort always exhausts its
 *       budget -- SURVEY F5), MTF/RLE2 (bz:compress.c:105-231), table selection
 *       and emission (bz:compress.c:238-598), Huffman (bz:huffman.c:63-166) and
 *       framing (bz:compress.c:37-97, 602-667).
 *
 * Parity pin: tests/test_oracle_*.py check this restatement against
 *   - the transform goldens captured from the reference binary
 *     (tests/golden/transform_*.json, made by tools/make_goldens.py), and
 *   - bzip2's own known-answer files (sample{1,2,3}.bz2 at -1/-2/-3) and
 *     per-stream goldens from the reference's vendored libbz2 (oracle/_ref).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ======================================================================= */
/* CRC-32/BZIP2: poly 0x04c11db7, MSB first (bz:crctable.c:31-99)          */
/* ======================================================================= */
static uint32_t g_crc[256];
static int g_crc_ready = 0;

static void crc_setup(void)
{
    if (g_crc_ready) return;
    for (uint32_t b = 0; b < 256; ++b) {
        uint32_t c = b << 24;
        for (int k = 0; k < 8; ++k) c = (c & 0x80000000u) ? (c << 1) ^ 0x04c11db7u : (c << 1);
        g_crc[b] = c;
    }
    g_crc_ready = 1;
}

uint32_t oracle_crc32_bzip2(const uint8_t* p, size_t n)
{
    crc_setup();
    uint32_t c = 0xffffffffu;                       /* BZ_INITIALISE_CRC */
    for (size_t i = 0; i < n; ++i) c = (c << 8) ^ g_crc[(c >> 24) ^ p[i]];  /* BZ_UPDATE_CRC */
    return ~c;                                       /* BZ_FINALISE_CRC */
}

/* ======================================================================= */
/* (1) Starch transform -- SURVEY Appendix A                               */
/* ======================================================================= */
typedef struct {
    uint64_t name_off;    /* offset of the chromosome name in the INPUT */
    uint64_t name_len;    /* strlen() of the chr token (stops at NUL)   */
    uint64_t line_count;  /* transform_state_t.line_count (hpp:503)      */
    uint64_t text_off;    /* offset of the segment text in the output    */
    uint64_t text_len;
} oracle_segment;

static int is_c_space(uint8_t c)
{
    return c == ' ' || c == '\t' || c == '\n' || c == '\v' || c == '\f' || c == '\r';
}

/* sscanf(s, "%" SCNd64, &v) on the C-string s[0..len) (hpp:306-307):
 * leading isspace skipped, optional sign, decimal digits; glibc clamps on
 * overflow.  Returns 1 on success (v written), 0 on failure (v untouched). */
static int scan_i64(const uint8_t* s, size_t len, int64_t* v)
{
    size_t i = 0;
    while (i < len && is_c_space(s[i])) ++i;
    int neg = 0;
    if (i < len && (s[i] == '+' || s[i] == '-')) { neg = (s[i] == '-'); ++i; }
    if (i >= len || s[i] < '0' || s[i] > '9') return 0;
    uint64_t acc = 0; int over = 0;
    const uint64_t lim = neg ? (uint64_t)INT64_MAX + 1u : (uint64_t)INT64_MAX;
    for (; i < len && s[i] >= '0' && s[i] <= '9'; ++i) {
        uint64_t d = (uint64_t)(s[i] - '0');
        if (!over && acc <= (lim - d) / 10u) acc = acc * 10u + d; else over = 1;
    }
    if (over) acc = lim;
    *v = neg ? (int64_t)(0u - acc) : (int64_t)acc;
    return 1;
}

/* n_digits (hpp:559-581): digits of |i|; INT64_MIN stays negative -> 1. */
static int n_digits_ref(int64_t i)
{
    uint64_t u = (i < 0) ? 0u - (uint64_t)i : (uint64_t)i;
    if ((int64_t)u < 0) return 1;
    int d = 1;
    while (d < 19 && u >= 10u) { u /= 10u; ++d; }
    return d;
}

static size_t put_i64(uint8_t* o, int64_t v)   /* "%" PRId64 */
{
    uint8_t tmp[24]; int n = 0;
    uint64_t u = (v < 0) ? 0u - (uint64_t)v : (uint64_t)v;
    do { tmp[n++] = (uint8_t)('0' + (u % 10u)); u /= 10u; } while (u);
    size_t k = 0;
    if (v < 0) o[k++] = '-';
    while (n) o[k++] = tmp[--n];
    return k;
}

/* Effective C-string length of a token: stops at the first NUL. */
static size_t cstr_len(const uint8_t* p, size_t n)
{
    const uint8_t* z = (const uint8_t*)memchr(p, 0, n);
    return z ? (size_t)(z - p) : n;
}

/*
 * oracle_transform: whole-input restatement of produce_line / consume_line /
 * update_transformation_state / process_tf_buffer.
 *
 * Returns the number of output bytes, or (size_t)-1 when out_cap or seg_cap
 * is too small (the caller retries with larger buffers).
 */
size_t oracle_transform_init(const uint8_t* in, size_t n,
                             uint8_t* out, size_t out_cap,
                             oracle_segment* segs, size_t seg_cap, size_t* nseg_out,
                             int64_t init_start, int64_t init_stop);

size_t oracle_transform(const uint8_t* in, size_t n,
                        uint8_t* out, size_t out_cap,
                        oracle_segment* segs, size_t seg_cap, size_t* nseg_out)
{
    return oracle_transform_init(in, n, out, out_cap, segs, seg_cap, nseg_out, 0, 0);
}

/* Same, starting from given bed_t.start/stop values: a piece of an input that
 * begins at a segment boundary, with the sscanf values current before it. */
static size_t transform_core(const uint8_t* in, size_t n, uint8_t* out, size_t out_cap, oracle_segment* segs,
                             size_t seg_cap, size_t* nseg_out, int64_t init_start, int64_t init_stop,
                             uint64_t* base_unique, uint64_t* base_nonunique);

size_t oracle_transform_init(const uint8_t* in, size_t n,
                             uint8_t* out, size_t out_cap,
                             oracle_segment* segs, size_t seg_cap, size_t* nseg_out,
                             int64_t init_start, int64_t init_stop)
{
    return transform_core(in, n, out, out_cap, segs, seg_cap, nseg_out, init_start, init_stop, NULL, NULL);
}

/* Per-segment base counts (the reference declares
 * transform_state_t.base_count_unique / base_count_nonunique, hpp:61-62, and
 * zeroes them at every segment start, hpp:516-532, but never computes them).
 * Over the lines of a segment, with start/stop as the transform uses them
 * (stale sscanf values included): nonunique = sum of (stop - start); unique =
 * sum of max(0, stop - max(start, M)), M = the largest stop of the segment's
 * earlier lines -- the size of the union of the intervals for a BED sorted by
 * start.  Arithmetic is modulo 2^64 (read as int64).  No text is produced;
 * returns 0, or (size_t)-1 when seg_cap is too small. */
size_t oracle_base_counts(const uint8_t* in, size_t n, int64_t init_start, int64_t init_stop,
                          uint64_t* base_unique, uint64_t* base_nonunique, size_t seg_cap, size_t* nseg_out)
{
    oracle_segment* segs = (oracle_segment*)malloc((seg_cap ? seg_cap : 1) * sizeof(oracle_segment));
    if (!segs) return (size_t)-1;
    size_t r = transform_core(in, n, NULL, 0, segs, seg_cap, nseg_out, init_start, init_stop, base_unique,
                              base_nonunique);
    free(segs);
    return r == (size_t)-1 ? r : 0;
}

static size_t transform_core(const uint8_t* in, size_t n, uint8_t* out, size_t out_cap, oracle_segment* segs,
                             size_t seg_cap, size_t* nseg_out, int64_t init_start, int64_t init_stop,
                             uint64_t* base_unique, uint64_t* base_nonunique)
{
    /* Framing (hpp:170-191): byte 0xFF reads as EOF (char compared with EOF,
     * hpp:181); a trailing line without '\n' is never transformed. */
    const uint8_t* ff = (const uint8_t*)memchr(in, 0xFF, n);
    size_t lim = ff ? (size_t)(ff - in) : n;

    int64_t start = init_start, stop = init_stop;   /* bed_t.start/stop persist on sscanf failure (hpp:306-307) */
    int64_t last_cd = 0, last_stop = 0;
    uint64_t line_count = 0;
    size_t o = 0, nseg = 0;
    size_t cur_name_off = 0, cur_name_len = 0; int have_cur = 0;
    size_t seg_text_start = 0;
    uint64_t bu = 0, bn = 0;           /* base counts of the current segment */
    int64_t run_max = 0; int have_max = 0;

    size_t pos = 0;
    while (pos < lim) {
        const uint8_t* nl = (const uint8_t*)memchr(in + pos, '\n', lim - pos);
        if (!nl) break;                                 /* unterminated tail dropped */
        size_t ls = pos, le = (size_t)(nl - in) + 1;    /* [ls, le) includes '\n' */
        pos = le;

        /* Tokenizer (hpp:220-305): a tab advances the token (first three only)
         * and the byte after it is copied unconditionally. */
        size_t f_beg[4] = {0, 0, 0, 0}, f_end[4] = {0, 0, 0, 0};
        int tok = 0;
        f_beg[0] = ls;
        size_t p = ls;
        for (;;) {
            if (in[p] == '\t' && tok != 3) { f_end[tok] = p; ++tok; ++p; f_beg[tok] = p; }
            ++p;                                       /* copy in[p-1] into field tok */
            if (in[p - 1] == '\n') break;
        }
        f_end[tok] = p;
        for (int t = tok + 1; t < 4; ++t) { f_beg[t] = f_end[t] = p; }   /* empty */
        if (tok == 2 || tok == 3) f_end[tok] -= 1;    /* strip '\n' (hpp:298-305) */

        size_t len[4];
        for (int t = 0; t < 4; ++t) len[t] = cstr_len(in + f_beg[t], f_end[t] - f_beg[t]);
        scan_i64(in + f_beg[1], len[1], &start);
        scan_i64(in + f_beg[2], len[2], &stop);

        /* Segmentation (hpp:325-342, 347-407) */
        int new_seg = !have_cur || len[0] != cur_name_len ||
                      memcmp(in + f_beg[0], in + cur_name_off, len[0]) != 0;
        if (new_seg) {
            if (have_cur) {
                if (nseg >= seg_cap) return (size_t)-1;
                segs[nseg].name_off = cur_name_off; segs[nseg].name_len = cur_name_len;
                segs[nseg].line_count = line_count;
                segs[nseg].text_off = seg_text_start; segs[nseg].text_len = o - seg_text_start;
                if (base_unique) { base_unique[nseg] = bu; base_nonunique[nseg] = bn; }
                ++nseg;
            }
            have_cur = 1; cur_name_off = f_beg[0]; cur_name_len = len[0];
            last_cd = 0; last_stop = 0; line_count = 0;          /* hpp:523-536 */
            seg_text_start = o;
            bu = bn = 0; have_max = 0;
        }

        int64_t cd = (int64_t)((uint64_t)stop - (uint64_t)start);
        if (base_unique) {
            const int64_t lo = (have_max && run_max > start) ? run_max : start;
            bn += (uint64_t)cd;
            if (stop > lo) bu += (uint64_t)stop - (uint64_t)lo;
            run_max = (have_max && run_max > stop) ? run_max : stop;
            have_max = 1;
        }
        if (!out) { last_stop = stop; ++line_count; continue; }

        /* Transform (hpp:428-504) */
        if (o + 64 + len[3] > out_cap) return (size_t)-1;
        if (cd != last_cd) {
            last_cd = cd;
            size_t keep = (size_t)(2 + n_digits_ref(cd));      /* tf_line[len]='\0' (hpp:452) */
            uint8_t tmp[32]; size_t k = 0;
            tmp[k++] = 'p'; k += put_i64(tmp + k, cd); tmp[k++] = '\n';
            if (keep > k) keep = k;
            memcpy(out + o, tmp, keep); o += keep;
        }
        int64_t v = (last_stop != 0) ? (int64_t)((uint64_t)start - (uint64_t)last_stop) : start;
        o += put_i64(out + o, v);
        if (len[3] > 0) { out[o++] = '\t'; memcpy(out + o, in + f_beg[3], len[3]); o += len[3]; }
        out[o++] = '\n';
        last_stop = stop;
        ++line_count;
    }
    if (have_cur) {
        if (nseg >= seg_cap) return (size_t)-1;
        segs[nseg].name_off = cur_name_off; segs[nseg].name_len = cur_name_len;
        segs[nseg].line_count = line_count;
        segs[nseg].text_off = seg_text_start; segs[nseg].text_len = o - seg_text_start;
        if (base_unique) { base_unique[nseg] = bu; base_nonunique[nseg] = bn; }
        ++nseg;
    }
    *nseg_out = nseg;
    return o;
}

/* ======================================================================= */
/* (2) bzip2 -N compressor restatement                                      */
/* ======================================================================= */

/* MSB-first bit writer; equivalent to bsW/bsNEEDW/bsFinishWrite
 * (bz:compress.c:37-97): the 32-bit staging word only changes when bytes
 * are released, never the bit order. */
typedef struct {
    uint8_t* buf; size_t cap; size_t nbytes;
    uint64_t acc; int nacc; int overflow;
} bitw_t;

static void bw_put(bitw_t* w, int n, uint32_t v)
{
    w->acc = (w->acc << n) | (uint64_t)(v & ((n == 32) ? 0xffffffffu : ((1u << n) - 1u)));
    w->nacc += n;
    while (w->nacc >= 8) {
        w->nacc -= 8;
        if (w->nbytes < w->cap) w->buf[w->nbytes] = (uint8_t)(w->acc >> w->nacc);
        else w->overflow = 1;
        w->nbytes++;
    }
}
static void bw_finish(bitw_t* w)
{
    if (w->nacc > 0) bw_put(w, 8 - w->nacc, 0);
}

/* ---- fallbackSort restatement (bz:blocksort.c:30-329) ------------------ */
#define FB_SMALL 10
#define FB_STACK 100

static void fb_simple_sort(uint32_t* fmap, const uint32_t* ecls, int32_t lo, int32_t hi)
{
    /* bz:blocksort.c:30-59: a stride-4 insertion pass (when the range holds
     * more than four entries) followed by a stride-1 insertion pass, both
     * walking right-to-left and shifting over strictly smaller keys. */
    if (lo == hi) return;
    if (hi - lo > 3) {
        for (int32_t a = hi - 4; a >= lo; --a) {
            uint32_t x = fmap[a], kx = ecls[x];
            int32_t b = a + 4;
            while (b <= hi && kx > ecls[fmap[b]]) { fmap[b - 4] = fmap[b]; b += 4; }
            fmap[b - 4] = x;
        }
    }
    for (int32_t a = hi - 1; a >= lo; --a) {
        uint32_t x = fmap[a], kx = ecls[x];
        int32_t b = a + 1;
        while (b <= hi && kx > ecls[fmap[b]]) { fmap[b - 1] = fmap[b]; ++b; }
        fmap[b - 1] = x;
    }
}

static void fb_swap_run(uint32_t* fmap, int32_t a, int32_t b, int32_t cnt)
{
    for (; cnt > 0; --cnt, ++a, ++b) { uint32_t t = fmap[a]; fmap[a] = fmap[b]; fmap[b] = t; }
}

static void fb_qsort3(uint32_t* fmap, const uint32_t* ecls, int32_t lo0, int32_t hi0)
{
    /* bz:blocksort.c:92-180: 3-way partition around eclass of lo/mid/hi picked
     * by the LCG r = (r*7621+1) % 32768 (r restarts at 0 on every call). */
    int32_t slo[FB_STACK], shi[FB_STACK];
    int32_t sp = 0;
    uint32_t r = 0;
    slo[sp] = lo0; shi[sp] = hi0; ++sp;
    while (sp > 0) {
        --sp;
        int32_t lo = slo[sp], hi = shi[sp];
        if (hi - lo < FB_SMALL) { fb_simple_sort(fmap, ecls, lo, hi); continue; }
        r = (r * 7621u + 1u) % 32768u;
        uint32_t pv;
        switch (r % 3u) {
            case 0: pv = ecls[fmap[lo]]; break;
            case 1: pv = ecls[fmap[(lo + hi) >> 1]]; break;
            default: pv = ecls[fmap[hi]]; break;
        }
        int32_t ulo = lo, lt = lo, uhi = hi, gt = hi;
        for (;;) {
            while (ulo <= uhi) {
                int64_t d = (int64_t)ecls[fmap[ulo]] - (int64_t)pv;
                if (d == 0) { uint32_t t = fmap[ulo]; fmap[ulo] = fmap[lt]; fmap[lt] = t; ++lt; ++ulo; continue; }
                if (d > 0) break;
                ++ulo;
            }
            while (ulo <= uhi) {
                int64_t d = (int64_t)ecls[fmap[uhi]] - (int64_t)pv;
                if (d == 0) { uint32_t t = fmap[uhi]; fmap[uhi] = fmap[gt]; fmap[gt] = t; --gt; --uhi; continue; }
                if (d < 0) break;
                --uhi;
            }
            if (ulo > uhi) break;
            { uint32_t t = fmap[ulo]; fmap[ulo] = fmap[uhi]; fmap[uhi] = t; }
            ++ulo; --uhi;
        }
        if (gt < lt) continue;                       /* everything equal to the pivot */
        int32_t k = (lt - lo < ulo - lt) ? lt - lo : ulo - lt;
        fb_swap_run(fmap, lo, ulo - k, k);
        int32_t m = (hi - gt < gt - uhi) ? hi - gt : gt - uhi;
        fb_swap_run(fmap, ulo, hi - m + 1, m);
        int32_t a_hi = lo + ulo - lt - 1;            /* [lo, a_hi]  : keys < pivot */
        int32_t b_lo = hi - (gt - uhi) + 1;          /* [b_lo, hi]  : keys > pivot */
        if (a_hi - lo > hi - b_lo) {
            slo[sp] = lo; shi[sp] = a_hi; ++sp;
            slo[sp] = b_lo; shi[sp] = hi; ++sp;
        } else {
            slo[sp] = b_lo; shi[sp] = hi; ++sp;
            slo[sp] = lo; shi[sp] = a_hi; ++sp;
        }
    }
}

/* Sorted order of the cyclic rotations of blk[0..n) into fmap; returns origPtr. */
static int32_t fb_block_sort(const uint8_t* blk, int32_t n, uint32_t* fmap, uint32_t* ecls, uint8_t* head)
{
    /* initial 1-byte bucket sort: each bucket filled from its end while i
     * walks forward (bz:blocksort.c:236-249) */
    int32_t cnt[257];
    memset(cnt, 0, sizeof(cnt));
    for (int32_t i = 0; i < n; ++i) cnt[blk[i]]++;
    for (int32_t c = 1; c < 257; ++c) cnt[c] += cnt[c - 1];
    for (int32_t i = 0; i < n; ++i) fmap[--cnt[blk[i]]] = (uint32_t)i;
    memset(head, 0, (size_t)n + 1);
    for (int32_t c = 0; c < 256; ++c) if (cnt[c] < n) head[cnt[c]] = 1;
    head[n] = 1;                                      /* sentinel (bz:blocksort.c:259-262) */

    for (int32_t H = 1;; H *= 2) {
        /* eclass[x] = bucket head of rotation x+H (bz:blocksort.c:275-280) */
        int32_t j = 0;
        for (int32_t i = 0; i < n; ++i) {
            if (head[i]) j = i;
            int32_t k = (int32_t)fmap[i] - H;
            if (k < 0) k += n;
            ecls[k] = (uint32_t)j;
        }
        int64_t not_done = 0;
        int32_t l = 0;
        while (l < n) {                               /* every bucket [l, r] of size >= 2 */
            int32_t r = l + 1;
            while (r < n && !head[r]) ++r;
            --r;
            if (r > l) {
                not_done += r - l + 1;
                fb_qsort3(fmap, ecls, l, r);
                uint32_t prev = 0xffffffffu;
                for (int32_t i = l; i <= r; ++i) {
                    uint32_t e = ecls[fmap[i]];
                    if (e != prev) { head[i] = 1; prev = e; }
                }
            }
            l = r + 1;
        }
        if ((int64_t)H * 2 > n || not_done == 0) break;
    }
    for (int32_t i = 0; i < n; ++i) if (fmap[i] == 0) return i;    /* bz:blocksort.c:1083-1088 */
    return -1;
}

/* Exposed for the BWT unit tests: sorted rotation order + origPtr. */
int32_t oracle_block_sort(const uint8_t* blk, int32_t n, uint32_t* fmap_out)
{
    uint32_t* ecls = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)(n + 1));
    uint8_t* head = (uint8_t*)malloc((size_t)n + 2);
    int32_t op = fb_block_sort(blk, n, fmap_out, ecls, head);
    free(ecls); free(head);
    return op;
}

/* ---- Huffman code lengths (bz:huffman.c:63-148) ---------------------- */
static void hb_make_lengths(uint8_t* len, const int32_t* freq, int32_t alpha, int32_t max_len)
{
    int32_t heap[260 + 2], weight[258 * 2], parent[258 * 2];
    for (int32_t i = 0; i < alpha; ++i) weight[i + 1] = (freq[i] == 0 ? 1 : freq[i]) << 8;
    for (;;) {
        int32_t nodes = alpha, nheap = 0;
        heap[0] = 0; weight[0] = 0; parent[0] = -2;
#define HB_UP(z) do { int32_t zz = (z), t = heap[zz];                         \
            while (weight[t] < weight[heap[zz >> 1]]) { heap[zz] = heap[zz >> 1]; zz >>= 1; } \
            heap[zz] = t; } while (0)
#define HB_DOWN(z) do { int32_t zz = (z), t = heap[zz];                       \
            for (;;) { int32_t yy = zz << 1; if (yy > nheap) break;              \
                if (yy < nheap && weight[heap[yy + 1]] < weight[heap[yy]]) ++yy;  \
                if (weight[t] < weight[heap[yy]]) break;                        \
                heap[zz] = heap[yy]; zz = yy; }                                  \
            heap[zz] = t; } while (0)
        for (int32_t i = 1; i <= alpha; ++i) { parent[i] = -1; heap[++nheap] = i; HB_UP(nheap); }
        while (nheap > 1) {
            int32_t a = heap[1]; heap[1] = heap[nheap--]; HB_DOWN(1);
            int32_t b = heap[1]; heap[1] = heap[nheap--]; HB_DOWN(1);
            ++nodes;
            parent[a] = parent[b] = nodes;
            int32_t da = weight[a] & 0xff, db = weight[b] & 0xff;
            weight[nodes] = (int32_t)(((uint32_t)weight[a] & 0xffffff00u) + ((uint32_t)weight[b] & 0xffffff00u))
                            | (1 + (da > db ? da : db));
            parent[nodes] = -1;
            heap[++nheap] = nodes; HB_UP(nheap);
        }
#undef HB_UP
#undef HB_DOWN
        int too_long = 0;
        for (int32_t i = 1; i <= alpha; ++i) {
            int32_t d = 0, k = i;
            while (parent[k] >= 0) { k = parent[k]; ++d; }
            len[i - 1] = (uint8_t)d;
            if (d > max_len) too_long = 1;
        }
        if (!too_long) break;
        for (int32_t i = 1; i <= alpha; ++i) weight[i] = (1 + ((weight[i] >> 8) / 2)) << 8;
    }
}

/* canonical codes (bz:huffman.c:152-166) */
static void hb_assign_codes(int32_t* code, const uint8_t* len, int32_t minl, int32_t maxl, int32_t alpha)
{
    int32_t v = 0;
    for (int32_t L = minl; L <= maxl; ++L) {
        for (int32_t i = 0; i < alpha; ++i) if (len[i] == L) code[i] = v++;
        v <<= 1;
    }
}

/* ---- block encoder state ----------------------------------------------- */
typedef struct {
    int32_t bs100k, nblock_max;
    uint8_t* block; int32_t nblock;
    uint32_t crc, combined;
    uint8_t in_use[256];
    int32_t block_no;
    uint32_t rl_ch; int32_t rl_len;
    uint32_t *fmap, *ecls; uint8_t* head; uint16_t* mtfv;
    bitw_t bw;
} ora_bz_t;

static void ob_new_block(ora_bz_t* s)              /* prepare_new_block (bz:bzlib.c:116-126) */
{
    s->nblock = 0; s->crc = 0xffffffffu;
    memset(s->in_use, 0, sizeof(s->in_use));
    s->block_no++;
}

static void ob_add_run(ora_bz_t* s)                 /* add_pair_to_block (bz:bzlib.c:224-256) */
{
    uint8_t ch = (uint8_t)s->rl_ch;
    for (int32_t i = 0; i < s->rl_len; ++i) s->crc = (s->crc << 8) ^ g_crc[(s->crc >> 24) ^ ch];
    s->in_use[ch] = 1;
    int32_t reps = s->rl_len < 4 ? s->rl_len : 4;
    for (int32_t i = 0; i < reps; ++i) s->block[s->nblock++] = ch;
    if (s->rl_len >= 4) {
        s->in_use[s->rl_len - 4] = 1;
        s->block[s->nblock++] = (uint8_t)(s->rl_len - 4);
    }
}

static void ob_add_char(ora_bz_t* s, uint8_t c)     /* ADD_CHAR_TO_BLOCK (bz:bzlib.c:269-293) */
{
    if ((uint32_t)c != s->rl_ch || s->rl_len == 255) {
        if (s->rl_ch < 256) ob_add_run(s);
        s->rl_ch = c; s->rl_len = 1;
    } else {
        s->rl_len++;
    }
}

static void ob_mtf_send(ora_bz_t* s, int32_t orig_ptr);

static void ob_compress_block(ora_bz_t* s, int last)   /* BZ2_compressBlock (bz:compress.c:602-667) */
{
    int32_t orig_ptr = 0;
    if (s->nblock > 0) {
        s->crc = ~s->crc;
        s->combined = ((s->combined << 1) | (s->combined >> 31)) ^ s->crc;
        orig_ptr = fb_block_sort(s->block, s->nblock, s->fmap, s->ecls, s->head);
    }
    if (s->block_no == 1) {
        bw_put(&s->bw, 8, 'B'); bw_put(&s->bw, 8, 'Z'); bw_put(&s->bw, 8, 'h');
        bw_put(&s->bw, 8, (uint32_t)('0' + s->bs100k));
    }
    if (s->nblock > 0) {
        bw_put(&s->bw, 24, 0x314159u); bw_put(&s->bw, 24, 0x265359u);
        bw_put(&s->bw, 32, s->crc);
        bw_put(&s->bw, 1, 0);
        bw_put(&s->bw, 24, (uint32_t)orig_ptr);
        ob_mtf_send(s, orig_ptr);
    }
    if (last) {
        bw_put(&s->bw, 24, 0x177245u); bw_put(&s->bw, 24, 0x385090u);
        bw_put(&s->bw, 32, s->combined);
        bw_finish(&s->bw);
    }
}

static void ob_mtf_send(ora_bz_t* s, int32_t orig_ptr)
{
    (void)orig_ptr;
    /* makeMaps_e + generateMTFValues (bz:compress.c:105-231) */
    uint8_t seq_of[256]; int32_t n_in_use = 0;
    for (int32_t c = 0; c < 256; ++c) if (s->in_use[c]) seq_of[c] = (uint8_t)n_in_use++;
    int32_t eob = n_in_use + 1;
    int32_t freq[258];
    memset(freq, 0, sizeof(freq));
    uint8_t list[256];
    for (int32_t i = 0; i < n_in_use; ++i) list[i] = (uint8_t)i;
    int32_t wr = 0, zrun = 0;
    uint16_t* mtfv = s->mtfv;
#define FLUSH_ZRUN() do { if (zrun > 0) { zrun--;                                    \
            for (;;) { uint16_t sym = (zrun & 1) ? 1 : 0; mtfv[wr++] = sym; freq[sym]++;     \
                if (zrun < 2) break; zrun = (zrun - 2) / 2; }                              \
            zrun = 0; } } while (0)
    for (int32_t i = 0; i < s->nblock; ++i) {
        int32_t j = (int32_t)s->fmap[i] - 1;
        if (j < 0) j += s->nblock;
        uint8_t sym = seq_of[s->block[j]];
        if (list[0] == sym) { zrun++; continue; }
        FLUSH_ZRUN();
        int32_t k = 1;
        uint8_t carry = list[0];
        while (list[k] != sym) { uint8_t t = list[k]; list[k] = carry; carry = t; ++k; }
        list[k] = carry;
        list[0] = sym;
        mtfv[wr++] = (uint16_t)(k + 1); freq[k + 1]++;
    }
    FLUSH_ZRUN();
#undef FLUSH_ZRUN
    mtfv[wr++] = (uint16_t)eob; freq[eob]++;
    int32_t n_mtf = wr;

    /* sendMTFValues (bz:compress.c:238-598) */
    int32_t alpha = n_in_use + 2;
    uint8_t len[6][258];
    int32_t code[6][258];
    int32_t rfreq[6][258];
    uint8_t selector[18002 + 16];
    uint8_t selmtf[18002 + 16];
    for (int t = 0; t < 6; ++t) for (int32_t v = 0; v < alpha; ++v) len[t][v] = 15;
    int32_t n_groups = n_mtf < 200 ? 2 : n_mtf < 600 ? 3 : n_mtf < 1200 ? 4 : n_mtf < 2400 ? 5 : 6;

    {   /* initial equal-frequency bands (bz:compress.c:280-317) */
        int32_t parts = n_groups, rem = n_mtf, gs = 0;
        while (parts > 0) {
            int32_t target = rem / parts, ge = gs - 1, acc = 0;
            while (acc < target && ge < alpha - 1) { ++ge; acc += freq[ge]; }
            if (ge > gs && parts != n_groups && parts != 1 && ((n_groups - parts) % 2 == 1)) {
                acc -= freq[ge]; --ge;
            }
            for (int32_t v = 0; v < alpha; ++v) len[parts - 1][v] = (v >= gs && v <= ge) ? 0 : 15;
            --parts; gs = ge + 1; rem -= acc;
        }
    }

    int32_t n_sel = 0;
    for (int iter = 0; iter < 4; ++iter) {                  /* BZ_N_ITERS */
        for (int t = 0; t < n_groups; ++t) for (int32_t v = 0; v < alpha; ++v) rfreq[t][v] = 0;
        n_sel = 0;
        for (int32_t gs = 0; gs < n_mtf; gs += 50) {
            int32_t ge = gs + 49; if (ge >= n_mtf) ge = n_mtf - 1;
            uint32_t cost[6] = {0, 0, 0, 0, 0, 0};
            for (int32_t i = gs; i <= ge; ++i)
                for (int t = 0; t < n_groups; ++t) cost[t] += len[t][mtfv[i]];
            int bt = 0; uint32_t bc = cost[0];
            for (int t = 1; t < n_groups; ++t) if (cost[t] < bc) { bc = cost[t]; bt = t; }
            selector[n_sel++] = (uint8_t)bt;
            for (int32_t i = gs; i <= ge; ++i) rfreq[bt][mtfv[i]]++;
        }
        for (int t = 0; t < n_groups; ++t) hb_make_lengths(len[t], rfreq[t], alpha, 17);
    }

    {   /* selector MTF (bz:compress.c:461-478) */
        uint8_t pos[6];
        for (int i = 0; i < n_groups; ++i) pos[i] = (uint8_t)i;
        for (int32_t i = 0; i < n_sel; ++i) {
            uint8_t want = selector[i];
            int j = 0; uint8_t carry = pos[0];
            while (carry != want) { ++j; uint8_t t = pos[j]; pos[j] = carry; carry = t; }
            pos[0] = carry;
            selmtf[i] = (uint8_t)j;
        }
    }
    for (int t = 0; t < n_groups; ++t) {
        int32_t mn = 32, mx = 0;
        for (int32_t i = 0; i < alpha; ++i) { if (len[t][i] > mx) mx = len[t][i]; if (len[t][i] < mn) mn = len[t][i]; }
        hb_assign_codes(code[t], len[t], mn, mx, alpha);
    }

    /* mapping table (bz:compress.c:494-516) */
    int used16[16];
    for (int i = 0; i < 16; ++i) {
        used16[i] = 0;
        for (int j = 0; j < 16; ++j) if (s->in_use[i * 16 + j]) used16[i] = 1;
    }
    for (int i = 0; i < 16; ++i) bw_put(&s->bw, 1, (uint32_t)used16[i]);
    for (int i = 0; i < 16; ++i)
        if (used16[i]) for (int j = 0; j < 16; ++j) bw_put(&s->bw, 1, s->in_use[i * 16 + j] ? 1u : 0u);

    bw_put(&s->bw, 3, (uint32_t)n_groups);
    bw_put(&s->bw, 15, (uint32_t)n_sel);
    for (int32_t i = 0; i < n_sel; ++i) {
        for (int j = 0; j < selmtf[i]; ++j) bw_put(&s->bw, 1, 1);
        bw_put(&s->bw, 1, 0);
    }
    for (int t = 0; t < n_groups; ++t) {                   /* delta-coded lengths (bz:compress.c:532-541) */
        int32_t cur = len[t][0];
        bw_put(&s->bw, 5, (uint32_t)cur);
        for (int32_t i = 0; i < alpha; ++i) {
            while (cur < len[t][i]) { bw_put(&s->bw, 2, 2); ++cur; }
            while (cur > len[t][i]) { bw_put(&s->bw, 2, 3); --cur; }
            bw_put(&s->bw, 1, 0);
        }
    }
    int32_t sel = 0;                                       /* data (bz:compress.c:548-593) */
    for (int32_t gs = 0; gs < n_mtf; gs += 50, ++sel) {
        int32_t ge = gs + 49; if (ge >= n_mtf) ge = n_mtf - 1;
        int t = selector[sel];
        for (int32_t i = gs; i <= ge; ++i) bw_put(&s->bw, len[t][mtfv[i]], (uint32_t)code[t][mtfv[i]]);
    }
}

/*
 * oracle_bz2_compress: the bytes of BZ2_bzCompressInit(bs100k) followed by a
 * single BZ2_bzCompress(BZ_FINISH) call with all n input bytes (the harness of
 * SURVEY Appendix C.2).  Returns the stream length, or (size_t)-1 if out_cap
 * is too small.
 */
size_t oracle_bz2_compress(const uint8_t* in, size_t n, int bs100k, uint8_t* out, size_t out_cap)
{
    crc_setup();
    if (bs100k < 1 || bs100k > 9) return (size_t)-1;
    ora_bz_t s;
    memset(&s, 0, sizeof(s));
    s.bs100k = bs100k;
    s.nblock_max = 100000 * bs100k - 19;
    size_t cap = (size_t)s.nblock_max + 64;
    s.block = (uint8_t*)malloc(cap);
    s.fmap = (uint32_t*)malloc(cap * sizeof(uint32_t));
    s.ecls = (uint32_t*)malloc(cap * sizeof(uint32_t));
    s.head = (uint8_t*)malloc(cap + 2);
    s.mtfv = (uint16_t*)malloc((cap + 2) * sizeof(uint16_t));
    s.bw.buf = out; s.bw.cap = out_cap;
    s.rl_ch = 256; s.rl_len = 0;                    /* init_RL */
    ob_new_block(&s);
    for (size_t i = 0; i < n; ++i) {                /* handle_compress, FINISH mode */
        if (s.nblock >= s.nblock_max) { ob_compress_block(&s, 0); ob_new_block(&s); }
        ob_add_char(&s, in[i]);
    }
    if (s.rl_ch < 256) ob_add_run(&s);              /* flush_RL */
    ob_compress_block(&s, 1);
    free(s.block); free(s.fmap); free(s.ecls); free(s.head); free(s.mtfv);
    if (s.bw.overflow) return (size_t)-1;
    return s.bw.nbytes;
}

/* -------------------------------------------------------------------------
 * (3) The inverse transform (unstarch): one segment's text ->
 * BED lines "chr\tstart\tstop[\trem]\n", walking the forward transform's state
 * (hpp:428-504) line by line: "p<cd>" sets cd; "<v>[\t<rem>]" gives
 * start = last_stop ? last_stop + v : v, stop = start + cd, last_stop = stop.
 * Arithmetic modulo 2^64 like the forward int64 differences.  Returns the
 * output length, or (size_t)-1 for text the forward transform cannot produce
 * in an invertible way (a negative p-value: its newline was dropped,
 * hpp:440,452; a malformed line; a final line without its newline).
 * ------------------------------------------------------------------------- */
static int ut_parse(const uint8_t* t, size_t b, size_t e, int64_t* v)
{
    int neg = 0;
    uint64_t a = 0;
    if (b < e && t[b] == '-') { neg = 1; ++b; }
    if (b >= e || e - b > 19) return 0;
    for (size_t k = b; k < e; ++k) {
        if (t[k] < '0' || t[k] > '9') return 0;
        a = a * 10u + (uint64_t)(t[k] - '0');
    }
    *v = neg ? (int64_t)(0ull - a) : (int64_t)a;
    return 1;
}

static size_t ut_put(uint8_t* o, int64_t v)
{
    char buf[24];
    uint64_t u = v < 0 ? 0ull - (uint64_t)v : (uint64_t)v;
    int k = 0;
    do { buf[k++] = (char)('0' + u % 10u); u /= 10u; } while (u);
    size_t n = 0;
    if (v < 0) o[n++] = '-';
    while (k) o[n++] = (uint8_t)buf[--k];
    return n;
}

size_t oracle_untransform(const uint8_t* t, size_t n, const uint8_t* chr, size_t chr_len, uint8_t* out, size_t cap)
{
    uint64_t last_stop = 0;
    int64_t cd = 0;
    size_t o = 0, pos = 0;
    while (pos < n) {
        const uint8_t* nl = (const uint8_t*)memchr(t + pos, '\n', n - pos);
        if (!nl) return (size_t)-1;
        size_t ls = pos, le = (size_t)(nl - t);                 /* le: the '\n' */
        pos = le + 1;
        if (t[ls] == 'p') {
            if (!ut_parse(t, ls + 1, le, &cd) || cd < 0) return (size_t)-1;
            continue;
        }
        size_t e = ls;
        while (e < le && t[e] != '\t') ++e;
        int64_t v;
        if (!ut_parse(t, ls, e, &v)) return (size_t)-1;
        const uint64_t start = last_stop ? last_stop + (uint64_t)v : (uint64_t)v;
        const uint64_t stop = start + (uint64_t)cd;
        if (o + chr_len + 48 + (le - e) > cap) return (size_t)-1;
        memcpy(out + o, chr, chr_len);
        o += chr_len;
        out[o++] = '\t';
        o += ut_put(out + o, (int64_t)start);
        out[o++] = '\t';
        o += ut_put(out + o, (int64_t)stop);
        if (e < le) {
            out[o++] = '\t';
            memcpy(out + o, t + e + 1, le - e - 1);
            o += le - e - 1;
        }
        out[o++] = '\n';
        last_stop = stop;
    }
    return o;
}
