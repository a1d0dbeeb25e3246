// starch_amd/csrc/transform.hip -- Starch coordinate transform on MI355X.
//
// Restates, as data-parallel kernels, the per-line pipeline of the reference
// (include/starch3api.hpp): line framing (produce_line, hpp:158-199),
// tokenizing + sscanf (consume_line, hpp:201-345), chromosome segmentation
// (hpp:325-342, 347-407) and update_transformation_state (hpp:428-504).
// Normative semantics, including the reference's quirks, are SURVEY.md
// Appendix A; tests/test_transform_gpu.py checks byte equality against the
// oracle and the reference goldens.
//
// Layout in HBM (all per-line arrays are struct-of-arrays, indexed by line):
//   bed      u8[n]          input bytes
//   line_end u64[L]         offset one past each line's '\n'
//   start/stop i64[L]       parsed integers (stale values propagated)
//   rem_beg u64[L], rem_len u32[L], chr_len u32[L], flags u8[L]
//   out_off u64[L]          exclusive scan of per-line output lengths
//   text     u8[T]          transformed text, segments back to back
#include <string.h>

#include <algorithm>

#include "common.hpp"
#include "transform.hpp"

namespace tf {

constexpr int kTileBytes = 16384;   // 256 threads x 64 B
constexpr int kThreads = 256;

enum : uint8_t { F_START_OK = 1, F_STOP_OK = 2, F_NEW_SEG = 4 };

// --- framing -------------------------------------------------------------
__global__ void __launch_bounds__(kThreads)
k_count_nl(const uint8_t* __restrict__ bed, uint64_t n, uint32_t* __restrict__ tile_cnt,
           unsigned long long* __restrict__ ff_pos)
{
    const uint64_t base = (uint64_t)blockIdx.x * kTileBytes + (uint64_t)threadIdx.x * 64;
    uint32_t c = 0;
    uint64_t ff = ~0ull;
    if (base + 64 <= n && ((reinterpret_cast<uintptr_t>(bed) & 15u) == 0)) {
        const uint4* p = reinterpret_cast<const uint4*>(bed + base);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            uint4 v = p[k];
            uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                uint32_t x = w[j];
                uint32_t t = ((x ^ 0x0a0a0a0au) & 0x7f7f7f7fu) + 0x7f7f7f7fu;
                c += __popc(~(t | (x ^ 0x0a0a0a0au)) & 0x80808080u);
                uint32_t f = ~(((~x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | ~x) & 0x80808080u;   // bytes == 0xff
                if (f && ff == ~0ull) ff = base + k * 16 + j * 4 + ((uint32_t)__builtin_ctz(f) >> 3);
            }
        }
    } else {
        for (uint64_t i = base; i < n && i < base + 64; ++i) {
            uint8_t by = bed[i];
            c += (by == '\n');
            if (by == 0xff && ff == ~0ull) ff = i;
        }
    }
    if (ff != ~0ull) atomicMin(ff_pos, (unsigned long long)ff);
    __shared__ uint32_t sh[kThreads / 64 + 1];
    uint32_t tot;
    (void)block_excl_scan_add<uint32_t>(c, sh, &tot);
    if (threadIdx.x == 0) tile_cnt[blockIdx.x] = tot;
}

// exact per-byte '\n' flags of a little-endian word (bit 7 of each byte)
__device__ __forceinline__ uint32_t nl_flags(uint32_t w)
{
    uint32_t x = w ^ 0x0a0a0a0au;
    uint32_t t = ((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x;
    return ~t & 0x80808080u;
}

__global__ void __launch_bounds__(kThreads)
k_index_nl(const uint8_t* __restrict__ bed, uint64_t n, const uint64_t* __restrict__ tile_off,
           uint64_t* __restrict__ line_end)
{
    const uint64_t base = (uint64_t)blockIdx.x * kTileBytes + (uint64_t)threadIdx.x * 64;
    uint32_t fl[16];
    uint32_t c = 0;
    if (base + 64 <= n && ((reinterpret_cast<uintptr_t>(bed) & 15u) == 0)) {
        const uint4* p = reinterpret_cast<const uint4*>(bed + base);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            uint4 v = p[k];
            fl[4 * k + 0] = nl_flags(v.x);
            fl[4 * k + 1] = nl_flags(v.y);
            fl[4 * k + 2] = nl_flags(v.z);
            fl[4 * k + 3] = nl_flags(v.w);
        }
    } else {
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            uint32_t w = 0;
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                uint64_t i = base + 4 * j + b;
                uint32_t by = (i < n) ? bed[i] : 0u;
                w |= by << (8 * b);
            }
            uint32_t f = nl_flags(w);
#pragma unroll
            for (int b = 0; b < 4; ++b)
                if (base + 4 * j + b >= n) f &= ~(0x80u << (8 * b));
            fl[j] = f;
        }
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) c += __popc(fl[j]);
    __shared__ uint32_t sh[kThreads / 64 + 1];
    uint32_t pre = block_excl_scan_add<uint32_t>(c, sh, (uint32_t*)nullptr);
    uint64_t o = tile_off[blockIdx.x] + pre;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        uint32_t m = fl[j];
        while (m) {
            uint32_t bpos = (uint32_t)__builtin_ctz(m) >> 3;
            line_end[o++] = base + 4 * j + bpos + 1;
            m &= m - 1;
        }
    }
}

// number of lines whose '\n' precedes the first 0xFF (hpp:181: 0xFF reads as EOF)
__global__ void k_lines_before(const uint64_t* __restrict__ line_end, uint64_t nl, const unsigned long long* ff_pos,
                               uint64_t* __restrict__ out)
{
    uint64_t lim = *ff_pos;
    uint64_t lo = 0, hi = nl;     // first index with line_end > lim
    while (lo < hi) {
        uint64_t mid = (lo + hi) >> 1;
        if (line_end[mid] <= lim) lo = mid + 1; else hi = mid;
    }
    *out = lo;
}

// --- parsing ---------------------------------------------------------------
__device__ __forceinline__ bool is_c_space(uint8_t c)
{
    return c == ' ' || c == '\t' || c == '\n' || c == '\v' || c == '\f' || c == '\r';
}

// byte sources for the parser: global memory, or an LDS copy of [base, ...)
struct GSrc {
    const uint8_t* p;
    __device__ __forceinline__ uint8_t operator[](uint64_t x) const { return p[x]; }
};
struct LSrc {
    const uint8_t* t;
    uint64_t base;
    __device__ __forceinline__ uint8_t operator[](uint64_t x) const { return t[x - base]; }
};

// sscanf "%" SCNd64 on the C-string s[0..len) (hpp:306-307); glibc clamps on overflow.
template <class S>
__device__ __forceinline__ bool scan_i64(const S& src, uint64_t off, uint64_t len, int64_t& v)
{
    struct { const S& s; uint64_t o; __device__ uint8_t operator[](uint64_t i) const { return s[o + i]; } } s{src, off};
    uint64_t i = 0;
    while (i < len && is_c_space(s[i])) ++i;
    bool neg = false;
    if (i < len && (s[i] == '+' || s[i] == '-')) { neg = (s[i] == '-'); ++i; }
    if (i >= len || s[i] < '0' || s[i] > '9') return false;
    const uint64_t lim = neg ? 0x8000000000000000ull : 0x7fffffffffffffffull;
    uint64_t acc = 0;
    bool over = false;
    for (; i < len; ++i) {
        uint8_t c = s[i];
        if (c < '0' || c > '9') break;
        uint64_t d = c - '0';
        if (!over && acc <= (lim - d) / 10u) acc = acc * 10u + d; else over = true;
    }
    if (over) acc = lim;
    v = neg ? (int64_t)(0ull - acc) : (int64_t)acc;
    return true;
}

// effective C-string length (first NUL ends a token: strcmp/strlen/sscanf)
template <class S>
__device__ __forceinline__ uint64_t cstr_len(const S& s, uint64_t off, uint64_t n)
{
    for (uint64_t i = 0; i < n; ++i) if (s[off + i] == 0) return i;
    return n;
}

// Tokenize one line [ls, le) (le-1 is '\n'): fields per hpp:220-305.
struct Fields { uint64_t b[4], e[4]; int tok; };

template <class S>
__device__ __forceinline__ Fields tokenize(const S& bed, uint64_t ls, uint64_t le)
{
    // field bounds kept in scalars (a dynamically indexed array would live in
    // scratch memory); same scan as the reference, including the byte after a
    // tab not being tested for a tab
    uint64_t b1 = 0, b2 = 0, b3 = 0, e0 = 0, e1 = 0, e2 = 0;
    int tok = 0;
    uint64_t p = ls;
    for (;;) {
        if (bed[p] == '\t' && tok != 3) {
            if (tok == 0) e0 = p; else if (tok == 1) e1 = p; else e2 = p;
            ++tok;
            ++p;
            if (tok == 1) b1 = p; else if (tok == 2) b2 = p; else b3 = p;
        }
        ++p;
        if (bed[p - 1] == '\n') break;
    }
    Fields f;
    f.tok = tok;
    f.b[0] = ls;
    f.b[1] = tok >= 1 ? b1 : p;
    f.b[2] = tok >= 2 ? b2 : p;
    f.b[3] = tok >= 3 ? b3 : p;
    f.e[0] = tok >= 1 ? e0 : p;
    f.e[1] = tok >= 2 ? e1 : p;
    f.e[2] = tok >= 3 ? e2 : p;
    f.e[3] = p;
    if (tok >= 2) {                                 // strip '\n' from stop or rem
        if (tok == 2) f.e[2] -= 1; else f.e[3] -= 1;
    }
    return f;
}

// chromosome token only (bytes before the first tab; '\n' kept if no tab)
template <class S>
__device__ __forceinline__ uint64_t chr_end(const S& bed, uint64_t ls)
{
    uint64_t p = ls;
    for (;;) {
        uint8_t c = bed[p];
        if (c == '\t') return p;
        ++p;
        if (c == '\n') return p;
    }
}

// Parsed fields of line i (hpp:220-328): start/stop values, whether each
// parsed, whether the chromosome differs from line i-1's, and the remainder.
struct LineVals {
    int64_t a, b;
    uint64_t rem_b;
    uint32_t rem_len, chr_len;
    bool aok, bok, newseg;
};

template <class S>
__device__ __forceinline__ LineVals parse_vals(const S& bed, const uint64_t* __restrict__ line_end, uint64_t i)
{
    LineVals r;
    const uint64_t ls = i ? line_end[i - 1] : 0, le = line_end[i];
    const Fields f = tokenize(bed, ls, le);
    uint64_t len[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) len[t] = cstr_len(bed, f.b[t], f.e[t] - f.b[t]);
    r.a = 0;
    r.b = 0;
    r.aok = scan_i64(bed, f.b[1], len[1], r.a);
    r.bok = scan_i64(bed, f.b[2], len[2], r.b);
    r.newseg = true;
    if (i > 0) {
        const uint64_t ps = (i > 1) ? line_end[i - 2] : 0;
        const uint64_t pe = chr_end(bed, ps);
        const uint64_t plen = cstr_len(bed, ps, pe - ps);
        if (plen == len[0]) {
            r.newseg = false;
            for (uint64_t k = 0; k < plen; ++k)
                if (bed[ps + k] != bed[ls + k]) { r.newseg = true; break; }
        }
    }
    r.rem_b = f.b[3];
    r.rem_len = (uint32_t)len[3];
    r.chr_len = (uint32_t)len[0];
    return r;
}

// start/stop of line i only (the line before a workgroup's first line)
template <class S>
__device__ __forceinline__ void parse_ab(const S& bed, const uint64_t* __restrict__ line_end, uint64_t i, int64_t& a,
                                         int64_t& b)
{
    const uint64_t ls = i ? line_end[i - 1] : 0, le = line_end[i];
    const Fields f = tokenize(bed, ls, le);
    a = 0;
    b = 0;
    scan_i64(bed, f.b[1], cstr_len(bed, f.b[1], f.e[1] - f.b[1]), a);
    scan_i64(bed, f.b[2], cstr_len(bed, f.b[2], f.e[2] - f.b[2]), b);
}

template <class S>
__device__ __forceinline__ void parse_line(const S& bed, const uint64_t* __restrict__ line_end, uint64_t i,
                                           int64_t* __restrict__ start, int64_t* __restrict__ stop,
                                           uint8_t* __restrict__ flags, uint64_t* __restrict__ rem_beg,
                                           uint32_t* __restrict__ rem_len, uint32_t* __restrict__ chr_len,
                                           uint32_t* __restrict__ any_fail)
{
    const LineVals r = parse_vals(bed, line_end, i);
    start[i] = r.a;
    stop[i] = r.b;
    flags[i] = (r.aok ? F_START_OK : 0) | (r.bok ? F_STOP_OK : 0) | (r.newseg ? F_NEW_SEG : 0);
    rem_beg[i] = r.rem_b;
    rem_len[i] = r.rem_len;
    chr_len[i] = r.chr_len;
    if (!r.aok || !r.bok) atomicOr(any_fail, 1u);
}

// One workgroup per 256 lines.  The bytes of those lines and of the line
// before them (its chromosome decides F_NEW_SEG) are staged in LDS with
// coalesced 16-B loads when they fit; every thread then parses its line from
// LDS.  Longer spans (very long lines) parse straight from global memory.
constexpr uint32_t kParseCap = 24576;

__global__ void __launch_bounds__(kThreads)
k_parse(const uint8_t* __restrict__ bed, const uint64_t* __restrict__ line_end, uint64_t nl,
        int64_t* __restrict__ start, int64_t* __restrict__ stop, uint8_t* __restrict__ flags,
        uint64_t* __restrict__ rem_beg, uint32_t* __restrict__ rem_len, uint32_t* __restrict__ chr_len,
        uint32_t* __restrict__ any_fail)
{
    __shared__ uint4 tb4[kParseCap / 16 + 2];
    const uint64_t L0 = (uint64_t)blockIdx.x * kThreads;
    const uint64_t i = L0 + threadIdx.x;
    const uint64_t L1 = L0 + kThreads < nl ? L0 + kThreads : nl;
    const uint64_t rb = L0 >= 2 ? line_end[L0 - 2] : 0;            // start of line L0-1 (or 0)
    const uint64_t re = line_end[L1 - 1];
    // 16-B aligned in absolute address terms (bed itself may be unaligned); a0 is
    // bed-relative and may wrap below 0 -- LSrc indexes with modular arithmetic
    const uintptr_t abs0 = reinterpret_cast<uintptr_t>(bed + rb) & ~(uintptr_t)15;
    const uint64_t a0 = (uint64_t)(abs0 - reinterpret_cast<uintptr_t>(bed));
    const uint64_t nw = (reinterpret_cast<uintptr_t>(bed + re) - abs0 + 15) / 16;
    if (nw * 16 <= kParseCap) {
        const uint4* src = reinterpret_cast<const uint4*>(abs0);
        for (uint64_t w = threadIdx.x; w < nw; w += kThreads) tb4[w] = src[w];
        __syncthreads();
        if (i < nl) {
            LSrc ls{reinterpret_cast<const uint8_t*>(tb4), a0};
            parse_line(ls, line_end, i, start, stop, flags, rem_beg, rem_len, chr_len, any_fail);
        }
    } else if (i < nl) {
        GSrc gs{bed};
        parse_line(gs, line_end, i, start, stop, flags, rem_beg, rem_len, chr_len, any_fail);
    }
}

// stale-value propagation: idx[i] = ok ? i+1 : 0  -> inclusive max-scan -> gather
__global__ void k_ok_index(const uint8_t* __restrict__ flags, uint64_t nl, uint8_t bit, uint64_t* __restrict__ idx)
{
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nl) idx[i] = (flags[i] & bit) ? i + 1 : 0;
}
// `init` is the value before the first line: 0 for a whole input (uninitialised
// malloc memory was observed as 0), the previous unit's
// last parsed value for a shard that starts mid-input.
__global__ void k_gather_stale(const int64_t* __restrict__ cp, const uint64_t* __restrict__ idx, uint64_t nl,
                               int64_t init, int64_t* __restrict__ v)
{
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nl) {
        uint64_t j = idx[i];
        v[i] = j ? cp[j - 1] : init;
    }
}

// --- per-line output length ----------------------------------------------------
__device__ __forceinline__ int ndig_u64(uint64_t u)
{
    // compare against powers of ten (no 64-bit divisions)
    if (u < 10000000000ull) {
        const uint32_t w = (uint32_t)u;
        if (u <= 0xFFFFFFFFull)
            return 1 + (w >= 10u) + (w >= 100u) + (w >= 1000u) + (w >= 10000u) + (w >= 100000u) +
                   (w >= 1000000u) + (w >= 10000000u) + (w >= 100000000u) + (w >= 1000000000u);
        return 10;
    }
    int d = 10;
    uint64_t p = 10000000000ull;
    while (d < 20 && u >= p) { ++d; p = (d < 20) ? p * 10u : p; }
    return d;
}
// n_digits (hpp:559-581): |i| digits, INT64_MIN -> 1
__device__ __forceinline__ int n_digits_ref(int64_t i)
{
    uint64_t u = (i < 0) ? 0ull - (uint64_t)i : (uint64_t)i;
    if ((int64_t)u < 0) return 1;
    int d = ndig_u64(u);
    return d > 19 ? 19 : d;
}
__device__ __forceinline__ int dec_len(int64_t v)
{
    uint64_t u = (v < 0) ? 0ull - (uint64_t)v : (uint64_t)v;
    return ndig_u64(u) + (v < 0 ? 1 : 0);
}

struct LineState { int64_t cd, last_cd, v; bool emit_p; };

__device__ __forceinline__ LineState line_state(const int64_t* start, const int64_t* stop, const uint8_t* flags,
                                                uint64_t i)
{
    LineState s;
    int64_t a = start[i], b = stop[i];
    s.cd = (int64_t)((uint64_t)b - (uint64_t)a);
    int64_t last_stop = 0;
    s.last_cd = 0;
    if (!(flags[i] & F_NEW_SEG)) {
        int64_t pa = start[i - 1], pb = stop[i - 1];
        s.last_cd = (int64_t)((uint64_t)pb - (uint64_t)pa);
        last_stop = pb;
    }
    s.emit_p = (s.cd != s.last_cd);
    s.v = (last_stop != 0) ? (int64_t)((uint64_t)a - (uint64_t)last_stop) : a;
    return s;
}

__global__ void __launch_bounds__(kThreads)
k_line_len(const int64_t* __restrict__ start, const int64_t* __restrict__ stop, const uint8_t* __restrict__ flags,
           const uint32_t* __restrict__ rem_len, uint64_t nl, uint32_t* __restrict__ out_len,
           uint32_t* __restrict__ seg_flag)
{
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nl) return;
    LineState s = line_state(start, stop, flags, i);
    uint32_t L = 0;
    if (s.emit_p) L += 2 + n_digits_ref(s.cd);          // "p%ld\n" truncated (hpp:440,452)
    L += dec_len(s.v) + 1;
    if (rem_len[i]) L += 1 + rem_len[i];
    out_len[i] = L;
    seg_flag[i] = (flags[i] & F_NEW_SEG) ? 1u : 0u;
}

__device__ __forceinline__ uint64_t put_dec(uint8_t* o, int64_t v)
{
    uint64_t u = (v < 0) ? 0ull - (uint64_t)v : (uint64_t)v;
    const int nd = ndig_u64(u);
    uint64_t k = 0;
    if (v < 0) o[k++] = '-';
    if (u <= 0xFFFFFFFFull) {                          // 32-bit divisions
        uint32_t w = (uint32_t)u;
        for (int d = nd - 1; d >= 0; --d) { o[k + d] = (uint8_t)('0' + (w % 10u)); w /= 10u; }
    } else {
        for (int d = nd - 1; d >= 0; --d) { o[k + d] = (uint8_t)('0' + (u % 10u)); u /= 10u; }
    }
    return k + nd;
}

__global__ void __launch_bounds__(kThreads)
k_emit(const uint8_t* __restrict__ bed, const int64_t* __restrict__ start, const int64_t* __restrict__ stop,
       const uint8_t* __restrict__ flags, const uint64_t* __restrict__ rem_beg, const uint32_t* __restrict__ rem_len,
       const uint64_t* __restrict__ out_off, uint64_t nl, uint8_t* __restrict__ text)
{
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nl) return;
    LineState s = line_state(start, stop, flags, i);
    uint8_t* o = text + out_off[i];
    if (s.emit_p) {
        int keep = 2 + n_digits_ref(s.cd);
        uint8_t tmp[24];
        tmp[0] = 'p';
        uint64_t k = 1 + put_dec(tmp + 1, s.cd);
        tmp[k++] = '\n';
        for (int j = 0; j < keep; ++j) o[j] = tmp[j];
        o += keep;
    }
    o += put_dec(o, s.v);
    uint32_t rl = rem_len[i];
    if (rl) {
        *o++ = '\t';
        const uint8_t* r = bed + rem_beg[i];
        for (uint32_t j = 0; j < rl; ++j) o[j] = r[j];
        o += rl;
    }
    *o = '\n';
}

// --- fused two-pass transform -------------------------------------------------
// Taken when every line's start and stop parse (the stale-value rule of
// hpp:306-316 never fires).  Each workgroup owns 256 lines and stages their
// bytes, plus the line before them, in LDS once per pass.  Pass 1 (k_tf1)
// reduces the workgroup's output bytes and new-segment count; after a scan over
// workgroups, pass 2 (k_tf2) re-parses, scans inside the workgroup, builds the
// output text in LDS, stores it with coalesced 4-B writes and records the
// segments that start in it.  No per-line array is materialised.
//
// Lines are parsed with a SWAR scanner over a 128-B register window (tab and
// NUL masks, digit fields of 1..18 plain digits); a line it does not cover
// (longer, NUL bytes, signs/spaces, 19+ digits, fewer than two tabs) takes the
// byte-serial reference parser (parse_vals), which is the definition.

constexpr uint32_t kStagePad = 256;    // reads past the staged span stay inside the LDS array

__device__ __forceinline__ uint32_t eq4(uint32_t x, uint32_t pat)      // 4-bit mask: bytes of x == pat's
{
    const uint32_t t = x ^ pat;
    const uint32_t z = ~(((t & 0x7f7f7f7fu) + 0x7f7f7f7fu) | t) & 0x80808080u;
    return (((z >> 7) * 0x204081u) >> 21) & 15u;
}
__device__ __forceinline__ uint64_t lowbits(uint32_t n) { return n >= 64 ? ~0ull : ((1ull << n) - 1ull); }

// first set bit >= pos of the 128-bit mask (lo, hi); 128 if none
__device__ __forceinline__ uint32_t next_bit(uint64_t lo, uint64_t hi, uint32_t pos)
{
    if (pos < 64) {
        const uint64_t m = lo & ~lowbits(pos);
        if (m) return (uint32_t)__builtin_ctzll(m);
        pos = 64;
    }
    if (pos >= 128) return 128;
    const uint64_t m = hi & ~lowbits(pos - 64);
    return m ? 64u + (uint32_t)__builtin_ctzll(m) : 128u;
}

// 8 bytes of LDS from byte offset b (any alignment): three aligned words, two
// byte-aligns (first byte lowest)
__device__ __forceinline__ uint64_t lds_u64(const uint8_t* tb, uint32_t b)
{
    const uint32_t* w = reinterpret_cast<const uint32_t*>(tb + (b & ~3u));
    const uint32_t sh = b & 3u;
    const uint32_t w0 = w[0], w1 = w[1], w2 = w[2];
    return ((uint64_t)__builtin_amdgcn_alignbyte(w2, w1, sh) << 32) | __builtin_amdgcn_alignbyte(w1, w0, sh);
}

// value of the 1..8 ASCII digits in the low n bytes of x (first digit lowest);
// false if one of them is not a digit.  SWAR: digit pairs, then quads, then
// the 8-digit value, three multiplies in all.
__device__ __forceinline__ bool swar8(uint64_t x, uint32_t n, uint64_t& v)
{
    const uint64_t keep = n >= 8u ? ~0ull : ((1ull << (8u * n)) - 1ull);
    // a byte < '0' sets its top bit in x - '0', a byte > '9' in x + 0x46 (or, past 0xB9, in x - '0')
    if (((x + 0x4646464646464646ull) | (x - 0x3030303030303030ull)) & 0x8080808080808080ull & keep) return false;
    x = ((x - 0x3030303030303030ull) & keep) << (8u * (8u - n));    // leading zero digits
    x = (x * 10u + (x >> 8)) & 0x00FF00FF00FF00FFull;
    x = (x * 100u + (x >> 16)) & 0x0000FFFF0000FFFFull;
    v = (uint32_t)(x * 10000u + (x >> 32));
    return true;
}

// 1..18 plain digits at tb[b..b+n) -> v (sscanf gives the same value for them)
__device__ __forceinline__ bool dig_fast(const uint8_t* tb, uint32_t b, uint32_t n, int64_t& v)
{
    if (n - 1u >= 18u) return false;
    if (n <= 8u) {
        uint64_t x;
        if (!swar8(lds_u64(tb, b), n, x)) return false;
        v = (int64_t)x;
        return true;
    }
    if (n <= 16u) {                                  // the first n - 8 digits, then the last 8
        uint64_t hi, lo;
        if (!swar8(lds_u64(tb, b), n - 8u, hi) || !swar8(lds_u64(tb, b + n - 8u), 8u, lo)) return false;
        v = (int64_t)(hi * 100000000ull + lo);
        return true;
    }
    uint64_t acc = 0;
    uint32_t bad = 0;
    for (uint32_t k = 0; k < n; ++k) {
        const uint32_t d = (uint32_t)tb[b + k] - 48u;
        bad |= (d > 9u) ? 1u : 0u;
        acc = acc * 10u + d;
    }
    v = (int64_t)acc;
    return bad == 0;
}

// Fast parse of the line at stage index r0 (bed offset ls), len bytes incl. '\n'.
// Fills a, b, chr_len, rem_b, rem_len (newseg is decided by the caller).
__device__ __forceinline__ bool parse_fast(const uint8_t* tb, uint32_t r0, uint32_t len, uint64_t ls, LineVals& r)
{
    const uint32_t off = r0 & 15u, q = r0 - off, end = off + len;     // window-relative [off, end)
    if (end > 128u) return false;
    const uint4* tb4 = reinterpret_cast<const uint4*>(tb + q);
    uint64_t tl = 0, th = 0, zl = 0, zh = 0;
#pragma unroll
    for (uint32_t k = 0; k < 8; ++k) {
        if (16u * k < end) {
            const uint4 v = tb4[k];
            const uint64_t tm = (uint64_t)(eq4(v.x, 0x09090909u) | (eq4(v.y, 0x09090909u) << 4) |
                                           (eq4(v.z, 0x09090909u) << 8) | (eq4(v.w, 0x09090909u) << 12));
            const uint64_t zm = (uint64_t)(eq4(v.x, 0u) | (eq4(v.y, 0u) << 4) | (eq4(v.z, 0u) << 8) |
                                           (eq4(v.w, 0u) << 12));
            if (k < 4) { tl |= tm << (16 * k); zl |= zm << (16 * k); }
            else { th |= tm << (16 * (k - 4)); zh |= zm << (16 * (k - 4)); }
        }
    }
    const uint32_t e64 = end < 64u ? end : 64u, o64 = off < 64u ? off : 64u;
    const uint64_t rl = lowbits(e64) & ~lowbits(o64);
    const uint64_t rh = lowbits(end > 64u ? end - 64u : 0u) & ~lowbits(off > 64u ? off - 64u : 0u);
    if ((zl & rl) | (zh & rh)) return false;                  // NUL bytes: C-string rules apply
    const uint32_t nlp = end - 1u;                            // the '\n'
    tl &= rl & ~(nlp < 64u ? (1ull << nlp) : 0ull);
    th &= rh & ~(nlp >= 64u ? (1ull << (nlp - 64u)) : 0ull);
    // the reference's scan does not test the byte after a tab for a tab (tokenize)
    const uint32_t t1 = next_bit(tl, th, off);
    if (t1 >= 128u) return false;
    const uint32_t t2 = next_bit(tl, th, t1 + 2u);
    if (t2 >= 128u) return false;
    const uint32_t t3 = next_bit(tl, th, t2 + 2u);
    const uint32_t e2 = t3 < 128u ? t3 : nlp;
    if (!dig_fast(tb, q + t1 + 1u, t2 - t1 - 1u, r.a)) return false;
    if (!dig_fast(tb, q + t2 + 1u, e2 - t2 - 1u, r.b)) return false;
    r.aok = r.bok = true;
    r.chr_len = t1 - off;
    if (t3 < 128u) {
        r.rem_b = ls + (t3 + 1u - off);
        r.rem_len = nlp - (t3 + 1u);
    } else {
        r.rem_b = ls + len;
        r.rem_len = 0;
    }
    return true;
}

// parse_fast with the tab positions read from precomputed LDS bit masks
// (tabm bit i of word c: staged byte 32c + i is a tab) instead of SWAR over the
// line's bytes; for tiles with no NUL byte (C-string rules then never apply).
// Same acceptance rules and results as parse_fast; line at stage offset r0,
// len bytes incl. its newline (<= 128), bed offset ls.
__device__ __forceinline__ bool parse_mask(const uint8_t* tb, const uint32_t* tabm, uint32_t r0, uint32_t len,
                                           uint64_t ls, LineVals& r)
{
    if (len - 1u >= 128u) return false;
    const uint32_t w = r0 >> 5, sh = r0 & 31u;
    const uint32_t m0 = tabm[w], m1 = tabm[w + 1], m2 = tabm[w + 2], m3 = tabm[w + 3], m4 = tabm[w + 4];
    const uint32_t e = len - 1u;                           // the newline, line-relative
    uint64_t tl = ((uint64_t)__builtin_amdgcn_alignbit(m2, m1, sh) << 32) | __builtin_amdgcn_alignbit(m1, m0, sh);
    uint64_t th = ((uint64_t)__builtin_amdgcn_alignbit(m4, m3, sh) << 32) | __builtin_amdgcn_alignbit(m3, m2, sh);
    tl &= lowbits(e);
    th &= lowbits(e > 64u ? e - 64u : 0u);
    // the reference's scan does not test the byte after a tab for a tab (tokenize)
    const uint32_t t1 = next_bit(tl, th, 0);
    if (t1 >= 128u) return false;
    const uint32_t t2 = next_bit(tl, th, t1 + 2u);
    if (t2 >= 128u) return false;
    const uint32_t t3 = next_bit(tl, th, t2 + 2u);
    const uint32_t e2 = t3 < 128u ? t3 : e;
    if (!dig_fast(tb, r0 + t1 + 1u, t2 - t1 - 1u, r.a)) return false;
    if (!dig_fast(tb, r0 + t2 + 1u, e2 - t2 - 1u, r.b)) return false;
    r.aok = r.bok = true;
    r.chr_len = t1;
    if (t3 < 128u) {
        r.rem_b = ls + t3 + 1u;
        r.rem_len = e - (t3 + 1u);
    } else {
        r.rem_b = ls + len;
        r.rem_len = 0;
    }
    return true;
}

// start/stop and chromosome length of line i, byte-serial (the line before a workgroup)
template <class S>
__device__ __forceinline__ void parse_abc(const S& bed, const uint64_t* __restrict__ line_end, uint64_t i, int64_t& a,
                                          int64_t& b, uint32_t& clen)
{
    const uint64_t ls = i ? line_end[i - 1] : 0, le = line_end[i];
    const Fields f = tokenize(bed, ls, le);
    a = 0;
    b = 0;
    scan_i64(bed, f.b[1], cstr_len(bed, f.b[1], f.e[1] - f.b[1]), a);
    scan_i64(bed, f.b[2], cstr_len(bed, f.b[2], f.e[2] - f.b[2]), b);
    clen = (uint32_t)cstr_len(bed, f.b[0], f.e[0] - f.b[0]);
}

// LDS staging of bytes [start of line L0-1, end of line L1-1); false when they
// do not fit in cap bytes (the workgroup then parses from global memory).
__device__ __forceinline__ bool stage_lines(const uint8_t* __restrict__ bed, const uint64_t* __restrict__ line_end,
                                            uint64_t L0, uint64_t L1, uint4* tb4, uint32_t cap, uint64_t& a0)
{
    const uint64_t rb = L0 >= 2 ? line_end[L0 - 2] : 0;
    const uint64_t re = line_end[L1 - 1];
    const uintptr_t abs0 = reinterpret_cast<uintptr_t>(bed + rb) & ~(uintptr_t)15;
    a0 = (uint64_t)(abs0 - reinterpret_cast<uintptr_t>(bed));
    const uint64_t nw = (reinterpret_cast<uintptr_t>(bed + re) - abs0 + 15) / 16;
    if (nw * 16 > cap) return false;
    const uint4* src = reinterpret_cast<const uint4*>(abs0);
    for (uint64_t w = threadIdx.x; w < nw; w += kThreads) tb4[w] = src[w];
    __syncthreads();
    return true;
}

struct OutDesc { int64_t cd, v; bool emit_p; uint32_t len; };

// hpp:430-470 -- pa/pb are line i-1's start/stop (ignored on a new segment)
__device__ __forceinline__ OutDesc out_desc(const LineVals& r, int64_t pa, int64_t pb)
{
    OutDesc d;
    const int64_t last_cd = r.newseg ? 0 : (int64_t)((uint64_t)pb - (uint64_t)pa);
    const int64_t last_stop = r.newseg ? 0 : pb;
    d.cd = (int64_t)((uint64_t)r.b - (uint64_t)r.a);
    d.emit_p = (d.cd != last_cd);
    d.v = (last_stop != 0) ? (int64_t)((uint64_t)r.a - (uint64_t)last_stop) : r.a;
    uint32_t L = d.emit_p ? 2u + (uint32_t)n_digits_ref(d.cd) : 0u;
    L += (uint32_t)dec_len(d.v) + 1u;
    if (r.rem_len) L += 1u + r.rem_len;
    d.len = L;
    return d;
}

struct TfShared {                     // per-workgroup line exchange
    int64_t a[kThreads + 1], b[kThreads + 1];
    uint32_t cls[kThreads + 1], clen[kThreads + 1];
};

// Parse this thread's line (L0 + tid) and the line before it; returns whether
// the line exists.  t.r.newseg follows hpp:393-407 (strcmp of chromosomes).
struct TfLine {
    LineVals r;
    int64_t pa, pb;
    uint64_t ls;
};

__device__ __forceinline__ bool tf_parse(const uint8_t* __restrict__ bed, const uint64_t* __restrict__ line_end,
                                         uint64_t nl, uint64_t L0, bool staged, const uint8_t* tb, uint64_t a0,
                                         TfShared& sh, TfLine& t)
{
    const uint32_t tid = threadIdx.x;
    const uint64_t i = L0 + tid;
    const bool have = i < nl;
    bool fast = false;
    t.ls = 0;
    if (have) {
        t.ls = i ? line_end[i - 1] : 0;
        const uint64_t le = line_end[i];
        if (staged) {
            fast = parse_fast(tb, (uint32_t)(t.ls - a0), (uint32_t)(le - t.ls), t.ls, t.r);
            if (!fast) t.r = parse_vals(LSrc{tb, a0}, line_end, i);
        } else {
            t.r = parse_vals(GSrc{bed}, line_end, i);
        }
        sh.a[tid + 1] = t.r.a;
        sh.b[tid + 1] = t.r.b;
        sh.cls[tid + 1] = (uint32_t)(t.ls - a0);
        sh.clen[tid + 1] = t.r.chr_len;
    }
    if (tid == 0) {
        int64_t a = 0, b = 0;
        uint32_t clen = 0;
        uint64_t pls = 0;
        if (L0 > 0) {
            pls = (L0 > 1) ? line_end[L0 - 2] : 0;
            LineVals pr;
            if (staged && parse_fast(tb, (uint32_t)(pls - a0), (uint32_t)(line_end[L0 - 1] - pls), pls, pr)) {
                a = pr.a;
                b = pr.b;
                clen = pr.chr_len;
            } else if (staged) {
                parse_abc(LSrc{tb, a0}, line_end, L0 - 1, a, b, clen);
            } else {
                parse_abc(GSrc{bed}, line_end, L0 - 1, a, b, clen);
            }
        }
        sh.a[0] = a;
        sh.b[0] = b;
        sh.cls[0] = (uint32_t)(pls - a0);
        sh.clen[0] = clen;
    }
    __syncthreads();
    if (!have) return false;
    t.pa = sh.a[tid];
    t.pb = sh.b[tid];
    if (fast) {                          // chromosome vs. the previous line's
        bool newseg = true;
        if (i > 0) {
            const uint32_t pc = sh.cls[tid], pcl = sh.clen[tid], cl = t.r.chr_len, c = (uint32_t)(t.ls - a0);
            bool same = (pcl == cl);
            for (uint32_t k = 0; same && k < cl; k += 8) {
#pragma unroll
                for (uint32_t j = 0; j < 8; ++j) {
                    const bool e = tb[pc + k + j] == tb[c + k + j];
                    if (k + j < cl) same = same && e;
                }
            }
            newseg = !same;
        }
        t.r.newseg = newseg;
    }
    return true;
}

// LDS staging sizes are chosen per launch from the input's mean line length
// (and, for pass 2, mean output length): small for BED3, so many workgroups
// stay resident and their loads overlap; a workgroup whose lines do not fit
// parses from global memory / writes its output directly.
constexpr uint32_t kTfCapMax = kParseCap;
constexpr uint32_t kTfOutCapMax = 16384;
extern __shared__ uint4 tf_dyn_lds[];

__global__ void __launch_bounds__(kThreads)
k_tf1(const uint8_t* __restrict__ bed, const uint64_t* __restrict__ line_end, uint64_t nl,
      uint64_t* __restrict__ wg_len, uint32_t* __restrict__ wg_seg, uint32_t* __restrict__ any_fail, uint32_t cap)
{
    uint4* tb4 = tf_dyn_lds;                       // cap + kStagePad bytes
    __shared__ TfShared sh;
    __shared__ uint64_t red[kThreads / 64];
    const uint64_t L0 = (uint64_t)blockIdx.x * kThreads;
    const uint64_t L1 = L0 + kThreads < nl ? L0 + kThreads : nl;
    uint64_t a0 = 0;
    const bool staged = stage_lines(bed, line_end, L0, L1, tb4, cap, a0);
    TfLine t;
    uint64_t v = 0;
    if (tf_parse(bed, line_end, nl, L0, staged, reinterpret_cast<const uint8_t*>(tb4), a0, sh, t)) {
        if (!t.r.aok || !t.r.bok) atomicOr(any_fail, 1u);
        v = ((uint64_t)out_desc(t.r, t.pa, t.pb).len << 20) | (t.r.newseg ? 1u : 0u);
    }
    v = wave_reduce_add(v);                     // bytes << 20 | segments (<= 256 per workgroup)
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint64_t s = red[0] + red[1] + red[2] + red[3];
        wg_len[blockIdx.x] = s >> 20;
        wg_seg[blockIdx.x] = (uint32_t)(s & 0xFFFFFu);
    }
}

template <class S>
__device__ __forceinline__ void tf_write(const S& src, const TfLine& t, uint8_t* o)
{
    const OutDesc d = out_desc(t.r, t.pa, t.pb);
    if (d.emit_p) {                                   // "p%ld\n" truncated to keep bytes (hpp:440,452)
        const int keep = 2 + n_digits_ref(d.cd);
        o[0] = 'p';
        if (dec_len(d.cd) + 2 == keep) {
            o[1 + put_dec(o + 1, d.cd)] = '\n';
        } else {                                      // negative or INT64_MIN: the text is cut short
            const uint64_t u = (d.cd < 0) ? 0ull - (uint64_t)d.cd : (uint64_t)d.cd;
            const int nd = ndig_u64(u), sg = d.cd < 0 ? 1 : 0;
            for (int j = 1; j < keep; ++j) {
                const int q = j - 1 - sg;             // digit index, or the sign
                uint8_t c;
                if (q < 0) c = '-';
                else if (q >= nd) c = '\n';
                else {
                    uint64_t x = u;
                    for (int r = nd - 1 - q; r > 0; --r) x /= 10u;
                    c = (uint8_t)('0' + x % 10u);
                }
                o[j] = c;
            }
        }
        o += keep;
    }
    o += put_dec(o, d.v);
    if (t.r.rem_len) {
        *o++ = '\t';
        for (uint32_t j = 0; j < t.r.rem_len; ++j) o[j] = src[t.r.rem_b + j];
        o += t.r.rem_len;
    }
    *o = '\n';
}

__global__ void __launch_bounds__(kThreads)
k_tf2(const uint8_t* __restrict__ bed, const uint64_t* __restrict__ line_end, uint64_t nl,
      const uint64_t* __restrict__ wg_off, const uint64_t* __restrict__ wg_sego, uint8_t* __restrict__ text,
      SegInfo* __restrict__ info, uint32_t cap, uint32_t ocap)
{
    uint4* tb4 = tf_dyn_lds;                                                    // cap + kStagePad bytes
    uint32_t* ob4 = reinterpret_cast<uint32_t*>(tf_dyn_lds + (cap + kStagePad) / 16);   // ocap bytes
    __shared__ TfShared sh;
    __shared__ uint64_t scan_sh[kThreads / 64 + 1];
    const uint64_t L0 = (uint64_t)blockIdx.x * kThreads;
    const uint64_t L1 = L0 + kThreads < nl ? L0 + kThreads : nl;
    const uint64_t i = L0 + threadIdx.x;
    uint64_t a0 = 0;
    const bool staged = stage_lines(bed, line_end, L0, L1, tb4, cap, a0);
    const uint8_t* tb = reinterpret_cast<const uint8_t*>(tb4);
    TfLine t;
    const bool have = tf_parse(bed, line_end, nl, L0, staged, tb, a0, sh, t);
    const uint64_t len = have ? out_desc(t.r, t.pa, t.pb).len : 0u;
    const uint64_t ns = (have && t.r.newseg) ? 1u : 0u;
    uint64_t tot = 0;
    const uint64_t ex = block_excl_scan_add<uint64_t>((len << 20) | ns, scan_sh, &tot);
    const uint64_t o0 = wg_off[blockIdx.x];
    const uint64_t loc = ex >> 20, wlen = tot >> 20;
    const bool in_lds = wlen <= ocap;
    if (have) {
        if (ns) {
            SegInfo& s = info[wg_sego[blockIdx.x] + (ex & 0xFFFFFu)];
            s.first_line = i;
            s.name_off = t.ls;
            s.name_len = t.r.chr_len;
            s.text_off = o0 + loc;
        }
        uint8_t* ob = reinterpret_cast<uint8_t*>(ob4);
        if (staged) {
            const LSrc ls{tb, a0};
            if (in_lds) tf_write(ls, t, ob + loc); else tf_write(ls, t, text + o0 + loc);
        } else {
            const GSrc gs{bed};
            if (in_lds) tf_write(gs, t, ob + loc); else tf_write(gs, t, text + o0 + loc);
        }
    }
    if (!in_lds) return;
    __syncthreads();
    const uint8_t* ob = reinterpret_cast<const uint8_t*>(ob4);
    const uint32_t wl = (uint32_t)wlen;
    uint32_t head = (uint32_t)((4u - (o0 & 3u)) & 3u);
    head = head < wl ? head : wl;
    if (threadIdx.x < head) text[o0 + threadIdx.x] = ob[threadIdx.x];
    const uint32_t nw = (wl - head) / 4u;
    uint32_t* dst = reinterpret_cast<uint32_t*>(text + o0 + head);
    for (uint32_t w = threadIdx.x; w < nw; w += kThreads) {
        const uint32_t q = head + 4u * w;
        dst[w] = (uint32_t)ob[q] | ((uint32_t)ob[q + 1] << 8) | ((uint32_t)ob[q + 2] << 16) |
                 ((uint32_t)ob[q + 3] << 24);
    }
    for (uint32_t k = head + 4u * nw + threadIdx.x; k < wl; k += kThreads) text[o0 + k] = ob[k];
}

// line_count / text_len of each segment from its successor (fused path)
__global__ void k_seg_close(SegInfo* __restrict__ info, uint64_t nseg, uint64_t nl, uint64_t ttot)
{
    const uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= nseg) return;
    const uint64_t nf = (s + 1 < nseg) ? info[s + 1].first_line : nl;
    const uint64_t nt = (s + 1 < nseg) ? info[s + 1].text_off : ttot;
    info[s].line_count = nf - info[s].first_line;
    info[s].text_len = nt - info[s].text_off;
}

// segment table: for each new-segment line, its ordinal -> first line
__global__ void k_seg_first(const uint32_t* __restrict__ seg_flag, const uint64_t* __restrict__ seg_ord, uint64_t nl,
                            uint64_t* __restrict__ seg_first)
{
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nl && seg_flag[i]) seg_first[seg_ord[i]] = i;
}

__global__ void k_seg_info(const uint64_t* __restrict__ seg_first, uint64_t nseg, uint64_t nl,
                           const uint64_t* __restrict__ line_end, const uint32_t* __restrict__ chr_len,
                           const uint64_t* __restrict__ out_off, uint64_t text_total, SegInfo* __restrict__ info)
{
    uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= nseg) return;
    uint64_t f = seg_first[s], g = (s + 1 < nseg) ? seg_first[s + 1] : nl;
    SegInfo r;
    r.first_line = f;
    r.line_count = g - f;
    r.name_off = f ? line_end[f - 1] : 0;
    r.name_len = chr_len[f];
    r.text_off = out_off[f];
    r.text_len = ((g < nl) ? out_off[g] : text_total) - r.text_off;
    info[s] = r;
}


// --- single-pass transform (default) -----------------------------------------
// One workgroup per 8 KiB byte tile.  A line belongs to the tile holding its
// '\n'; the tile is staged in LDS with a 1 KiB halo before it (the start of
// its first line and the whole previous line, whose chromosome and
// start/stop the first line depends on).  The workgroup finds its newlines,
// parses its lines 256 at a time (parse_fast / the byte-serial parser) and
// builds their output in LDS, then writes it to a bump-allocated piece of an
// arena with the tile's (bytes, lines, segments) counts and segment records;
// a 0xFF (hpp:181: EOF) is recorded as the first tile holding one.  Three
// scans over the tiles give every tile's output offset, k_tf_place moves the
// arena pieces there and k_tf_segs writes the segment records; tiles after
// the first 0xFF are dropped.  Input is read once; no per-line array exists
// in HBM.  Anything outside this shape sets a flag and the host takes the
// two-pass path: a stale sscanf value (FX_FAIL: general path), a line longer
// than the halo or a tile of > 2048 lines (FX_FALLBACK), or text / segment
// capacity (FX_TEXT_CAP / FX_SEG_CAP: grow, rerun).
#ifndef STARCH_FT
#define STARCH_FT 8192
#endif
constexpr uint32_t kFT = STARCH_FT;            // tile bytes
#ifndef STARCH_FH
#define STARCH_FH 1024
#endif
constexpr uint32_t kFH = STARCH_FH;            // halo bytes before the tile
#ifndef STARCH_FTHREADS
#define STARCH_FTHREADS 256
#endif
constexpr int kFThreads = STARCH_FTHREADS;     // threads of a k_tf_fused workgroup (one tile)
static_assert(kFT <= 2u * 32u * (uint32_t)kFThreads, "two 32-byte mask chunks per thread cover the tile");
constexpr uint32_t kFMaxLines = kFT / 4;
constexpr uint32_t kFOut = kFT + kFT / 4;      // LDS output bytes per tile
static_assert(kFT <= 16384, "tested tile sizes: 4, 8, 16 KiB (8 KiB measured fastest)");
constexpr uint32_t kFSeg = 64;                 // segment records per tile in LDS
enum : uint32_t { FX_FAIL = 1, FX_FALLBACK = 2, FX_TEXT_CAP = 4, FX_SEG_CAP = 8 };

template <class S>
__device__ __forceinline__ LineVals parse_line_at(const S& bed, uint64_t ls, uint64_t le)
{
    LineVals r;
    const Fields f = tokenize(bed, ls, le);
    uint64_t len[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) len[t] = cstr_len(bed, f.b[t], f.e[t] - f.b[t]);
    r.a = 0;
    r.b = 0;
    r.aok = scan_i64(bed, f.b[1], len[1], r.a);
    r.bok = scan_i64(bed, f.b[2], len[2], r.b);
    r.newseg = true;
    r.rem_b = f.b[3];
    r.rem_len = (uint32_t)len[3];
    r.chr_len = (uint32_t)len[0];
    return r;
}

struct FusedSeg { uint32_t line, name_ls, name_len, text; };
struct ArenaSeg { uint32_t tile, q, line, name_len; uint64_t name_off; uint32_t text, pad; };
struct FusedOut {                  // k_tf_fused's outputs (arena form) and the scans over them
    uint8_t* arena;                // tile t's text at arena + t * kFOut (a fixed slot: no allocator)
    uint64_t text_cap;             // capacity of the final text buffer (k_tf_place)
    uint32_t* xflags;
    uint32_t *tile_bytes, *tile_lines, *tile_segs;
    uint32_t* first_ff;            // first tile holding a 0xFF (ntiles: none)
    ArenaSeg* seg_arena;
    uint64_t seg_cap;
    unsigned long long* seg_ctr;
    uint64_t *bytes_pre, *lines_pre, *segs_pre;   // ntiles + 1 exclusive prefixes
};
struct LineKey { int64_t a, b; uint32_t cls, clen; };   // what the next line needs of its predecessor

struct FusedShared {
    uint4 tb4[(kFH + kFT + 32 + kStagePad) / 16];
    uint16_t nlp[kFMaxLines];                  // LDS position of each line's '\n'
    uint32_t tabm[(kFH + kFT + 32 + kStagePad) / 32 + 8];   // tab bit masks of the staged bytes (parse_mask)
    uint32_t ob4[kFOut / 4];
    uint64_t scan[kFThreads / 64 + 1];
    FusedSeg seg[kFSeg];
    LineKey wlast[kFThreads / 64 + 1];         // [0]: carry into the chunk; [w+1]: wave w's last line
    uint32_t tile, ffpos, p1, p2, over, nul;
    struct { uint64_t segs; } excl;          // the tile's first record in the segment arena
};

__device__ __forceinline__ LineKey shfl_up_key(const LineKey& k)
{
    LineKey r;
    r.a = __shfl_up(k.a, 1, 64);
    r.b = __shfl_up(k.b, 1, 64);
    r.cls = __shfl_up(k.cls, 1, 64);
    r.clen = __shfl_up(k.clen, 1, 64);
    return r;
}

// The tile's lines, 512 at a time, two consecutive lines per thread: parse,
// output length, one block scan, output and segment records into LDS at
// tile-relative offsets.  A line's predecessor comes by shuffle (wave
// boundaries and chunk starts through LDS).  Returns (bytes, segments).
// prev_ls < first_ls: the line before the tile's first one, [prev_ls, first_ls),
// still to be parsed -- by the last thread, whose two line slots of the first
// chunk are empty (nl <= 2 * kFThreads - 2), while the others parse theirs.
__device__ __forceinline__ void fused_lines(FusedShared& S, const uint8_t* tb, uint64_t a0, uint32_t nl,
                                            uint32_t first_ls, bool input_start, uint32_t* __restrict__ xflags,
                                            uint64_t& bytes_out, uint32_t& segs_out, uint32_t prev_ls = 0,
                                            bool parse_prev = false, bool no_write = false)
{
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (parse_prev && tid == kFThreads - 1) {      // its slots 2*tid, 2*tid+1 are past nl
        LineVals pr;
        if (!parse_mask(tb, S.tabm, prev_ls, first_ls - prev_ls, a0 + prev_ls, pr)) {
            S.over = 1;                           // not the fast shape: the two-pass path takes the input
            pr.a = pr.b = 0;
            pr.chr_len = 0;
        }
        S.wlast[0] = LineKey{pr.a, pr.b, prev_ls, pr.chr_len};   // read after the chunk's first barrier
    }
    const LSrc lsrc{tb, a0};
    uint8_t* ob = reinterpret_cast<uint8_t*>(S.ob4);
    uint64_t run = 0;
    uint32_t segrun = 0;
    for (uint32_t c0 = 0; c0 < nl; c0 += 2 * kFThreads) {
        TfLine t[2];
        uint32_t ls[2] = {0, 0};
        LineKey key[2];
        bool have[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const uint32_t k = c0 + 2 * tid + u;
            have[u] = k < nl;
            key[u] = LineKey{0, 0, 0, 0};
            if (have[u]) {
                ls[u] = k ? (uint32_t)S.nlp[k - 1] + 1u : first_ls;
                const uint32_t le = (uint32_t)S.nlp[k] + 1u;
                t[u].ls = a0 + ls[u];
                // only the fast shape here (no NUL in the tile, line <= 128 bytes,
                // plain digit fields): anything else hands the input to the
                // two-pass path, whose byte-serial parser is the definition
                if (!parse_mask(tb, S.tabm, ls[u], le - ls[u], t[u].ls, t[u].r)) {
                    S.over = 1;
                    t[u].r = LineVals{0, 0, t[u].ls, 0u, 0u, true, true, false};
                }
                if (!t[u].r.aok || !t[u].r.bok) atomicOr(xflags, FX_FAIL);
                key[u] = LineKey{t[u].r.a, t[u].r.b, ls[u], t[u].r.chr_len};
            }
        }
        if (lane == 63) S.wlast[wave + 1] = key[1];
        const LineKey up = shfl_up_key(key[1]);
        __syncthreads();
        const LineKey prev0 = lane ? up : S.wlast[wave];
        uint64_t len[2] = {0, 0}, ns[2] = {0, 0};
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            if (!have[u]) continue;
            const LineKey& p = u ? key[0] : prev0;
            t[u].pa = p.a;
            t[u].pb = p.b;
            bool newseg = true;
            if (!(c0 + 2 * tid + u == 0 && input_start)) {
                const uint32_t cl = t[u].r.chr_len;
                bool same = (p.clen == cl);
                for (uint32_t q = 0; same && q < cl; q += 8) {   // 8 bytes of both names at a time
                    const uint64_t x = lds_u64(tb, p.cls + q) ^ lds_u64(tb, ls[u] + q);
                    const uint32_t k = cl - q;
                    same = (k >= 8u ? x : (x & ((1ull << (8u * k)) - 1ull))) == 0;
                }
                newseg = !same;
            }
            t[u].r.newseg = newseg;
            len[u] = out_desc(t[u].r, t[u].pa, t[u].pb).len;
            ns[u] = newseg ? 1u : 0u;
        }
        uint64_t tot = 0;
        const uint64_t ex = block_excl_scan_add<uint64_t>(((len[0] + len[1]) << 20) | (ns[0] + ns[1]), S.scan, &tot);
        uint64_t off = run + (ex >> 20);
        uint32_t sl = segrun + (uint32_t)(ex & 0xFFFFFu);
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            if (!have[u]) continue;
            if (no_write) { /* timing experiment */ }
            else if (off + len[u] <= kFOut) tf_write(lsrc, t[u], ob + off);
            else S.over = 1;
            if (ns[u]) {
                if (sl < kFSeg) S.seg[sl] = FusedSeg{c0 + 2 * tid + u, ls[u], t[u].r.chr_len, (uint32_t)off};
                else S.over = 1;
                ++sl;
            }
            off += len[u];
        }
        run += tot >> 20;
        segrun += (uint32_t)(tot & 0xFFFFFu);
        // carry: the chunk's last line is the next chunk's first predecessor
        const uint32_t last = (nl - c0 < 2 * kFThreads ? nl - c0 : 2 * kFThreads) - 1;
        if (2 * tid == last) S.wlast[0] = key[0];
        if (2 * tid + 1 == last) S.wlast[0] = key[1];
        __syncthreads();
    }
    bytes_out = run;
    segs_out = segrun;
}

// register budget: 6 waves/SIMD (80 VGPRs, a few spilled) measured 3 % faster
// than the unconstrained 95 VGPRs / 5 waves (the kernel waits on LDS / HBM)
#ifndef STARCH_TF_WPE
#define STARCH_TF_WPE 6
#endif
// STARCH_TF_PROF (timing experiment, dev builds only): per-wave shader-clock
// time of k_tf_fused's phases, summed into g_tfprof (printed by run())
#ifdef STARCH_TF_PROF
__device__ unsigned long long g_tfprof[8];
#define TPROF(v) const uint64_t v = __builtin_readcyclecounter()
#else
#define TPROF(v)
#endif
__global__ void __launch_bounds__(kFThreads) __attribute__((amdgpu_waves_per_eu(STARCH_TF_WPE)))
k_tf_fused(const uint8_t* __restrict__ bed, uint64_t n, const FusedOut fo, uint32_t* __restrict__ xflags,
           uint32_t dbg_mode)
{
    __shared__ FusedShared S;
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    TPROF(p0);
    if (tid == 0) {
        S.tile = blockIdx.x;
        S.ffpos = 0xFFFFFFFFu;
        S.p1 = 0;
        S.p2 = 0;
        S.over = 0;
        S.nul = 0;
    }
    __syncthreads();
    const uint32_t tile = S.tile;
    const uint64_t t0 = (uint64_t)tile * kFT;
    const uint64_t tend = t0 + kFT < n ? t0 + kFT : n;
    const uint64_t s0 = t0 > kFH ? t0 - kFH : 0;
    const uintptr_t abs0 = reinterpret_cast<uintptr_t>(bed + s0) & ~(uintptr_t)15;
    const uint64_t a0 = (uint64_t)(abs0 - reinterpret_cast<uintptr_t>(bed));   // bed-relative (may wrap)
    const uint32_t nw = (uint32_t)((reinterpret_cast<uintptr_t>(bed + tend) - abs0 + 15) / 16);
    {
        const uint4* src = reinterpret_cast<const uint4*>(abs0);
        for (uint32_t w = tid; w < nw; w += kFThreads) S.tb4[w] = src[w];
    }
    __syncthreads();
    TPROF(p1);
    const uint8_t* tb = reinterpret_cast<const uint8_t*>(S.tb4);
    const uint32_t Lt0 = (uint32_t)(t0 - a0), Lend = (uint32_t)(tend - a0), Ls0 = (uint32_t)(s0 - a0);
    // newline / 0xFF masks of 32-byte LDS chunks covering [Lt0, Lend); a thread
    // owns two consecutive chunks, so scan order is byte order
    const uint32_t cbeg = Lt0 >> 5, cend = (Lend + 31) >> 5;
    uint32_t nlm[2] = {0, 0};
#pragma unroll
    for (uint32_t it = 0; it < 2; ++it) {
        const uint32_t ch = cbeg + 2 * tid + it;
        if (ch >= cend) continue;
        const uint4* q = reinterpret_cast<const uint4*>(tb + ch * 32);
        const uint4 x = q[0], y = q[1];
        const uint32_t w[8] = {x.x, x.y, x.z, x.w, y.x, y.y, y.z, y.w};
        uint32_t nm = 0, tm = 0, anyz = 0, anyf = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            nm |= eq4(w[j], 0x0a0a0a0au) << (4 * j);
            tm |= eq4(w[j], 0x09090909u) << (4 * j);
            anyz |= (w[j] - 0x01010101u) & ~w[j] & 0x80808080u;    // some byte is NUL
            anyf |= (~w[j] - 0x01010101u) & w[j] & 0x80808080u;    // some byte is 0xFF
        }
        S.tabm[ch] = tm;
        const uint32_t lo = ch * 32 < Lt0 ? Lt0 - ch * 32 : 0u;
        const uint32_t hi = Lend - ch * 32 < 32u ? Lend - ch * 32 : 32u;
        const uint32_t keep = (hi >= 32u ? 0xFFFFFFFFu : ((1u << hi) - 1u)) & ~((1u << lo) - 1u);
        // exact per-byte NUL / 0xFF masks only where a word holds one, or in the
        // chunk that runs past the tile's end (its last bytes are not staged)
        uint32_t zm = 0, fm = 0;
        if (anyz | anyf | (hi < 32u)) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                zm |= eq4(w[j], 0u) << (4 * j);
                fm |= eq4(w[j], 0xffffffffu) << (4 * j);
            }
        }
        // a NUL among the staged bytes (everything from a0 up to the tile's end;
        // the bytes after it are not staged)
        if (zm & (hi >= 32u ? 0xFFFFFFFFu : ((1u << hi) - 1u))) S.nul = 1;
        nlm[it] = nm & keep;
        fm &= keep;
        if (fm) atomicMin(&S.ffpos, ch * 32 + (uint32_t)__builtin_ctz(fm));
    }
    // tab masks and the NUL flag of the halo chunks as well (a tile's first
    // line starts in its halo)
    for (uint32_t ch = tid; ch < cbeg; ch += kFThreads) {
        const uint4* q = reinterpret_cast<const uint4*>(tb + ch * 32);
        const uint4 x = q[0], y = q[1];
        const uint32_t w[8] = {x.x, x.y, x.z, x.w, y.x, y.y, y.z, y.w};
        uint32_t tm = 0, zf = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            tm |= eq4(w[j], 0x09090909u) << (4 * j);
            zf |= (w[j] - 0x01010101u) & ~w[j] & 0x80808080u;
        }
        S.tabm[ch] = tm;
        if (zf) S.nul = 1;
    }
    // the halo's last two newlines (wave 0, 64 bytes at a time, backwards):
    // the previous line is [p2, p1), the first line starts at p1
    if (tid < 64 && Lt0 > Ls0) {
        uint32_t found = 0, p1 = 0, p2 = 0;
        for (uint32_t e = Lt0; e > Ls0 && found < 2;) {
            const uint32_t b0 = e - Ls0 > 64u ? e - 64u : Ls0;
            const uint32_t j = b0 + lane;
            uint64_t m = __ballot(j < e && tb[j] == '\n');
            while (m && found < 2) {
                const uint32_t pos = b0 + (uint32_t)(63 - __clzll((long long)m));
                if (found == 0) p1 = pos + 1; else p2 = pos + 1;
                ++found;
                m &= ~(1ull << (pos - b0));
            }
            e = b0;
        }
        if (lane == 0) { S.p1 = p1; S.p2 = p2; }
    }
    __syncthreads();
    const uint32_t ffpos = S.ffpos;
    uint32_t cnt = 0;
#pragma unroll
    for (uint32_t it = 0; it < 2; ++it) {
        const uint32_t ch = cbeg + 2 * tid + it;
        if (ffpos != 0xFFFFFFFFu && ch * 32 + 32 > ffpos) {   // lines ending after the 0xFF are dropped
            const uint32_t lim = ffpos > ch * 32 ? ffpos - ch * 32 : 0u;
            nlm[it] &= lim >= 32u ? 0xFFFFFFFFu : ((1u << lim) - 1u);
        }
        cnt += __popc(nlm[it]);
    }
    uint32_t nl_tile = 0;
    const uint32_t pre = block_excl_scan_add<uint32_t>(cnt, reinterpret_cast<uint32_t*>(S.scan), &nl_tile);
    bool fallback = nl_tile > kFMaxLines || S.nul;   // (a NUL: C-string rules apply, the two-pass path)
    if (!fallback) {
        uint32_t o = pre;
#pragma unroll
        for (uint32_t it = 0; it < 2; ++it) {
            const uint32_t ch = cbeg + 2 * tid + it;
            uint32_t m = nlm[it];
            while (m) {
                S.nlp[o++] = (uint16_t)(ch * 32 + (uint32_t)__builtin_ctz(m));
                m &= m - 1;
            }
        }
    }
    // first line start and the previous line
    bool input_start = false;
    uint32_t first_ls = Lt0, prev_ls = 0;
    if (t0 == 0) {
        input_start = true;
    } else if (S.p1) {
        first_ls = S.p1;
        if (S.p2) prev_ls = S.p2;
        else if (s0 == 0) prev_ls = Ls0;
        else fallback = true;                      // previous line longer than the halo
    } else if (s0 == 0) {
        first_ls = Ls0;                            // no line ended before the tile: the input's first line
        input_start = true;
    } else {
        fallback = fallback || nl_tile > 0;        // first line longer than the halo
    }
    // the previous line: parsed inside fused_lines by an idle thread when the
    // tile's lines leave one free, else here by thread 0
    const bool need_prev = !fallback && !input_start && nl_tile > 0;
    const bool prev_in_lines = need_prev && nl_tile <= 2 * kFThreads - 2;
    if (tid == 0) {
        LineKey pk{0, 0, 0, 0};
        if (need_prev && !prev_in_lines) {
            LineVals pr;
            const uint32_t ple = first_ls;         // one past the previous line's '\n'
            if (!fallback && parse_mask(tb, S.tabm, prev_ls, ple - prev_ls, a0 + prev_ls, pr))
                pk = LineKey{pr.a, pr.b, prev_ls, pr.chr_len};
            else
                S.over = 1;
        }
        S.wlast[0] = pk;
    }
    __syncthreads();
    TPROF(p2);
    uint64_t bytes = 0;
    uint32_t segs = 0;
    if (dbg_mode == 1 || dbg_mode == 2) {           // timing experiments: no output (empty tiles)
        if (tid == 0) {
            fo.tile_bytes[tile] = 0u;
            fo.tile_lines[tile] = 0u;
            fo.tile_segs[tile] = 0u;
        }
        if (dbg_mode == 2) return;                  // staging + masks only
    }
    if (!fallback && nl_tile > 0)
        fused_lines(S, tb, a0, nl_tile, first_ls, input_start, xflags, bytes, segs, prev_ls, prev_in_lines,
                    dbg_mode == 3);
    TPROF(p3);
    fallback = fallback || S.over;
    if (fallback && tid == 0) atomicOr(xflags, FX_FALLBACK);
    if (dbg_mode == 1) return;                      // timing experiment: parse only (tile counts zeroed above)
    TPROF(p4);
    // No look-back: the tile's text goes to its fixed slot of the arena and its
    // counts to per-tile arrays; k_tf_place moves it to its final offset after
    // a scan over the tiles.  (Waiting here for the previous tiles' prefix,
    // with the workgroup's LDS held, took ~65% of the workgroups' time
    // (STARCH_TF_PROF); a bump allocator -- one atomic per tile on one counter
    // -- serialised the tiles' tails: 1.7 of 4.4 ms, STARCH_TF_DBG=1.)
    if (tid == 0) {
        const bool ff = ffpos != 0xFFFFFFFFu;
        fo.tile_bytes[tile] = fallback ? 0u : (uint32_t)bytes;
        fo.tile_lines[tile] = fallback ? 0u : nl_tile;
        fo.tile_segs[tile] = fallback ? 0u : segs;
        if (ff) atomicMin(fo.first_ff, tile);
        uint64_t sb = 0;
        if (!fallback && segs) sb = atomicAdd(fo.seg_ctr, (uint64_t)segs);   // tiles with a segment start only
        S.excl.segs = sb;
        if (sb + segs > fo.seg_cap) atomicOr(xflags, FX_SEG_CAP);
    }
    __syncthreads();
    if (fallback || nl_tile == 0) return;
    const uint64_t ab = (uint64_t)tile * kFOut, sb = S.excl.segs;
    if (sb + segs > fo.seg_cap) return;
    for (uint32_t q = tid; q < segs; q += kFThreads) {
        const FusedSeg f = S.seg[q];
        fo.seg_arena[sb + q] = ArenaSeg{tile, q, f.line, (uint32_t)f.name_len, a0 + f.name_ls, f.text};
    }
    const uint32_t* ob4 = S.ob4;
    uint32_t* dst = reinterpret_cast<uint32_t*>(fo.arena + ab);   // 4-byte aligned
    const uint32_t nw4 = ((uint32_t)bytes + 3u) / 4u;
    for (uint32_t w = tid; w < nw4; w += kFThreads) dst[w] = ob4[w];
#ifdef STARCH_TF_PROF
    TPROF(p5);
    if (lane == 0) {
        atomicAdd(&g_tfprof[3], (unsigned long long)(p4 - p3));
        atomicAdd(&g_tfprof[4], (unsigned long long)(p5 - p4));
        atomicAdd(&g_tfprof[5], 1ull);
    }
#endif
}

// after the scans over the tiles (exclusive prefixes of bytes, lines and
// segments in fo.*_pre): every tile's text from its arena slot to its final
// offset, tiles after the first one holding a 0xFF dropped.  The slot is
// staged in LDS with 16-byte loads; the destination is written with 16-byte
// stores from its first 16-aligned byte (each built from five aligned LDS
// words by byte funnel shifts), the bytes before and after bytewise.
__global__ void __launch_bounds__(256) k_tf_place(const FusedOut fo, uint8_t* __restrict__ text, uint32_t ntiles)
{
    __shared__ uint4 buf[kFOut / 16 + 2];
    const uint32_t t = blockIdx.x, tid = threadIdx.x;
    if (t > *fo.first_ff || t >= ntiles) return;
    const uint32_t bytes = fo.tile_bytes[t];
    if (!bytes) return;
    const uint64_t o0 = fo.bytes_pre[t];
    if (o0 + bytes > fo.text_cap) {                 // the host grows the text buffer and reruns
        if (tid == 0) atomicOr(fo.xflags, FX_TEXT_CAP);
        return;
    }
    const uint4* src = reinterpret_cast<const uint4*>(fo.arena + (uint64_t)t * kFOut);
    const uint32_t n16 = (bytes + 15u) / 16u;
    for (uint32_t w = tid; w < n16; w += 256) buf[w] = src[w];
    if (tid == 0) buf[n16] = make_uint4(0, 0, 0, 0);   // the funnel shifts read one word past the end
    __syncthreads();
    const uint8_t* ob = reinterpret_cast<const uint8_t*>(buf);
    const uint32_t* ow = reinterpret_cast<const uint32_t*>(buf);
    uint32_t head = (uint32_t)((16u - (o0 & 15u)) & 15u);
    head = head < bytes ? head : bytes;
    if (tid < head) text[o0 + tid] = ob[tid];
    const uint32_t nw = (bytes - head) / 16u;
    uint4* dst = reinterpret_cast<uint4*>(text + o0 + head);
    const uint32_t sh = head & 3u, wb = head >> 2;
    for (uint32_t w = tid; w < nw; w += 256) {
        const uint32_t* q = ow + wb + 4u * w;
        const uint32_t a0 = q[0], a1 = q[1], a2 = q[2], a3 = q[3], a4 = q[4];
        dst[w] = make_uint4(__builtin_amdgcn_alignbyte(a1, a0, sh), __builtin_amdgcn_alignbyte(a2, a1, sh),
                            __builtin_amdgcn_alignbyte(a3, a2, sh), __builtin_amdgcn_alignbyte(a4, a3, sh));
    }
    for (uint32_t k = head + 16u * nw + tid; k < bytes; k += 256) text[o0 + k] = ob[k];
}

// segment records of the kept tiles at their final index; totals (lines,
// segments, bytes, saw 0xFF) as k_seg_close_dev expects them
__global__ void k_tf_segs(const FusedOut fo, SegInfo* __restrict__ info, uint64_t* __restrict__ totals, uint32_t ntiles)
{
    const uint32_t ff = *fo.first_ff;
    const uint64_t nseg = *fo.seg_ctr < fo.seg_cap ? *fo.seg_ctr : fo.seg_cap;
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i == 0) {
        const uint32_t last = ff < ntiles ? ff + 1 : ntiles;      // tiles kept: [0, last)
        totals[0] = fo.lines_pre[last];
        totals[1] = fo.segs_pre[last];
        totals[2] = fo.bytes_pre[last];
        totals[3] = ff < ntiles ? 1 : 0;
    }
    for (uint64_t j = i; j < nseg; j += (uint64_t)gridDim.x * blockDim.x) {
    const ArenaSeg e = fo.seg_arena[j];
    if (e.tile > ff || fo.segs_pre[e.tile] + e.q >= fo.seg_cap) continue;
    SegInfo& g = info[fo.segs_pre[e.tile] + e.q];
    g.first_line = fo.lines_pre[e.tile] + e.line;
    g.name_off = e.name_off;
    g.name_len = e.name_len;
    g.text_off = fo.bytes_pre[e.tile] + e.text;
    }
}

// line_count / text_len of each segment from its successor; totals on the device
__global__ void k_seg_close_dev(SegInfo* __restrict__ info, const uint64_t* __restrict__ totals, uint64_t seg_cap)
{
    const uint64_t nseg = totals[1], nl = totals[0], ttot = totals[2];
    for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < nseg && s < seg_cap;
         s += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t nf = (s + 1 < nseg) ? info[s + 1].first_line : nl;
        const uint64_t nt = (s + 1 < nseg) ? info[s + 1].text_off : ttot;
        info[s].line_count = nf - info[s].first_line;
        info[s].text_len = nt - info[s].text_off;
    }
}

// ---------------------------------------------------------------------------
// Base counts per segment (transform_state_t.base_count_unique /
// base_count_nonunique, hpp:61-62, declared and zeroed by the reference but
// never computed).  Over a segment's lines, with the start / stop values the
// transform uses (stale sscanf values included): nonunique = sum of (stop -
// start); unique = sum of max(0, stop - max(start, M)), M = the largest stop
// of the segment's earlier lines (INT64_MIN before the first) -- the size of
// the union of the intervals for a BED sorted by start.  Modulo 2^64, as the
// oracle (oracle/starch_oracle.c oracle_base_counts).
//
// M is a segmented max-scan: elements (reset, max) with
// (a, b) -> (a.reset | b.reset, b.reset ? b.max : max(a.max, b.max)).
// Three passes: per-workgroup aggregates, one workgroup scanning them, then
// every line's contribution, reduced per segment in LDS (a workgroup's 256
// lines touch at most 256 segments) and added to the segment's totals.
// ---------------------------------------------------------------------------
struct SegMax { uint32_t r; int64_t m; };
__device__ __forceinline__ SegMax segmax(SegMax a, SegMax b)
{
    return SegMax{a.r | b.r, b.r ? b.m : (a.m > b.m ? a.m : b.m)};
}

// in-workgroup inclusive segmented max-scan over 256 elements (one per thread)
__device__ __forceinline__ SegMax segmax_scan(SegMax x, uint32_t* sr, int64_t* sm)
{
    const int t = threadIdx.x;
    for (int d = 1; d < kThreads; d <<= 1) {
        sr[t] = x.r;
        sm[t] = x.m;
        __syncthreads();
        if (t >= d) x = segmax(SegMax{sr[t - d], sm[t - d]}, x);
        __syncthreads();
    }
    return x;
}

__global__ void __launch_bounds__(kThreads)
k_bc_agg(const int64_t* __restrict__ stop, const uint8_t* __restrict__ flags, uint64_t nl, uint32_t* __restrict__ agg_r,
         int64_t* __restrict__ agg_m)
{
    __shared__ uint32_t sr[kThreads];
    __shared__ int64_t sm[kThreads];
    const uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
    SegMax x{0u, INT64_MIN};
    if (i < nl) x = SegMax{(flags[i] & F_NEW_SEG) ? 1u : 0u, stop[i]};
    x = segmax_scan(x, sr, sm);
    if (threadIdx.x == kThreads - 1) { agg_r[blockIdx.x] = x.r; agg_m[blockIdx.x] = x.m; }
}

// one workgroup: exclusive scan of the workgroup aggregates -> incoming max
__global__ void __launch_bounds__(1024)
k_bc_scan(const uint32_t* __restrict__ agg_r, const int64_t* __restrict__ agg_m, uint64_t nb, int64_t* __restrict__ pre_m)
{
    __shared__ uint32_t cr[1024];
    __shared__ int64_t cm[1024];
    const uint64_t per = (nb + 1023) / 1024, b0 = threadIdx.x * per, b1 = b0 + per < nb ? b0 + per : nb;
    SegMax a{0u, INT64_MIN};
    for (uint64_t b = b0; b < b1; ++b) a = segmax(a, SegMax{agg_r[b], agg_m[b]});
    cr[threadIdx.x] = a.r;
    cm[threadIdx.x] = a.m;
    __syncthreads();
    if (threadIdx.x == 0) {   // exclusive over the 1024 chunk aggregates
        SegMax run{0u, INT64_MIN};
        for (int t = 0; t < 1024; ++t) {
            const SegMax v{cr[t], cm[t]};
            cr[t] = run.r;
            cm[t] = run.m;
            run = segmax(run, v);
        }
    }
    __syncthreads();
    SegMax run{cr[threadIdx.x], cm[threadIdx.x]};
    for (uint64_t b = b0; b < b1; ++b) {
        pre_m[b] = run.m;
        run = segmax(run, SegMax{agg_r[b], agg_m[b]});
    }
}

__global__ void __launch_bounds__(kThreads)
k_bc_final(const int64_t* __restrict__ start, const int64_t* __restrict__ stop, const uint8_t* __restrict__ flags,
           const uint64_t* __restrict__ seg_ord, uint64_t nl, const int64_t* __restrict__ pre_m,
           unsigned long long* __restrict__ out_u, unsigned long long* __restrict__ out_n)
{
    __shared__ uint32_t sr[kThreads];
    __shared__ int64_t sm[kThreads];
    __shared__ unsigned long long lu[kThreads], ln[kThreads];
    const int t = threadIdx.x;
    const uint64_t L0 = (uint64_t)blockIdx.x * kThreads, i = L0 + t;
    const bool valid = i < nl;
    const uint32_t f = valid && (flags[i] & F_NEW_SEG) ? 1u : 0u;
    const int64_t a = valid ? start[i] : 0, b = valid ? stop[i] : INT64_MIN;
    lu[t] = 0;
    ln[t] = 0;
    const SegMax incl = segmax_scan(SegMax{f, b}, sr, sm);   // (ends with __syncthreads)
    sr[t] = incl.r;
    sm[t] = incl.m;
    __syncthreads();
    // the max over the segment's earlier lines: the previous line's inclusive
    // value, after the workgroup's incoming one; nothing for a segment's first line
    SegMax prev{0u, pre_m[blockIdx.x]};
    if (t > 0) prev = segmax(prev, SegMax{sr[t - 1], sm[t - 1]});
    if (valid) {
        const int64_t M = f ? INT64_MIN : prev.m;
        const int64_t lo = M > a ? M : a;
        const unsigned long long u = b > lo ? (unsigned long long)((uint64_t)b - (uint64_t)lo) : 0ull;
        const unsigned long long cd = (unsigned long long)((uint64_t)b - (uint64_t)a);
        const uint64_t seg = seg_ord[i] + f - 1, sb = seg_ord[L0] + ((flags[L0] & F_NEW_SEG) ? 1u : 0u) - 1;
        atomicAdd(&lu[seg - sb], u);
        atomicAdd(&ln[seg - sb], cd);
    }
    __syncthreads();
    const uint64_t Lm = (L0 + kThreads < nl ? L0 + kThreads : nl) - 1;
    const uint64_t sb = seg_ord[L0] + ((flags[L0] & F_NEW_SEG) ? 1u : 0u) - 1;
    const uint64_t se = seg_ord[Lm] + ((flags[Lm] & F_NEW_SEG) ? 1u : 0u) - 1;
    if ((uint64_t)t <= se - sb) {
        atomicAdd(out_u + sb + t, lu[t]);
        atomicAdd(out_n + sb + t, ln[t]);
    }
}

__global__ void k_bc_flag(const uint8_t* __restrict__ flags, uint64_t nl, uint32_t* __restrict__ seg_flag)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nl) seg_flag[i] = (flags[i] & F_NEW_SEG) ? 1u : 0u;
}

}  // namespace tf

// ---------------------------------------------------------------------------
// Host driver
// ---------------------------------------------------------------------------
using namespace tf;

void TransformWorkspace::run(const uint8_t* d_bed, uint64_t n, hipStream_t st, TransformResult& res, int64_t init_start,
                             int64_t init_stop)
{
    res = TransformResult();
    // STARCH_TF=2pass / fused forces a path; by default the single pass runs
    // unless the last input produced more than 0.6 text bytes per input byte
    // (long remainder columns, e.g. narrowPeak: there the two-pass kernels,
    // which stage exactly 256 lines per workgroup, measured faster)
    static const int force = [] {
        const char* e = getenv("STARCH_TF");
        return !e ? 0 : !strcmp(e, "2pass") ? 2 : !strcmp(e, "fused") ? 1 : 0;
    }();
    if (n == 0 || force == 2 || (force == 0 && ratio_seen && text_ratio > 0.6))
        return run_two_pass(d_bed, n, st, res, init_start, init_stop);
    const uint32_t ntiles = (uint32_t)ceil_div(n, kFT);
    // per-tile counts (u32 x 3), their exclusive prefixes (u64 x 3, ntiles + 1
    // each)
    uint64_t* fw = b_faggs.as<uint64_t>(8ull * ntiles + 64);
    FusedOut fo;
    fo.tile_bytes = reinterpret_cast<uint32_t*>(fw);
    fo.tile_lines = fo.tile_bytes + ntiles;
    fo.tile_segs = fo.tile_lines + ntiles;
    fo.bytes_pre = fw + (3ull * ntiles + 2) / 2 + 1;
    fo.lines_pre = fo.bytes_pre + ntiles + 1;
    fo.segs_pre = fo.lines_pre + ntiles + 1;
    uint64_t* fx = b_fx.as<uint64_t>(16);   // [0..3] totals (lines, segments, bytes, saw 0xFF), [4] flags, [5] first 0xFF tile, [7] segs
    fo.first_ff = reinterpret_cast<uint32_t*>(fx + 5);
    fo.xflags = reinterpret_cast<uint32_t*>(fx + 4);
    fo.seg_ctr = reinterpret_cast<unsigned long long*>(fx + 7);
    uint64_t tcap = std::max<uint64_t>(1u << 20, (uint64_t)(text_ratio * 1.05 * (double)n) + 4096);
    uint64_t scap = std::max<uint64_t>(4096, 2 * seg_hint);
    for (int attempt = 0; attempt < 3; ++attempt) {
        uint8_t* txt = b_text.as<uint8_t>(tcap + 64);
        SegInfo* info = b_seg_info.as<SegInfo>(scap + 1);
        fo.arena = b_arena.as<uint8_t>((uint64_t)ntiles * kFOut + 64);   // one kFOut slot per tile
        fo.text_cap = tcap;
        fo.seg_arena = b_seg_arena.as<ArenaSeg>(scap + 1);
        fo.seg_cap = scap;
        HIP_CHECK(hipMemsetAsync(fx, 0, 8 * sizeof(uint64_t), st));
        HIP_CHECK(hipMemsetAsync(fo.first_ff, 0xFF, sizeof(uint32_t), st));
        // STARCH_TF_DBG (timing experiments only, wrong output): 1 parse without
        // the arena write, 2 staging + masks only, 3 parse + lengths without text
        static const uint32_t dbg_mode = getenv("STARCH_TF_DBG") ? (uint32_t)atoi(getenv("STARCH_TF_DBG")) : 0u;
        hipLaunchKernelGGL(k_tf_fused, dim3(ntiles), dim3(kFThreads), 0, st, d_bed, n, fo,
                           reinterpret_cast<uint32_t*>(fx + 4), dbg_mode);
        scan::excl_sum_u32_to_u64(fo.tile_bytes, fo.bytes_pre, ntiles, fo.bytes_pre + ntiles, b_tmp, st);
        scan::excl_sum_u32_to_u64(fo.tile_lines, fo.lines_pre, ntiles, fo.lines_pre + ntiles, b_tmp, st);
        scan::excl_sum_u32_to_u64(fo.tile_segs, fo.segs_pre, ntiles, fo.segs_pre + ntiles, b_tmp, st);
        hipLaunchKernelGGL(k_tf_place, dim3(ntiles), dim3(256), 0, st, fo, txt, ntiles);
        const uint32_t sg = (uint32_t)std::min<uint64_t>(65535, ceil_div(scap, 256));
        hipLaunchKernelGGL(k_tf_segs, dim3(sg), dim3(256), 0, st, fo, info, fx, ntiles);
        const uint32_t cg = (uint32_t)std::min<uint64_t>(1024, ceil_div(scap, 256));
        hipLaunchKernelGGL(k_seg_close_dev, dim3(cg), dim3(256), 0, st, info, fx, scap);
        HIP_CHECK(hipGetLastError());
        uint64_t h[5];
        HIP_CHECK(hipMemcpyAsync(h, fx, sizeof(h), hipMemcpyDeviceToHost, st));
        HIP_CHECK(hipStreamSynchronize(st));
        const uint32_t flags = (uint32_t)h[4];
        static const bool dbg = getenv("STARCH_TF_DEBUG") != nullptr;
        if (dbg) fprintf(stderr, "[tf] attempt %d flags %u lines %llu segs %llu bytes %llu\n", attempt, flags,
                         (unsigned long long)h[0], (unsigned long long)h[1], (unsigned long long)h[2]);
        if (flags & (FX_FAIL | FX_FALLBACK)) break;                 // stale values / long lines: two-pass path
        if (flags & (FX_TEXT_CAP | FX_SEG_CAP)) {                     // grow to the exact totals and rerun
            tcap = std::max(tcap, h[2] + 64);
            scap = std::max(scap, h[1] + 1);
            continue;
        }
#ifdef STARCH_TF_PROF
        {
            unsigned long long g[8];
            HIP_CHECK(hipMemcpyFromSymbol(g, HIP_SYMBOL(g_tfprof), sizeof(g)));
            static const unsigned long long zero[8] = {};
            HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_tfprof), zero, sizeof(zero)));
            const char* nm[5] = {"stage", "masks+nl-scan+halo", "fused_lines", "counts+arena alloc", "arena write"};
            const double tot = (double)(g[0] + g[1] + g[2] + g[3] + g[4]);
            for (int q = 0; q < 5; ++q)
                fprintf(stderr, "[tfprof] %-20s %14llu (%.1f%%)\n", nm[q], g[q], 100.0 * (double)g[q] / (tot ? tot : 1));
            fprintf(stderr, "[tfprof] waves %llu, cycles per wave-tile %.0f\n", g[5], tot / (double)(g[5] ? g[5] : 1));
        }
#endif
        res.n_lines = h[0];
        res.n_segments = h[1];
        res.text_bytes = h[2];
        res.ff_pos = h[3] ? 0 : ~0ull;                                 // (a 0xFF was met; its offset is not kept)
        text_ratio = (double)h[2] / (double)n;
        ratio_seen = true;
        seg_hint = h[1];
        text = txt;
        seg_info_dev = info;
        return;
    }
    run_two_pass(d_bed, n, st, res, init_start, init_stop);
}

uint64_t TransformWorkspace::index_lines(const uint8_t* d_bed, uint64_t n, hipStream_t st, uint64_t* ff_pos)
{
    uint64_t ntile = ceil_div(n, kTileBytes);
    uint32_t* tile_cnt = b_tile_cnt.as<uint32_t>(ntile + 1);
    uint64_t* tile_off = b_tile_off.as<uint64_t>(ntile + 1);
    uint64_t* scal = b_scal.as<uint64_t>(16);
    HIP_CHECK(hipMemsetAsync(scal, 0, 16 * sizeof(uint64_t), st));
    HIP_CHECK(hipMemsetAsync(scal + 1, 0xff, sizeof(uint64_t), st));
    if (n > 0) {
        hipLaunchKernelGGL(k_count_nl, dim3((unsigned)ntile), dim3(kThreads), 0, st, d_bed, n, tile_cnt,
                           (unsigned long long*)(scal + 1));
        scan::excl_sum_u32_to_u64(tile_cnt, tile_off, ntile, scal + 0, b_tmp, st);
    }
    uint64_t h[2];
    HIP_CHECK(hipMemcpyAsync(h, scal, 2 * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    uint64_t nl = h[0];
    uint64_t* line_end = b_line_end.as<uint64_t>(nl + 1);
    if (nl) {
        hipLaunchKernelGGL(k_index_nl, dim3((unsigned)ntile), dim3(kThreads), 0, st, d_bed, n, tile_off, line_end);
        if (h[1] != ~0ull) {
            hipLaunchKernelGGL(k_lines_before, dim3(1), dim3(1), 0, st, line_end, nl,
                               (const unsigned long long*)(scal + 1), scal + 2);
            HIP_CHECK(hipMemcpyAsync(&nl, scal + 2, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
            HIP_CHECK(hipStreamSynchronize(st));
        }
    }
    if (ff_pos) *ff_pos = h[1];
    return nl;
}

void TransformWorkspace::base_counts(const uint8_t* d_bed, uint64_t n, hipStream_t st, int64_t init_start,
                                     int64_t init_stop, std::vector<uint64_t>& unique, std::vector<uint64_t>& nonunique)
{
    unique.clear();
    nonunique.clear();
    const uint64_t nl = index_lines(d_bed, n, st, nullptr);
    if (nl == 0) return;
    const uint64_t* line_end = static_cast<const uint64_t*>(b_line_end.p);
    const unsigned nb = (unsigned)ceil_div(nl, kThreads);
    uint64_t* scal = b_scal.as<uint64_t>(16);
    uint32_t* any_fail = reinterpret_cast<uint32_t*>(scal + 5);
    int64_t* start = b_start.as<int64_t>(nl);
    int64_t* stop = b_stop.as<int64_t>(nl);
    uint8_t* flags = b_flags.as<uint8_t>(nl);
    hipLaunchKernelGGL(k_parse, dim3(nb), dim3(kThreads), 0, st, d_bed, line_end, nl, start, stop, flags,
                       b_rem_beg.as<uint64_t>(nl), b_rem_len.as<uint32_t>(nl), b_chr_len.as<uint32_t>(nl), any_fail);
    uint64_t* idx = b_idx.as<uint64_t>(nl);
    for (int w = 0; w < 2; ++w) {   // stale values, as the general path (hpp:306-316)
        hipLaunchKernelGGL(k_ok_index, dim3(nb), dim3(kThreads), 0, st, flags, nl,
                           (uint8_t)(w == 0 ? F_START_OK : F_STOP_OK), idx);
        scan::incl_max_u64(idx, nl, b_tmp, st);
        int64_t* v = (w == 0) ? start : stop;
        int64_t* cp = b_vcopy.as<int64_t>(nl);
        HIP_CHECK(hipMemcpyAsync(cp, v, nl * sizeof(int64_t), hipMemcpyDeviceToDevice, st));
        hipLaunchKernelGGL(k_gather_stale, dim3(nb), dim3(kThreads), 0, st, cp, idx, nl, w == 0 ? init_start : init_stop,
                           v);
    }
    uint32_t* seg_flag = b_seg_flag.as<uint32_t>(nl);
    uint64_t* seg_ord = b_seg_ord.as<uint64_t>(nl);
    hipLaunchKernelGGL(k_bc_flag, dim3(nb), dim3(kThreads), 0, st, flags, nl, seg_flag);
    scan::excl_sum_u32_to_u64(seg_flag, seg_ord, nl, scal + 3, b_tmp, st);
    uint64_t nseg = 0;
    HIP_CHECK(hipMemcpyAsync(&nseg, scal + 3, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
    // aggregates / incoming maxima live in the (now free) index buffers
    uint32_t* agg_r = b_out_len.as<uint32_t>(nb + 1);
    int64_t* agg_m = reinterpret_cast<int64_t*>(b_vcopy.as<int64_t>(nl > 2ull * nb ? nl : 2ull * nb));
    int64_t* pre_m = agg_m + nb;
    hipLaunchKernelGGL(k_bc_agg, dim3(nb), dim3(kThreads), 0, st, stop, flags, nl, agg_r, agg_m);
    hipLaunchKernelGGL(k_bc_scan, dim3(1), dim3(1024), 0, st, agg_r, agg_m, (uint64_t)nb, pre_m);
    HIP_CHECK(hipStreamSynchronize(st));
    unsigned long long* out = reinterpret_cast<unsigned long long*>(b_seg_first.as<uint64_t>(2 * nseg + 2));
    HIP_CHECK(hipMemsetAsync(out, 0, (2 * nseg + 2) * sizeof(uint64_t), st));
    hipLaunchKernelGGL(k_bc_final, dim3(nb), dim3(kThreads), 0, st, start, stop, flags, seg_ord, nl, pre_m, out,
                       out + nseg);
    HIP_CHECK(hipGetLastError());
    unique.resize(nseg);
    nonunique.resize(nseg);
    if (nseg) {
        HIP_CHECK(hipMemcpyAsync(unique.data(), out, nseg * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
        HIP_CHECK(hipMemcpyAsync(nonunique.data(), out + nseg, nseg * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
    }
    HIP_CHECK(hipStreamSynchronize(st));
}

void TransformWorkspace::run_two_pass(const uint8_t* d_bed, uint64_t n, hipStream_t st, TransformResult& res,
                                      int64_t init_start, int64_t init_stop)
{
    res = TransformResult();
    uint64_t ntile = ceil_div(n, kTileBytes);
    uint32_t* tile_cnt = b_tile_cnt.as<uint32_t>(ntile + 1);
    uint64_t* tile_off = b_tile_off.as<uint64_t>(ntile + 1);
    uint64_t* scal = b_scal.as<uint64_t>(16);      // [0]=nl_total [1]=ff_pos [2]=nl_eff [3]=nseg [4]=text_total [5]=any_fail
    HIP_CHECK(hipMemsetAsync(scal, 0, 16 * sizeof(uint64_t), st));
    HIP_CHECK(hipMemsetAsync(scal + 1, 0xff, sizeof(uint64_t), st));
    if (n > 0) {
        hipLaunchKernelGGL(k_count_nl, dim3((unsigned)ntile), dim3(kThreads), 0, st, d_bed, n, tile_cnt,
                           (unsigned long long*)(scal + 1));
        scan::excl_sum_u32_to_u64(tile_cnt, tile_off, ntile, scal + 0, b_tmp, st);
    }
    uint64_t h[2];
    HIP_CHECK(hipMemcpyAsync(h, scal, 2 * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    uint64_t nl = h[0];
    uint64_t* line_end = b_line_end.as<uint64_t>(nl + 1);
    if (nl) {
        hipLaunchKernelGGL(k_index_nl, dim3((unsigned)ntile), dim3(kThreads), 0, st, d_bed, n, tile_off, line_end);
        if (h[1] != ~0ull) {
            hipLaunchKernelGGL(k_lines_before, dim3(1), dim3(1), 0, st, line_end, nl,
                               (const unsigned long long*)(scal + 1), scal + 2);
            HIP_CHECK(hipMemcpyAsync(&nl, scal + 2, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
            HIP_CHECK(hipStreamSynchronize(st));
        }
    }
    res.n_lines = nl;
    res.ff_pos = h[1];
    if (nl == 0) { res.n_segments = 0; res.text_bytes = 0; return; }

    uint32_t* any_fail = reinterpret_cast<uint32_t*>(scal + 5);
    const unsigned nb = (unsigned)ceil_div(nl, kThreads);
    // fused path: pass 1 -> per-workgroup bytes / segments
    uint64_t* wg_len = b_out_off.as<uint64_t>(2ull * nb + 2);
    uint64_t* wg_off = wg_len + nb + 1;
    uint32_t* wg_seg = b_seg_flag.as<uint32_t>(nb + 1);
    uint64_t* wg_sego = b_seg_ord.as<uint64_t>(nb + 1);
    auto lds_cap = [](double per_line, uint32_t lo, uint32_t hi) {
        const double want = 1.3 * (kThreads + 1) * per_line + 256.0;
        uint32_t c = want > hi ? hi : (uint32_t)want;
        c = (c + 1023u) & ~1023u;
        return c < lo ? lo : (c > hi ? hi : c);
    };
    const uint32_t cap = lds_cap((double)n / (double)nl, 4096, kTfCapMax);
    hipLaunchKernelGGL(k_tf1, dim3(nb), dim3(kThreads), cap + kStagePad, st, d_bed, line_end, nl, wg_len, wg_seg,
                       any_fail, cap);
    scan::excl_sum_u64(wg_len, wg_off, nb, scal + 4, b_tmp, st);
    scan::excl_sum_u32_to_u64(wg_seg, wg_sego, nb, scal + 3, b_tmp, st);
    uint32_t fail = 0;
    HIP_CHECK(hipMemcpyAsync(h, scal + 3, 2 * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipMemcpyAsync(&fail, any_fail, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    uint64_t nseg = h[0], ttot = h[1];
    SegInfo* info = nullptr;
    if (!fail) {
        info = b_seg_info.as<SegInfo>(nseg + 1);
        text = b_text.as<uint8_t>(ttot + 64);
        const uint32_t ocap = lds_cap((double)ttot / (double)nl, 2048, kTfOutCapMax);
        hipLaunchKernelGGL(k_tf2, dim3(nb), dim3(kThreads), cap + kStagePad + ocap, st, d_bed, line_end, nl, wg_off,
                           wg_sego, text, info, cap, ocap);
        hipLaunchKernelGGL(k_seg_close, dim3((unsigned)ceil_div(nseg, 256)), dim3(256), 0, st, info, nseg, nl,
                           ttot);
    } else {
        // general path: some start/stop does not parse (stale values, hpp:306-316)
        res.general = true;
        int64_t* start = b_start.as<int64_t>(nl);
        int64_t* stop = b_stop.as<int64_t>(nl);
        uint8_t* flags = b_flags.as<uint8_t>(nl);
        uint64_t* rem_beg = b_rem_beg.as<uint64_t>(nl);
        uint32_t* rem_len = b_rem_len.as<uint32_t>(nl);
        uint32_t* chr_len = b_chr_len.as<uint32_t>(nl);
        hipLaunchKernelGGL(k_parse, dim3(nb), dim3(kThreads), 0, st, d_bed, line_end, nl, start, stop, flags,
                           rem_beg, rem_len, chr_len, any_fail);
        uint64_t* idx = b_idx.as<uint64_t>(nl);
        for (int w = 0; w < 2; ++w) {
            hipLaunchKernelGGL(k_ok_index, dim3(nb), dim3(kThreads), 0, st, flags, nl,
                               (uint8_t)(w == 0 ? F_START_OK : F_STOP_OK), idx);
            scan::incl_max_u64(idx, nl, b_tmp, st);
            // gather into a copy to avoid read/write races across blocks
            int64_t* v = (w == 0) ? start : stop;
            int64_t* cp = b_vcopy.as<int64_t>(nl);
            HIP_CHECK(hipMemcpyAsync(cp, v, nl * sizeof(int64_t), hipMemcpyDeviceToDevice, st));
            hipLaunchKernelGGL(k_gather_stale, dim3(nb), dim3(kThreads), 0, st, cp, idx, nl, w == 0 ? init_start : init_stop,
                               v);
        }
        uint32_t* out_len = b_out_len.as<uint32_t>(nl);
        uint32_t* seg_flag = b_seg_flag.as<uint32_t>(nl);
        hipLaunchKernelGGL(k_line_len, dim3(nb), dim3(kThreads), 0, st, start, stop, flags, rem_len, nl, out_len,
                           seg_flag);
        uint64_t* out_off = b_out_off.as<uint64_t>(nl);
        uint64_t* seg_ord = b_seg_ord.as<uint64_t>(nl);
        scan::excl_sum_u32_to_u64(out_len, out_off, nl, scal + 4, b_tmp, st);
        scan::excl_sum_u32_to_u64(seg_flag, seg_ord, nl, scal + 3, b_tmp, st);
        HIP_CHECK(hipMemcpyAsync(h, scal + 3, 2 * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
        HIP_CHECK(hipStreamSynchronize(st));
        nseg = h[0];
        ttot = h[1];
        uint64_t* seg_first = b_seg_first.as<uint64_t>(nseg + 1);
        hipLaunchKernelGGL(k_seg_first, dim3(nb), dim3(kThreads), 0, st, seg_flag, seg_ord, nl, seg_first);
        info = b_seg_info.as<SegInfo>(nseg + 1);
        hipLaunchKernelGGL(k_seg_info, dim3((unsigned)ceil_div(nseg, 256)), dim3(256), 0, st, seg_first, nseg, nl,
                           line_end, chr_len, out_off, ttot, info);
        text = b_text.as<uint8_t>(ttot + 64);
        hipLaunchKernelGGL(k_emit, dim3(nb), dim3(kThreads), 0, st, d_bed, start, stop, flags, rem_beg, rem_len,
                           out_off, nl, text);
    }
    HIP_CHECK(hipGetLastError());
    res.n_segments = nseg;
    res.text_bytes = ttot;
    seg_info_dev = info;
    if (n) {
        text_ratio = (double)ttot / (double)n;
        ratio_seen = true;
    }
}
