// starch_amd/csrc/untransform.hip -- inverse Starch coordinate transform on
// MI355X (the unstarch half): segment texts -> BED lines.
//
// The forward transform (hpp:428-504) writes, per line of a segment,
// "p<cd>\n" when cd = stop - start changes (cd starts at 0 per segment), then
// "<v>[\t<rem>]\n" with v = start - last_stop (v = start while last_stop is 0;
// last_stop starts at 0 per segment).  Inverting it:
//   cd_i   = the value of the last p-line at or before line i of its segment
//            (0 before the first): a max-scan of line indices
//   stop_i = sum over the segment's value lines j <= i of (v_j + cd_j)
//            (start_i = v_i + stop_{i-1}, including the last_stop == 0 case):
//            a global inclusive sum minus the segment's base, modulo 2^64
//   start_i = stop_i - cd_i
// and each value line prints "<chr>\t<start>\t<stop>[\t<rem>]\n".  Exact for
// canonical BED (decimal coordinates, stop >= start).  A p-line with a
// negative value is refused: the forward transform drops that line's newline
// (hpp:440,452, n_digits quirk), so its boundary with the next line is lost.
#include "transform.hpp"
#include "untransform.hpp"

#include <algorithm>
#include <string.h>

namespace ut {
namespace {

constexpr int kT = 256;

struct LineRec {
    int64_t val;          // cd (p-line) or v (value line)
    uint64_t rem_b;       // text offset of the remainder (after the tab)
    uint32_t rem_len;
    uint32_t flags;       // bit0 p-line, bit1 has tab, bit2 segment start, bit3 malformed
};
enum : uint32_t { L_P = 1, L_TAB = 2, L_SEG = 4, L_BAD = 8 };

__device__ __forceinline__ bool parse_i64(const uint8_t* t, uint64_t b, uint64_t e, int64_t& v)
{
    bool neg = false;
    if (b < e && t[b] == '-') { neg = true; ++b; }
    if (b >= e || e - b > 19) return false;
    uint64_t a = 0;
    for (uint64_t k = b; k < e; ++k) {
        const uint32_t d = (uint32_t)t[k] - 48u;
        if (d > 9u) return false;
        a = a * 10u + d;
    }
    v = neg ? (int64_t)(0ull - a) : (int64_t)a;
    return true;
}

// one thread per line: classify and parse; seg_off: sorted segment text offsets
__global__ void __launch_bounds__(kT) k_ut_parse(const uint8_t* __restrict__ t, const uint64_t* __restrict__ line_end,
                                                 uint64_t nl, const uint64_t* __restrict__ seg_off, uint32_t nseg,
                                                 LineRec* __restrict__ rec, uint64_t* __restrict__ key,
                                                 uint32_t* __restrict__ seg_first, uint32_t* __restrict__ bad)
{
    const uint64_t i = (uint64_t)blockIdx.x * kT + threadIdx.x;
    if (i >= nl) return;
    const uint64_t ls = i ? line_end[i - 1] : 0, le = line_end[i] - 1;   // le: the '\n'
    LineRec r{0, 0, 0, 0};
    // segment start: ls is some segment's text offset
    uint32_t lo = 0, hi = nseg;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (seg_off[mid] <= ls) lo = mid; else hi = mid;
    }
    if (seg_off[lo] == ls) {
        r.flags |= L_SEG;
        seg_first[lo] = (uint32_t)i;
    }
    bool ok;
    if (ls < le && t[ls] == 'p') {
        r.flags |= L_P;
        ok = parse_i64(t, ls + 1, le, r.val) && r.val >= 0;
    } else {
        uint64_t e = ls;
        while (e < le && t[e] != '\t') ++e;
        ok = parse_i64(t, ls, e, r.val);
        if (e < le) {
            r.flags |= L_TAB;
            r.rem_b = e + 1;
            r.rem_len = (uint32_t)(le - e - 1);
        }
    }
    if (!ok) {
        r.flags |= L_BAD;
        atomicOr(bad, 1u);
    }
    rec[i] = r;
    key[i] = (r.flags & (L_P | L_SEG)) ? i + 1 : 0;   // max-scan: the last p-line or segment start
}

// cd of every line and its (v + cd) contribution to the stop sum
__global__ void __launch_bounds__(kT) k_ut_contrib(const LineRec* __restrict__ rec, const uint64_t* __restrict__ key,
                                                   uint64_t nl, int64_t* __restrict__ cd, uint64_t* __restrict__ contrib)
{
    const uint64_t i = (uint64_t)blockIdx.x * kT + threadIdx.x;
    if (i >= nl) return;
    const uint64_t j = key[i] - 1;                     // >= 0: line 0 starts a segment
    const int64_t c = (rec[j].flags & L_P) ? rec[j].val : 0;
    cd[i] = c;
    contrib[i] = (rec[i].flags & L_P) ? 0ull : (uint64_t)rec[i].val + (uint64_t)c;
}

__device__ __forceinline__ uint32_t dec_len_i64(int64_t v)
{
    uint64_t u = v < 0 ? 0ull - (uint64_t)v : (uint64_t)v;
    uint32_t n = 1;
    while (u >= 10) { u /= 10; ++n; }
    return n + (v < 0 ? 1u : 0u);
}

__device__ __forceinline__ uint32_t put_i64(uint8_t* o, int64_t v)
{
    uint64_t u = v < 0 ? 0ull - (uint64_t)v : (uint64_t)v;
    uint32_t k = 0;
    if (v < 0) o[k++] = '-';
    const uint32_t nd = dec_len_i64(v) - k;
    for (int d = (int)nd - 1; d >= 0; --d) { o[k + d] = (uint8_t)('0' + u % 10u); u /= 10u; }
    return k + nd;
}

// stop / start of every value line and its output length (p-lines: 0).
// seg_of(i) = the last segment whose first line is <= i.
__device__ __forceinline__ uint32_t seg_of(const uint32_t* seg_first, uint32_t nseg, uint64_t i)
{
    uint32_t lo = 0, hi = nseg;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (seg_first[mid] <= i) lo = mid; else hi = mid;
    }
    return lo;
}

__global__ void __launch_bounds__(kT) k_ut_len(const LineRec* __restrict__ rec, const int64_t* __restrict__ cd,
                                               const uint64_t* __restrict__ excl, const uint64_t* __restrict__ contrib,
                                               const uint32_t* __restrict__ seg_first, const uint64_t* __restrict__ name_len,
                                               uint32_t nseg, uint64_t nl, int64_t* __restrict__ stop,
                                               uint64_t* __restrict__ olen)
{
    const uint64_t i = (uint64_t)blockIdx.x * kT + threadIdx.x;
    if (i >= nl) return;
    const uint32_t s = seg_of(seg_first, nseg, i);
    const int64_t sp = (int64_t)(excl[i] + contrib[i] - excl[seg_first[s]]);
    stop[i] = sp;
    const LineRec r = rec[i];
    if (r.flags & L_P) { olen[i] = 0; return; }
    const int64_t st = (int64_t)((uint64_t)sp - (uint64_t)cd[i]);
    olen[i] = name_len[s] + 1 + dec_len_i64(st) + 1 + dec_len_i64(sp) + ((r.flags & L_TAB) ? 1 + r.rem_len : 0) + 1;
}

__global__ void __launch_bounds__(kT) k_ut_write(const uint8_t* __restrict__ t, const LineRec* __restrict__ rec,
                                                 const int64_t* __restrict__ cd, const int64_t* __restrict__ stop,
                                                 const uint64_t* __restrict__ ooff, const uint32_t* __restrict__ seg_first,
                                                 const uint64_t* __restrict__ name_off, const uint64_t* __restrict__ name_len,
                                                 const uint8_t* __restrict__ names, uint32_t nseg, uint64_t nl,
                                                 uint8_t* __restrict__ out)
{
    const uint64_t i = (uint64_t)blockIdx.x * kT + threadIdx.x;
    if (i >= nl) return;
    const LineRec r = rec[i];
    if (r.flags & L_P) return;
    const uint32_t s = seg_of(seg_first, nseg, i);
    uint8_t* o = out + ooff[i];
    const uint8_t* nm = names + name_off[s];
    const uint64_t nlen = name_len[s];
    for (uint64_t k = 0; k < nlen; ++k) o[k] = nm[k];
    o += nlen;
    *o++ = '\t';
    const int64_t sp = stop[i];
    o += put_i64(o, (int64_t)((uint64_t)sp - (uint64_t)cd[i]));
    *o++ = '\t';
    o += put_i64(o, sp);
    if (r.flags & L_TAB) {
        *o++ = '\t';
        for (uint32_t k = 0; k < r.rem_len; ++k) o[k] = t[r.rem_b + k];
        o += r.rem_len;
    }
    *o = '\n';
}

}  // namespace

uint64_t Untransform::run(TransformWorkspace& tf, const uint8_t* d_text, uint64_t n, const std::vector<Seg>& segs,
                          hipStream_t st, DevBuf& out)
{
    if (n == 0 || segs.empty()) {
        out.as<uint8_t>(64);
        return 0;
    }
    const uint32_t nseg = (uint32_t)segs.size();
    for (uint32_t s = 0; s < nseg; ++s) {
        if (s && segs[s].text_off < segs[s - 1].text_off + segs[s - 1].text_len)
            throw StarchError(-2, "untransform: segments must be in text order");
        if (segs[s].text_len && segs[s].text_off + segs[s].text_len > n)
            throw StarchError(-2, "untransform: segment outside the text");
    }
    uint64_t ff = ~0ull;
    const uint64_t nl = tf.index_lines(d_text, n, st, &ff);
    const uint64_t* line_end = tf.b_line_end.as<uint64_t>(nl + 1);
    // every segment must end with a newline and hold at least one line;
    // segments are contiguous in line space (text order)
    std::vector<uint64_t> h_off(nseg), h_nlen(nseg), h_noff(nseg);
    std::string names;
    uint64_t covered = 0;
    for (uint32_t s = 0; s < nseg; ++s) {
        h_off[s] = segs[s].text_off;
        h_noff[s] = names.size();
        h_nlen[s] = segs[s].name.size();
        names += segs[s].name;
        covered += segs[s].text_len;
    }
    if (ff != ~0ull) throw StarchError(-12, "untransform: byte 0xFF in the text");
    uint64_t* d_segoff = b_seg.as<uint64_t>(3ull * nseg + 8);
    uint64_t* d_noff = d_segoff + nseg;
    uint64_t* d_nlen = d_noff + nseg;
    uint8_t* d_names = b_names.as<uint8_t>(names.size() + 64);
    uint32_t* d_segfirst = b_segfirst.as<uint32_t>(nseg + 8);
    uint32_t* d_bad = d_segfirst + nseg + 4;
    HIP_CHECK(hipMemcpyAsync(d_segoff, h_off.data(), nseg * sizeof(uint64_t), hipMemcpyHostToDevice, st));
    HIP_CHECK(hipMemcpyAsync(d_noff, h_noff.data(), nseg * sizeof(uint64_t), hipMemcpyHostToDevice, st));
    HIP_CHECK(hipMemcpyAsync(d_nlen, h_nlen.data(), nseg * sizeof(uint64_t), hipMemcpyHostToDevice, st));
    if (!names.empty()) HIP_CHECK(hipMemcpyAsync(d_names, names.data(), names.size(), hipMemcpyHostToDevice, st));
    HIP_CHECK(hipMemsetAsync(d_segfirst, 0xFF, (nseg + 8) * sizeof(uint32_t), st));
    HIP_CHECK(hipMemsetAsync(d_bad, 0, sizeof(uint32_t), st));
    LineRec* d_rec = reinterpret_cast<LineRec*>(b_rec.as<uint8_t>((nl + 1) * sizeof(LineRec)));
    uint64_t* d_key = b_key.as<uint64_t>(nl + 1);
    int64_t* d_cd = b_cd.as<int64_t>(nl + 1);
    uint64_t* d_contrib = b_contrib.as<uint64_t>(nl + 1);
    uint64_t* d_excl = b_excl.as<uint64_t>(nl + 2);
    int64_t* d_stop = b_stop.as<int64_t>(nl + 1);
    uint64_t* d_olen = b_olen.as<uint64_t>(nl + 2);
    const unsigned g = (unsigned)ceil_div(nl, kT);
    if (nl) {
        hipLaunchKernelGGL(k_ut_parse, dim3(g), dim3(kT), 0, st, d_text, line_end, nl, d_segoff, nseg, d_rec, d_key,
                           d_segfirst, d_bad);
        scan::incl_max_u64(d_key, nl, b_tmp, st);
        hipLaunchKernelGGL(k_ut_contrib, dim3(g), dim3(kT), 0, st, d_rec, d_key, nl, d_cd, d_contrib);
        scan::excl_sum_u64(d_contrib, d_excl, nl, d_excl + nl, b_tmp, st);
    }
    HIP_CHECK(hipGetLastError());
    std::vector<uint32_t> segfirst(nseg);
    uint32_t bad = 0;
    HIP_CHECK(hipMemcpyAsync(segfirst.data(), d_segfirst, nseg * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipMemcpyAsync(&bad, d_bad, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    if (bad) throw StarchError(-12, "untransform: malformed line (or a negative p-value, whose newline the "
                                    "forward transform drops)");
    for (uint32_t s = 0; s < nseg; ++s) {
        if (segs[s].text_len == 0 || segfirst[s] == 0xFFFFFFFFu)
            throw StarchError(-12, "untransform: segment " + std::to_string(s) + " does not start a line");
        if (s && segfirst[s] <= segfirst[s - 1]) throw StarchError(-12, "untransform: empty segment");
    }
    uint64_t last_end = 0;
    if (nl) HIP_CHECK(hipMemcpy(&last_end, line_end + nl - 1, sizeof(uint64_t), hipMemcpyDeviceToHost));
    if (segfirst[0] != 0 || covered != n || last_end != n)
        throw StarchError(-12, "untransform: segments must cover the text, every line ending in a newline");
    hipLaunchKernelGGL(k_ut_len, dim3(g), dim3(kT), 0, st, d_rec, d_cd, d_excl, d_contrib, d_segfirst, d_nlen, nseg,
                       nl, d_stop, d_olen);
    uint64_t* d_ooff = d_key;                          // the keys are dead
    scan::excl_sum_u64(d_olen, d_ooff, nl, d_olen + nl, b_tmp, st);
    uint64_t total = 0;
    HIP_CHECK(hipMemcpyAsync(&total, d_olen + nl, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    uint8_t* d_out = out.as<uint8_t>(total + 64);
    hipLaunchKernelGGL(k_ut_write, dim3(g), dim3(kT), 0, st, d_text, d_rec, d_cd, d_stop, d_ooff, d_segfirst, d_noff,
                       d_nlen, d_names, nseg, nl, d_out);
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipStreamSynchronize(st));
    return total;
}

}  // namespace ut
