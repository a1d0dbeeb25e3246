// starch_amd/csrc/shard.cpp -- host-side shard planning and archive layout for
// multi-GPU Starch.  No device code.
//
// The reference flushes one stream per chromosome segment (process_tf_buffer,
// include/starch3api.hpp:393-407) and segments are independent: a new one
// starts whenever the chr token differs from the current segment's name
// (hpp:325-342), and the transform state resets at every segment start
// (reset_transformation_state, hpp:523-536).  So the input can be cut at any
// line boundary where the chr token changes, and each piece ("unit") encoded
// on its own gives exactly the streams the whole input gives -- provided the
// piece starts with the sscanf values that were current before it: a start /
// stop that fails to parse keeps the previous line's value (hpp:306-307),
// also across segments.
//
// plan_units() finds such boundaries by galloping + bisection over line starts
// (O(log) probes per boundary, never a full scan), so units are the chromosome
// runs of a sorted BED; an unsorted input only makes some units span several
// segments, every unit boundary is still a segment boundary.  assign_lpt()
// balances units over shards; layout() puts the gathered segments back in
// input order.
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <thread>
#include <vector>

#include "shard.hpp"

namespace shard {
namespace {

constexpr int kProbes = 64;   // uniform probes after the gallop reaches the end

struct Tok {
    uint64_t off, len;   // chr token (C-string length: stops at the first NUL)
};

// start of the line containing byte p (p >= lo; lo is a line start)
uint64_t line_start(const uint8_t* b, uint64_t lo, uint64_t p)
{
    while (p > lo && b[p - 1] != '\n') --p;
    return p;
}

// start of the line after the one beginning at p (lim if it is the last)
uint64_t next_line(const uint8_t* b, uint64_t p, uint64_t lim)
{
    const void* nl = memchr(b + p, '\n', lim - p);
    return nl ? (uint64_t)(static_cast<const uint8_t*>(nl) - b) + 1 : lim;
}

// chr token of the line at ls: the bytes before the first tab; a line without
// a tab keeps its '\n' in the token (hpp:220-305)
Tok chr_tok(const uint8_t* b, uint64_t ls, uint64_t lim)
{
    uint64_t p = ls;
    while (p < lim && b[p] != '\t' && b[p] != '\n') ++p;
    uint64_t e = (p < lim && b[p] == '\n') ? p + 1 : p;
    const void* z = memchr(b + ls, 0, e - ls);
    return Tok{ls, z ? (uint64_t)(static_cast<const uint8_t*>(z) - (b + ls)) : e - ls};
}

bool same(const uint8_t* b, const Tok& a, const Tok& c)
{
    return a.len == c.len && memcmp(b + a.off, b + c.off, a.len) == 0;
}

bool is_c_space(uint8_t c) { return c == ' ' || c == '\t' || c == '\n' || c == '\v' || c == '\f' || c == '\r'; }

// sscanf("%" SCNd64) on s[0..len): 1 and *v on success, 0 (v untouched) on failure
int scan_i64(const uint8_t* s, uint64_t len, int64_t* v)
{
    uint64_t i = 0;
    while (i < len && is_c_space(s[i])) ++i;
    bool neg = false;
    if (i < len && (s[i] == '+' || s[i] == '-')) { neg = s[i] == '-'; ++i; }
    if (i >= len || s[i] < '0' || s[i] > '9') return 0;
    uint64_t acc = 0;
    bool over = false;
    const uint64_t lim = neg ? (uint64_t)INT64_MAX + 1u : (uint64_t)INT64_MAX;
    for (; i < len && s[i] >= '0' && s[i] <= '9'; ++i) {
        uint64_t d = (uint64_t)(s[i] - '0');
        if (!over && acc <= (lim - d) / 10u) acc = acc * 10u + d;
        else over = true;   // glibc clamps on overflow
    }
    if (over) acc = lim;
    *v = neg ? (int64_t)(0u - acc) : (int64_t)acc;
    return 1;
}

// the start / stop fields of the terminated line [ls, le) with the tokenizer's
// rules (hpp:220-305): a tab advances the token (first three only) and the
// byte after it is taken unconditionally; '\n' is stripped from stop / rem.
void parse_line(const uint8_t* b, uint64_t ls, uint64_t le, int64_t* start, bool* ok_start, int64_t* stop,
                bool* ok_stop)
{
    uint64_t fb[4] = {ls, le, le, le}, fe[4] = {le, le, le, le};
    int tok = 0;
    uint64_t p = ls;
    for (;;) {
        if (b[p] == '\t' && tok != 3) { fe[tok] = p; ++tok; ++p; fb[tok] = p; }
        ++p;
        if (b[p - 1] == '\n' || p >= le) break;
    }
    fe[tok] = p;
    if (tok == 2 || tok == 3) fe[tok] -= 1;
    auto clen = [&](int t) {
        uint64_t n = fe[t] > fb[t] ? fe[t] - fb[t] : 0;
        const void* z = n ? memchr(b + fb[t], 0, n) : nullptr;
        return z ? (uint64_t)(static_cast<const uint8_t*>(z) - (b + fb[t])) : n;
    };
    *ok_start = tok >= 1 && scan_i64(b + fb[1], clen(1), start);
    *ok_stop = tok >= 2 && scan_i64(b + fb[2], clen(2), stop);
}

}  // namespace

uint64_t input_limit(const uint8_t* b, uint64_t n)
{
    // 0xFF reads as EOF (hpp:181).  Large inputs: 16 threads scan a slice each
    // (one memchr stream runs at ~10 GB/s, and over a freshly mapped file it
    // also takes every page fault on one core)
    const int nt = n >= (64ull << 20) ? 16 : 1;
    if (nt == 1) {
        const void* ff = memchr(b, 0xFF, n);
        return ff ? (uint64_t)(static_cast<const uint8_t*>(ff) - b) : n;
    }
    const uint64_t per = (n + nt - 1) / nt;
    std::vector<uint64_t> at(nt, n);
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t)
        th.emplace_back([&, t]() {
            const uint64_t lo = std::min(n, (uint64_t)t * per), hi = std::min(n, lo + per);
            const void* ff = hi > lo ? memchr(b + lo, 0xFF, hi - lo) : nullptr;
            if (ff) at[t] = (uint64_t)(static_cast<const uint8_t*>(ff) - b);
        });
    for (auto& x : th) x.join();
    return *std::min_element(at.begin(), at.end());
}

void plan_units(const uint8_t* b, uint64_t n, uint64_t max_units, std::vector<Unit>& out, int64_t init_start0,
                int64_t init_stop0)
{
    plan_units_upto(b, input_limit(b, n), max_units, out, init_start0, init_stop0);
}

void plan_units_upto(const uint8_t* b, uint64_t lim, uint64_t max_units, std::vector<Unit>& out, int64_t init_start0,
                     int64_t init_stop0)
{
    out.clear();
    if (lim == 0) return;
    if (max_units < 1) max_units = 1;
    uint64_t s = 0;
    while (s < lim) {
        if (out.size() + 1 >= max_units) { out.push_back(Unit{s, lim - s, 0, 0}); break; }
        const Tok c0 = chr_tok(b, s, lim);
        uint64_t lo = s, hi = lim;
        bool found = false;
        // gallop: probe line starts at growing distances while the chr stays c0
        for (uint64_t step = 1u << 16;;) {
            const uint64_t p = lo + step;
            if (p >= lim) break;
            const uint64_t ls = line_start(b, lo, p);
            if (ls <= lo) { step *= 2; continue; }
            if (same(b, chr_tok(b, ls, lim), c0)) { lo = ls; step *= 2; }
            else { hi = ls; found = true; break; }
        }
        if (!found) {   // evenly spaced probes over the rest (revisited chromosomes), then its last line
            const uint64_t base = lo, span = lim - lo;
            for (int j = 1; j <= kProbes && !found; ++j) {
                const uint64_t p = j < kProbes ? base + span * (uint64_t)j / kProbes : lim - 1;
                const uint64_t ls = line_start(b, lo, p > lo ? p : lo);
                if (ls <= lo) continue;
                if (same(b, chr_tok(b, ls, lim), c0)) lo = ls;
                else { hi = ls; found = true; }
            }
        }
        if (found) {   // bisect to adjacent lines lo (chr c0) / hi (chr != c0)
            for (;;) {
                const uint64_t nx = next_line(b, lo, hi);
                if (nx >= hi) break;
                uint64_t ls = line_start(b, lo, lo + (hi - lo) / 2);
                if (ls <= lo) ls = nx;
                if (same(b, chr_tok(b, ls, lim), c0)) lo = ls;
                else hi = ls;
            }
        }
        out.push_back(Unit{s, hi - s, 0, 0});
        s = hi;
    }
    if (!out.empty()) { out[0].init_start = init_start0; out[0].init_stop = init_stop0; }
    // sscanf values current before each unit: those of the last line before it
    // whose field parses; scanning back stops at the previous unit's start
    // (older lines are summarised by that unit's own initial values)
    for (size_t k = 1; k < out.size(); ++k) {
        int64_t st = out[k - 1].init_start, sp = out[k - 1].init_stop;
        bool hs = false, hp = false;
        uint64_t le = out[k].offset;
        while (le > out[k - 1].offset && !(hs && hp)) {
            const uint64_t ls = line_start(b, out[k - 1].offset, le - 1);
            int64_t a = 0, c = 0;
            bool oa = false, oc = false;
            parse_line(b, ls, le, &a, &oa, &c, &oc);
            if (!hs && oa) { st = a; hs = true; }
            if (!hp && oc) { sp = c; hp = true; }
            le = ls;
        }
        out[k].init_start = st;
        out[k].init_stop = sp;
    }
}

void values_before(const uint8_t* b, uint64_t lo, uint64_t pos, int64_t* start, int64_t* stop)
{
    bool hs = false, hp = false;
    uint64_t le = pos;
    while (le > lo && !(hs && hp)) {
        const uint64_t ls = line_start(b, lo, le - 1);
        int64_t a = 0, c = 0;
        bool oa = false, oc = false;
        parse_line(b, ls, le, &a, &oa, &c, &oc);
        if (!hs && oa) { *start = a; hs = true; }
        if (!hp && oc) { *stop = c; hp = true; }
        le = ls;
    }
}

void assign_lpt(const std::vector<Unit>& units, int nshards, std::vector<int32_t>& shard_of)
{
    shard_of.assign(units.size(), 0);
    if (nshards <= 1) return;
    std::vector<size_t> order(units.size());
    for (size_t i = 0; i < order.size(); ++i) order[i] = i;
    std::stable_sort(order.begin(), order.end(),
                     [&](size_t a, size_t c) { return units[a].length > units[c].length; });
    std::vector<uint64_t> load(nshards, 0);
    for (size_t i : order) {
        int best = 0;
        for (int k = 1; k < nshards; ++k)
            if (load[k] < load[best]) best = k;
        shard_of[i] = best;
        load[best] += units[i].length;
    }
}

void layout(const uint64_t* unit_of, const uint64_t* bytes, uint64_t nseg, uint64_t base, std::vector<uint64_t>& order,
            std::vector<uint64_t>& offset, uint64_t* end)
{
    order.resize(nseg);
    for (uint64_t i = 0; i < nseg; ++i) order[i] = i;
    // a unit's segments are consecutive in its part and already in input order
    std::stable_sort(order.begin(), order.end(), [&](uint64_t a, uint64_t c) { return unit_of[a] < unit_of[c]; });
    offset.assign(nseg, 0);
    uint64_t pos = base;
    for (uint64_t k = 0; k < nseg; ++k) {
        offset[order[k]] = pos;
        pos += bytes[order[k]];
    }
    *end = pos;
}

}  // namespace shard
