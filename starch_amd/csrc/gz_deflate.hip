// starch_amd/csrc/gz_deflate.hip -- the gzip compression method (-g) on MI355X.
//
// The reference declares the method (starch3api.hpp:25, k_gzip; CLI -g at
// src/starch3.cpp:84,124) and exits with ENOSYS when it is selected
// (hpp:777-779), so there is no reference output to match: parity is
// unpinned, and correctness means every member inflates (RFC 1951/1952, any
// zlib) to exactly the segment's transformed text.  Each segment becomes one
// gzip member: a 10-byte header without timestamp (byte-stable archives),
// fixed-Huffman deflate blocks, CRC-32 and ISIZE.
//
// Shape (one 64-lane wave per 4 KiB sub-chunk of a segment's text, all
// sub-chunks of all segments at once):
//   k_gz_block   stage the sub-chunk in LDS; 64 positions per step: 4-byte
//                hash, the previous position with that hash (lanes of equal
//                hash paired by ballots, earlier steps through an LDS table:
//                the most recent occurrence, so matches are as near as
//                possible), match length by 4-byte compares in LDS; then a
//                scalar walk marks the greedy parse (literal, or the match
//                when it is >= 4 bytes) 64 positions at a time, a wave scan
//                places every token's fixed-Huffman bits, and LDS atomics
//                assemble the block (3-bit header .. end-of-block code); also
//                the sub-chunk's CRC-32 register (64-byte lane strips folded
//                by GF(2) multiplication with x^(8n) mod P).
//   k_gz_crc     per segment: fold its sub-chunk registers (workgroup tree).
//   k_gz_concat  every sub-chunk's bits into the member at its bit offset
//                (scan of block bit lengths); words shared by two blocks are
//                OR-ed (the output is zeroed first); header and trailer.
// A block is one deflate block (BFINAL on the segment's last), so blocks are
// bit-contiguous and need no alignment; matches never cross a sub-chunk.
#include "gz.hpp"
#include <atomic>

#include <algorithm>

namespace gz {
namespace {

struct EvTimer {                 // HIP-event stage timer (ms added to *out)
    hipEvent_t a = nullptr, b = nullptr;
    hipStream_t st;
    float* out;
    EvTimer(hipStream_t s, float* o) : st(s), out(o)
    {
        if (!out) return;
        HIP_CHECK(hipEventCreate(&a));
        HIP_CHECK(hipEventCreate(&b));
        HIP_CHECK(hipEventRecord(a, st));
    }
    void stop()
    {
        if (!out || !a) return;
        HIP_CHECK(hipEventRecord(b, st));
        HIP_CHECK(hipEventSynchronize(b));
        float ms = 0;
        HIP_CHECK(hipEventElapsedTime(&ms, a, b));
        *out += ms;
        (void)hipEventDestroy(a);
        (void)hipEventDestroy(b);
        a = b = nullptr;
    }
    ~EvTimer() { stop(); }
};

constexpr uint32_t SUB = 4096;                 // bytes per sub-chunk (one deflate block)
constexpr uint32_t HT = 4096;                  // hash table entries (12-bit hash)
constexpr uint32_t MAXW = (SUB * 9 + 3 + 7 + 31) / 32 + 2;   // bit-buffer words per block (all literals)
constexpr uint32_t MIN_MATCH = 4, MAX_MATCH = 258;

// ---- fixed Huffman tables (RFC 1951 3.2.6), codes bit-reversed for LSB-first packing
struct FixedTables {
    uint16_t lit_code[288];
    uint8_t lit_len[288];
    uint8_t dist_code[30];
    uint16_t len_base[29];
    uint8_t len_extra[29];
    uint16_t dist_base[30];
    uint8_t dist_extra[30];
    uint32_t x8pow[48];                        // x^(8 * 2^k) mod P (reflected CRC-32)
};
__constant__ FixedTables c_ft;
__constant__ uint32_t c_crc_tab[256];          // reflected CRC-32 (poly 0xEDB88320), byte at a time

uint32_t rev_bits(uint32_t v, int n)
{
    uint32_t r = 0;
    for (int i = 0; i < n; ++i) r |= ((v >> i) & 1u) << (n - 1 - i);
    return r;
}

// GF(2) product of two CRC-32 register values (reflected: bit 31 is x^0)
__host__ __device__ inline uint32_t gf_mul(uint32_t a, uint32_t b)
{
    uint32_t m = 1u << 31, p = 0;
    for (int i = 0; i < 32; ++i) {
        if (a & m) p ^= b;
        m >>= 1;
        b = (b & 1u) ? (b >> 1) ^ 0xEDB88320u : b >> 1;
    }
    return p;
}

__device__ __forceinline__ uint32_t x8n(uint64_t n)   // x^(8n) mod P
{
    uint32_t r = 1u << 31;                     // x^0
    for (int k = 0; n; ++k, n >>= 1)
        if (n & 1u) r = gf_mul(r, c_ft.x8pow[k]);
    return r;
}

// CRC register (init 0, no final xor) of A||B from those of A and B
__device__ __forceinline__ uint32_t crc_cat(uint32_t ra, uint32_t rb, uint64_t len_b)
{
    return gf_mul(ra, x8n(len_b)) ^ rb;
}

__device__ __forceinline__ uint32_t len_sym(uint32_t L)   // 3..258 -> index 0..28 of the length codes
{
    uint32_t lo = 0, hi = 28;
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (c_ft.len_base[mid] <= L) lo = mid; else hi = mid - 1;
    }
    return lo;
}
__device__ __forceinline__ uint32_t dist_sym(uint32_t d)   // 1..32768 -> 0..29
{
    uint32_t lo = 0, hi = 29;
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (c_ft.dist_base[mid] <= d) lo = mid; else hi = mid - 1;
    }
    return lo;
}

constexpr uint32_t NSYM = 286 + 30;            // literal/length + distance symbols

struct HuffScratch {
    uint16_t srt[320];                         // used symbols by (frequency, symbol)
    uint32_t wint[320];                        // internal node weights
    uint16_t pleaf[320], pint[320];            // parents (internal node index)
    uint16_t dep[320];                         // internal node depths
    uint32_t maxd;
};

// Huffman code lengths (<= maxlen) of symbols [base, base + n) from freq
// (scaled down and rebuilt while too long, as bzip2's BZ2_hbMakeCodeLengths
// does); a one-wave workgroup calls it with all lanes.  Used symbols are
// ranked by (frequency, symbol) in parallel, then lane 0 merges two queues
// (leaves in rank order, internal nodes in creation order).
__device__ void huff_lengths(uint32_t* freq, uint32_t base, uint32_t n, uint32_t maxlen, uint8_t* len, HuffScratch& h)
{
    const uint32_t lane = threadIdx.x & 63;
    for (;;) {
        uint32_t m = 0;
        for (uint32_t s = lane; s < n; s += 64) m += freq[base + s] ? 1u : 0u;
        m = wave_reduce_add(m);
        for (uint32_t s = lane; s < n; s += 64) {
            const uint32_t f = freq[base + s];
            len[base + s] = 0;
            if (!f) continue;
            uint32_t r = 0;
            for (uint32_t t = 0; t < n; ++t) {
                const uint32_t g = freq[base + t];
                r += (g && (g < f || (g == f && t < s))) ? 1u : 0u;
            }
            h.srt[r] = (uint16_t)s;
        }
        __syncthreads();
        if (lane == 0) {
            uint32_t il = 0, ii = 0, ni = 0, maxd = 0;
            auto pick = [&](uint32_t& w) -> int {   // >= 0: leaf rank; < 0: -(internal node + 1)
                if (il < m && (ii >= ni || freq[base + h.srt[il]] <= h.wint[ii])) {
                    w = freq[base + h.srt[il]];
                    return (int)il++;
                }
                w = h.wint[ii];
                return -(int)(++ii);
            };
            for (uint32_t q = 0; q + 1 < m; ++q) {
                uint32_t wa, wb;
                const int a = pick(wa), b = pick(wb);
                h.wint[ni] = wa + wb;
                if (a >= 0) h.pleaf[a] = (uint16_t)ni; else h.pint[-a - 1] = (uint16_t)ni;
                if (b >= 0) h.pleaf[b] = (uint16_t)ni; else h.pint[-b - 1] = (uint16_t)ni;
                ++ni;
            }
            if (m >= 2) {
                h.dep[ni - 1] = 0;
                for (int j = (int)ni - 2; j >= 0; --j) h.dep[j] = (uint16_t)(h.dep[h.pint[j]] + 1);
                for (uint32_t i = 0; i < m; ++i) {
                    const uint32_t d = h.dep[h.pleaf[i]] + 1u;
                    len[base + h.srt[i]] = (uint8_t)(d < 255 ? d : 255);
                    maxd = d > maxd ? d : maxd;
                }
            } else if (m == 1) {
                len[base + h.srt[0]] = 1;
                maxd = 1;
            }
            h.maxd = maxd;
        }
        __syncthreads();
        if (h.maxd <= maxlen) break;
        for (uint32_t s = lane; s < n; s += 64)
            if (freq[base + s]) freq[base + s] = 1 + freq[base + s] / 2;
        __syncthreads();
    }
}

struct SubDesc {                 // one sub-chunk = one deflate block
    uint64_t text_off;           // absolute text offset
    uint32_t len;                // bytes (0 only for an empty segment's single block)
    uint32_t seg;                // output member
    uint32_t final;              // BFINAL
    uint32_t pad;
};

__global__ void __launch_bounds__(64) k_gz_block(const uint8_t* __restrict__ text, const SubDesc* __restrict__ subs,
                                                 uint32_t nsub, uint32_t* __restrict__ bits_out,
                                                 uint32_t* __restrict__ nbits, uint32_t* __restrict__ crc_reg)
{
    __shared__ uint32_t tw[SUB / 4 + 72];      // the sub-chunk, zero padded (4-byte compares run past the end)
    __shared__ uint16_t ht[HT];                // last position + 1 per hash
    __shared__ uint16_t ml[SUB], md[SUB];      // match length / distance at each position
    __shared__ uint32_t bw[MAXW];              // the block's bits
    __shared__ uint32_t tokw[SUB / 32];        // token starts (greedy parse)
    __shared__ uint32_t hist[NSYM];            // literal/length 0..285, distance 286..315
    __shared__ uint32_t hf[NSYM + 24];         // frequencies fed to huff_lengths (+ 320..338: length codes)
    __shared__ uint8_t cl[NSYM + 24];          // code lengths
    __shared__ uint16_t cc[NSYM + 24];         // codes, bit-reversed
    __shared__ uint8_t rs[NSYM + 4], rx[NSYM + 4];   // run-length coded length sequence (symbol, extra)
    __shared__ uint32_t nrle_sh, ncl_sh;
    __shared__ HuffScratch hs;
    const uint32_t lane = threadIdx.x;
    const uint32_t k = blockIdx.x;
    if (k >= nsub) return;
    const SubDesc sd = subs[k];
    const uint32_t len = sd.len;
    const uint8_t* src = text + sd.text_off;
    uint8_t* tb = reinterpret_cast<uint8_t*>(tw);
    for (uint32_t i = lane; i < SUB / 4 + 72; i += 64) tw[i] = 0;
    for (uint32_t i = lane; i < HT; i += 64) ht[i] = 0;
    for (uint32_t i = lane; i < MAXW; i += 64) bw[i] = 0;
    __syncthreads();
    for (uint32_t i = lane; i < len; i += 64) tb[i] = src[i];
    __syncthreads();
    // CRC register of the lane's 64-byte strip, folded over the lanes in order
    uint32_t r = 0;
    const uint32_t sb = lane * 64u, se = sb + 64u < len ? sb + 64u : (sb < len ? len : sb);
    for (uint32_t i = sb; i < se; ++i) r = (r >> 8) ^ c_crc_tab[(r ^ tb[i]) & 0xffu];
    uint64_t slen = se - sb;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {          // combine with the strip d lanes before (lengths grow with d)
        const uint32_t ro = (uint32_t)__shfl_up((int)r, d, 64);
        const uint32_t lo = (uint32_t)__shfl_up((int)(uint32_t)slen, d, 64);
        if ((int)lane >= d && lane % (2 * d) == 2 * d - 1) {
            r = crc_cat(ro, r, slen);
            slen += lo;
        }
    }
    if (lane == 63) crc_reg[k] = r;
    // ---- matches: the previous position with the same 4 bytes ----
    for (uint32_t p0 = 0; p0 < len; p0 += 64) {
        const uint32_t p = p0 + lane;
        const bool hv = p + MIN_MATCH <= len;
        const uint32_t w = hv ? ((uint32_t)tb[p] | ((uint32_t)tb[p + 1] << 8) | ((uint32_t)tb[p + 2] << 16) |
                                 ((uint32_t)tb[p + 3] << 24))
                              : 0u;
        const uint32_t h = hv ? (w * 2654435761u) >> 20 : 0u;   // 12 bits
        uint64_t peers = __ballot(hv);
#pragma unroll
        for (int b = 0; b < 12; ++b) {
            const uint64_t m = __ballot((h >> b) & 1u);
            peers &= ((h >> b) & 1u) ? m : ~m;
        }
        const uint64_t below = peers & (lane ? (~0ull >> (64 - lane)) : 0ull);
        uint32_t prev = 0;                         // position + 1, 0: none
        if (hv) prev = below ? p0 + (63u - (uint32_t)__clzll((long long)below)) + 1u : ht[h];
        __builtin_amdgcn_wave_barrier();
        if (hv && (peers >> lane) == 1ull) ht[h] = (uint16_t)(p + 1);   // the highest lane of its hash
        uint32_t L = 0;
        if (prev) {
            const uint32_t j = prev - 1;
            const uint32_t lim = len - p < MAX_MATCH ? len - p : MAX_MATCH;
            while (L < lim) {                      // 4 bytes at a time (the tail is zero padded)
                const uint32_t a = (uint32_t)tb[j + L] | ((uint32_t)tb[j + L + 1] << 8) |
                                   ((uint32_t)tb[j + L + 2] << 16) | ((uint32_t)tb[j + L + 3] << 24);
                const uint32_t b = (uint32_t)tb[p + L] | ((uint32_t)tb[p + L + 1] << 8) |
                                   ((uint32_t)tb[p + L + 2] << 16) | ((uint32_t)tb[p + L + 3] << 24);
                const uint32_t x = a ^ b;
                if (x) { L += (uint32_t)__builtin_ctz(x) >> 3; break; }
                L += 4;
            }
            L = L < lim ? L : lim;
        }
        if (p < len) {
            ml[p] = (uint16_t)(L >= MIN_MATCH ? L : 0u);
            md[p] = (uint16_t)(prev ? p + 1 - prev : 0u);
        }
        __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();
    // ---- greedy parse, 64 positions per step: token starts and symbol counts ----
    for (uint32_t i = lane; i < NSYM; i += 64) hist[i] = 0;
    for (uint32_t i = lane; i < SUB / 32; i += 64) tokw[i] = 0;
    __syncthreads();
    uint32_t cur = 0, extra = 0;                  // first token start at or after p0; extra bits (lane sum)
    for (uint32_t p0 = 0; p0 < len; p0 += 64) {
        const uint32_t p = p0 + lane;
        const uint32_t L = p < len ? ml[p] : 0u;
        const uint32_t nx = p + (L ? L : 1u);       // next token start after a token at p
        uint64_t tok = 0;                          // scalar walk over this window's token starts
        while (cur < p0 + 64 && cur < len) {
            const uint32_t l = cur - p0;
            tok |= 1ull << l;
            cur = (uint32_t)__builtin_amdgcn_readlane((int)nx, (int)l);
        }
        if (lane < 2) tokw[(p0 >> 5) + lane] = (uint32_t)(tok >> (32 * lane));
        if ((tok >> lane) & 1ull) {
            if (L) {
                const uint32_t ls = len_sym(L), ds = dist_sym(md[p]);
                atomicAdd(&hist[257 + ls], 1u);
                atomicAdd(&hist[286 + ds], 1u);
                extra += c_ft.len_extra[ls] + c_ft.dist_extra[ds];
            } else {
                atomicAdd(&hist[tb[p]], 1u);
            }
        }
    }
    extra = wave_reduce_add(extra);
    if (lane == 0) hist[256] = 1;                 // end of block
    __syncthreads();
    // ---- codes: fixed (RFC 1951 3.2.6) or this block's own (3.2.7), whichever is shorter ----
    uint32_t fixed_bits = 0;
    for (uint32_t sy = lane; sy < NSYM; sy += 64)
        fixed_bits += hist[sy] * (sy < 286 ? (uint32_t)c_ft.lit_len[sy] : 5u);
    fixed_bits = 3 + wave_reduce_add(fixed_bits) + extra;
    for (uint32_t sy = lane; sy < NSYM; sy += 64) hf[sy] = hist[sy];
    if (lane == 0) {                               // complete trees: >= 2 used symbols each
        uint32_t nl = 0, nd = 0;
        for (uint32_t sy = 0; sy < 286; ++sy) nl += hf[sy] ? 1u : 0u;
        for (uint32_t sy = 286; sy < NSYM; ++sy) nd += hf[sy] ? 1u : 0u;
        for (uint32_t sy = 0; nl < 2 && sy < 286; ++sy) if (!hf[sy]) { hf[sy] = 1; ++nl; }
        for (uint32_t sy = 286; nd < 2 && sy < NSYM; ++sy) if (!hf[sy]) { hf[sy] = 1; ++nd; }
    }
    __syncthreads();
    huff_lengths(hf, 0, 286, 15, cl, hs);
    huff_lengths(hf, 286, 30, 15, cl, hs);
    __syncthreads();
    // lengths sent: literal/length codes up to the last used, distance codes likewise
    uint32_t nlit = 257, ndist = 1;
    for (uint32_t sy = lane; sy < 286; sy += 64) if (cl[sy]) nlit = sy + 1 > nlit ? sy + 1 : nlit;
    for (uint32_t sy = lane; sy < 30; sy += 64) if (cl[286 + sy]) ndist = sy + 1 > ndist ? sy + 1 : ndist;
    nlit = wave_reduce_max(nlit);
    ndist = wave_reduce_max(ndist);
    // run-length code of the length sequence (RFC 1951 3.2.7: 16 repeat previous, 17/18 zeros), by lane 0
    if (lane == 0) {
        for (uint32_t q = 0; q < 19; ++q) hf[320 + q] = 0;
        uint32_t nr = 0, i = 0, tot = nlit + ndist;
        auto at = [&](uint32_t q) -> uint32_t { return q < nlit ? cl[q] : cl[286 + q - nlit]; };
        while (i < tot) {
            const uint32_t v = at(i);
            uint32_t r = 1;
            while (i + r < tot && at(i + r) == v) ++r;
            uint32_t left = r;
            if (v == 0) {
                while (left >= 11) { const uint32_t c = left < 138 ? left : 138; rs[nr] = 18; rx[nr++] = (uint8_t)(c - 11); left -= c; }
                if (left >= 3) { rs[nr] = 17; rx[nr++] = (uint8_t)(left - 3); left = 0; }
            } else {
                rs[nr] = (uint8_t)v; rx[nr++] = 0; --left;
                while (left >= 3) { const uint32_t c = left < 6 ? left : 6; rs[nr] = 16; rx[nr++] = (uint8_t)(c - 3); left -= c; }
            }
            while (left) { rs[nr] = (uint8_t)v; rx[nr++] = 0; --left; }
            i += r;
        }
        for (uint32_t q = 0; q < nr; ++q) ++hf[320 + rs[q]];
        nrle_sh = nr;
        uint32_t u = 0;
        for (uint32_t q = 0; q < 19; ++q) u += hf[320 + q] ? 1u : 0u;
        for (uint32_t q = 0; u < 2 && q < 19; ++q) if (!hf[320 + q]) { hf[320 + q] = 1; ++u; }
    }
    __syncthreads();
    huff_lengths(hf, 320, 19, 7, cl, hs);
    __syncthreads();
    const bool dyn = [&] {
        static constexpr uint8_t ord[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
        uint32_t ncl = 19;
        while (ncl > 4 && cl[320 + ord[ncl - 1]] == 0) --ncl;
        uint32_t bits = 3 + 5 + 5 + 4 + 3 * ncl;
        const uint32_t nr = nrle_sh;
        for (uint32_t q = lane; q < nr; q += 64)
            bits += cl[320 + rs[q]] + (rs[q] == 16 ? 2u : rs[q] == 17 ? 3u : rs[q] == 18 ? 7u : 0u);
        uint32_t data = 0;
        for (uint32_t sy = lane; sy < NSYM; sy += 64) data += hist[sy] * cl[sy];
        bits = (uint32_t)wave_reduce_add(bits - (lane ? 3 + 5 + 5 + 4 + 3 * ncl : 0u)) + wave_reduce_add(data) + extra;
        if (lane == 0) ncl_sh = ncl;
        return bits < fixed_bits;
    }();
    __syncthreads();
    // canonical codes (bit-reversed for LSB-first packing): the block's, or the fixed ones
    if (lane == 0) {
        auto canon = [&](uint32_t base, uint32_t n) {
            uint32_t cnt[16] = {0}, next[16];
            for (uint32_t q = 0; q < n; ++q) ++cnt[cl[base + q]];
            cnt[0] = 0;
            uint32_t c = 0;
            for (int b = 1; b < 16; ++b) { c = (c + cnt[b - 1]) << 1; next[b] = c; }
            for (uint32_t q = 0; q < n; ++q) {
                const uint32_t l = cl[base + q];
                uint32_t v = l ? next[l]++ : 0u, r = 0;
                for (uint32_t b = 0; b < l; ++b) r |= ((v >> b) & 1u) << (l - 1 - b);
                cc[base + q] = (uint16_t)r;
            }
        };
        if (dyn) { canon(0, 286); canon(286, 30); canon(320, 19); }
        else {
            for (uint32_t q = 0; q < 286; ++q) { cl[q] = c_ft.lit_len[q]; cc[q] = c_ft.lit_code[q]; }
            for (uint32_t q = 0; q < 30; ++q) { cl[286 + q] = 5; cc[286 + q] = c_ft.dist_code[q]; }
        }
    }
    __syncthreads();
    // ---- header (lane 0, serial), then the tokens (wave scan), then end of block ----
    uint32_t bitpos = 0;
    if (lane == 0) {
        auto put = [&](uint32_t v, uint32_t n) {
            const uint64_t w = (uint64_t)v << (bitpos & 31u);
            bw[bitpos >> 5] |= (uint32_t)w;
            if (n + (bitpos & 31u) > 32) bw[(bitpos >> 5) + 1] |= (uint32_t)(w >> 32);
            bitpos += n;
        };
        put((sd.final ? 1u : 0u) | ((dyn ? 2u : 1u) << 1), 3);   // BFINAL, BTYPE
        if (dyn) {
            static constexpr uint8_t ord[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
            const uint32_t ncl = ncl_sh;
            put(nlit - 257, 5);
            put(ndist - 1, 5);
            put(ncl - 4, 4);
            for (uint32_t q = 0; q < ncl; ++q) put(cl[320 + ord[q]], 3);
            for (uint32_t q = 0; q < nrle_sh; ++q) {
                const uint32_t sy = rs[q];
                put(cc[320 + sy], cl[320 + sy]);
                if (sy == 16) put(rx[q], 2);
                else if (sy == 17) put(rx[q], 3);
                else if (sy == 18) put(rx[q], 7);
            }
        }
    }
    bitpos = (uint32_t)__builtin_amdgcn_readlane((int)bitpos, 0);
    __syncthreads();
    for (uint32_t p0 = 0; p0 < len; p0 += 64) {
        const uint32_t p = p0 + lane;
        const bool is_tok = p < len && ((tokw[p >> 5] >> (p & 31u)) & 1u);
        uint64_t v = 0;                            // up to 48 bits, LSB first
        uint32_t nb = 0;
        if (is_tok) {
            const uint32_t L = ml[p];
            if (L) {
                const uint32_t ls = len_sym(L), d = md[p], ds = dist_sym(d), lsym = 257 + ls;
                v = cc[lsym];
                nb = cl[lsym];
                v |= (uint64_t)(L - c_ft.len_base[ls]) << nb;
                nb += c_ft.len_extra[ls];
                v |= (uint64_t)cc[286 + ds] << nb;
                nb += cl[286 + ds];
                v |= (uint64_t)(d - c_ft.dist_base[ds]) << nb;
                nb += c_ft.dist_extra[ds];
            } else {
                const uint32_t c = tb[p];
                v = cc[c];
                nb = cl[c];
            }
        }
        const uint32_t incl = wave_incl_scan_add(nb);
        const uint32_t at = bitpos + incl - nb;
        if (nb) {
            const uint32_t sh = at & 31u;
            const uint64_t lo = v << sh, hi = sh ? v >> (64u - sh) : 0ull;
            atomicOr(&bw[at >> 5], (uint32_t)lo);
            if (nb + sh > 32) atomicOr(&bw[(at >> 5) + 1], (uint32_t)(lo >> 32));
            if (nb + sh > 64) atomicOr(&bw[(at >> 5) + 2], (uint32_t)hi);
        }
        bitpos += (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    }
    __syncthreads();
    if (lane == 0) {                               // end of block (code 256)
        const uint64_t w = (uint64_t)cc[256] << (bitpos & 31u);
        bw[bitpos >> 5] |= (uint32_t)w;
        if (cl[256] + (bitpos & 31u) > 32) bw[(bitpos >> 5) + 1] |= (uint32_t)(w >> 32);
    }
    bitpos += cl[256];                             // every lane
    if (lane == 0) nbits[k] = bitpos;
    __syncthreads();
    const uint32_t nw = (bitpos + 31) >> 5;
    uint32_t* dst = bits_out + (uint64_t)k * MAXW;
    for (uint32_t i = lane; i < nw; i += 64) dst[i] = bw[i];
}

// per member: fold its blocks' CRC registers (a workgroup: each thread folds a
// run of blocks, then a tree over threads); the gzip CRC-32 of n bytes is
// ~(R ^ 0xffffffff * x^(8n)) (init all ones, final xor)
__global__ void __launch_bounds__(256) k_gz_crc(const SubDesc* __restrict__ subs, const uint32_t* __restrict__ sub0,
                                                const uint32_t* __restrict__ crc_reg, const uint64_t* __restrict__ seg_len,
                                                uint32_t* __restrict__ crc_out)
{
    __shared__ uint32_t rs[256];
    __shared__ uint64_t ls[256];
    const uint32_t s = blockIdx.x, tid = threadIdx.x;
    const uint32_t a = sub0[s], e = sub0[s + 1], nb = e - a;
    const uint32_t per = (nb + 255) / 256, b0 = a + tid * per, b1 = b0 + per < e ? b0 + per : e;
    uint32_t r = 0;
    uint64_t l = 0;
    for (uint32_t b = b0; b < b1; ++b) {
        r = crc_cat(r, crc_reg[b], subs[b].len);
        l += subs[b].len;
    }
    rs[tid] = r;
    ls[tid] = l;
    __syncthreads();
    for (uint32_t d = 1; d < 256; d <<= 1) {
        if (tid % (2 * d) == 0 && tid + d < 256) {
            rs[tid] = crc_cat(rs[tid], rs[tid + d], ls[tid + d]);
            ls[tid] += ls[tid + d];
        }
        __syncthreads();
    }
    if (tid == 0) crc_out[s] = ~(rs[0] ^ gf_mul(0xFFFFFFFFu, x8n(seg_len[s])));
}

struct MemberOut {               // device copy of the member layout
    uint64_t out_off;            // absolute byte offset of the member
    uint64_t deflate_bits;
    uint64_t text_len;
};

// one workgroup per block: its words shifted into place; the shared words at
// both ends are OR-ed
__global__ void __launch_bounds__(256) k_gz_concat(const SubDesc* __restrict__ subs, uint32_t nsub,
                                                   const uint32_t* __restrict__ bits_in, const uint32_t* __restrict__ nbits,
                                                   const uint64_t* __restrict__ bitoff, uint32_t* __restrict__ out32)
{
    const uint32_t k = blockIdx.x;
    if (k >= nsub) return;
    const uint64_t at = bitoff[k];               // absolute bit offset in the output
    const uint32_t n = nbits[k], nw = (n + 31) >> 5, sh = (uint32_t)(at & 31u);
    const uint32_t* src = bits_in + (uint64_t)k * MAXW;
    uint32_t* dst = out32 + (at >> 5);
    const uint32_t nout = (sh + n + 31) >> 5;
    for (uint32_t i = threadIdx.x; i < nout; i += 256) {
        const uint32_t lo = i < nw ? src[i] : 0u, hi = (i >= 1 && i - 1 < nw) ? src[i - 1] : 0u;
        uint32_t v = sh ? ((lo << sh) | (hi >> (32u - sh))) : lo;
        // mask to the block's own bits (src words past n are zero already)
        if (i == 0 || i == nout - 1) atomicOr(dst + i, v);
        else dst[i] = v;
    }
}

// header (10 bytes) and trailer (CRC-32, ISIZE) of every member
__global__ void k_gz_frame(const MemberOut* __restrict__ mo, const uint32_t* __restrict__ crc, uint32_t nseg,
                           uint8_t* __restrict__ out)
{
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= nseg) return;
    uint8_t* m = out + mo[s].out_off;
    const uint8_t hdr[10] = {0x1f, 0x8b, 8, 0, 0, 0, 0, 0, 0, 0xff};   // deflate, no flags, no mtime, OS unknown
    for (int i = 0; i < 10; ++i) m[i] = hdr[i];
    uint8_t* t = m + 10 + (mo[s].deflate_bits + 7) / 8;
    const uint32_t c = crc[s], z = (uint32_t)mo[s].text_len;
    for (int i = 0; i < 4; ++i) { t[i] = (uint8_t)(c >> (8 * i)); t[4 + i] = (uint8_t)(z >> (8 * i)); }
}

void upload_tables()
{
    // __constant__ data is per device: upload once for every device used
    static std::atomic<uint64_t> done{0};
    int dev = 0;
    HIP_CHECK(hipGetDevice(&dev));
    const uint64_t bit = 1ull << (dev & 63);
    if (done.load() & bit) return;
    FixedTables ft{};
    for (uint32_t s = 0; s < 288; ++s) {
        uint32_t code, n;
        if (s < 144) { code = 0x30 + s; n = 8; }
        else if (s < 256) { code = 0x190 + (s - 144); n = 9; }
        else if (s < 280) { code = s - 256; n = 7; }
        else { code = 0xC0 + (s - 280); n = 8; }
        ft.lit_code[s] = (uint16_t)rev_bits(code, (int)n);
        ft.lit_len[s] = (uint8_t)n;
    }
    for (uint32_t d = 0; d < 30; ++d) ft.dist_code[d] = (uint8_t)rev_bits(d, 5);
    const uint16_t lb[29] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99, 115,
                             131, 163, 195, 227, 258};
    const uint8_t le[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
    const uint16_t db[30] = {1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769, 1025, 1537,
                             2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
    const uint8_t de[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
    std::copy(lb, lb + 29, ft.len_base);
    std::copy(le, le + 29, ft.len_extra);
    std::copy(db, db + 30, ft.dist_base);
    std::copy(de, de + 30, ft.dist_extra);
    // x^8 mod P, then squarings: x^(8 * 2^k)
    uint32_t x8 = 1u << 23;                      // reflected x^8
    for (int k = 0; k < 48; ++k) { ft.x8pow[k] = x8; x8 = gf_mul(x8, x8); }
    uint32_t tab[256];
    for (uint32_t i = 0; i < 256; ++i) {
        uint32_t c = i;
        for (int j = 0; j < 8; ++j) c = (c & 1u) ? (c >> 1) ^ 0xEDB88320u : c >> 1;
        tab[i] = c;
    }
    HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(c_ft), &ft, sizeof(ft)));
    HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(c_crc_tab), tab, sizeof(tab)));
    done.fetch_or(bit);
}

}  // namespace

void Encoder::plan(const uint8_t* d_text, const std::vector<bz::StreamIn>& streams, hipStream_t st,
                   std::vector<bz::StreamOut>& outs, bz::Stats* stats)
{
    upload_tables();
    nseg_ = (uint32_t)streams.size();
    outs.assign(nseg_, bz::StreamOut());
    std::vector<SubDesc> subs;
    std::vector<uint32_t> sub0(nseg_ + 1, 0);
    seg_len_.assign(nseg_, 0);
    for (uint32_t s = 0; s < nseg_; ++s) {
        if (streams[s].group != s) throw StarchError(-2, "gzip: one piece per stream");
        sub0[s] = (uint32_t)subs.size();
        const uint64_t n = streams[s].text_len;
        seg_len_[s] = n;
        const uint64_t nb = n ? (n + SUB - 1) / SUB : 1;
        for (uint64_t b = 0; b < nb; ++b) {
            SubDesc d{};
            d.text_off = streams[s].text_off + b * SUB;
            d.len = (uint32_t)std::min<uint64_t>(SUB, n - std::min<uint64_t>(n, b * SUB));
            d.seg = s;
            d.final = b + 1 == nb ? 1u : 0u;
            subs.push_back(d);
        }
    }
    sub0[nseg_] = (uint32_t)subs.size();
    nsub_ = (uint32_t)subs.size();
    sub0_ = sub0;
    outs_.assign(nseg_, bz::StreamOut());
    if (nseg_ == 0) return;
    EvTimer tb(st, stats ? &stats->bwt : nullptr);
    SubDesc* d_subs = b_subs.as<SubDesc>(nsub_);
    HIP_CHECK(hipMemcpyAsync(d_subs, subs.data(), nsub_ * sizeof(SubDesc), hipMemcpyHostToDevice, st));
    uint32_t* d_bits = b_bits.as<uint32_t>((uint64_t)nsub_ * MAXW);
    uint32_t* d_nbits = b_nbits.as<uint32_t>(nsub_);
    uint32_t* d_crc = b_crc.as<uint32_t>(nsub_ + nseg_);
    hipLaunchKernelGGL(k_gz_block, dim3(nsub_), dim3(64), 0, st, d_text, d_subs, nsub_, d_bits, d_nbits, d_crc);
    HIP_CHECK(hipGetLastError());
    uint32_t* d_sub0 = b_sub0.as<uint32_t>(nseg_ + 1);
    uint64_t* d_slen = b_slen.as<uint64_t>(nseg_);
    HIP_CHECK(hipMemcpyAsync(d_sub0, sub0.data(), (nseg_ + 1) * sizeof(uint32_t), hipMemcpyHostToDevice, st));
    HIP_CHECK(hipMemcpyAsync(d_slen, seg_len_.data(), nseg_ * sizeof(uint64_t), hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_gz_crc, dim3(nseg_), dim3(256), 0, st, d_subs, d_sub0, d_crc, d_slen, d_crc + nsub_);
    HIP_CHECK(hipGetLastError());
    nbits_.resize(nsub_);
    crc_.resize(nseg_);
    HIP_CHECK(hipMemcpyAsync(nbits_.data(), d_nbits, nsub_ * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipMemcpyAsync(crc_.data(), d_crc + nsub_, nseg_ * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    tb.stop();
    uint64_t off = 0;
    for (uint32_t s = 0; s < nseg_; ++s) {
        uint64_t bits = 0;
        for (uint32_t b = sub0[s]; b < sub0[s + 1]; ++b) bits += nbits_[b];
        outs[s].out_off = off;
        outs[s].bytes = 10 + (bits + 7) / 8 + 8;
        outs[s].first_block = sub0[s];
        outs[s].n_blocks = sub0[s + 1] - sub0[s];
        outs[s].combined_crc = crc_[s];
        off += outs[s].bytes;
    }
    outs_ = outs;
    if (stats) stats->n_blocks += nsub_;
}

void Encoder::emit(uint8_t* d_out, uint64_t out_cap, uint64_t out_base, std::vector<bz::StreamOut>& outs,
                   hipStream_t st, bz::Stats* stats)
{
    if (nseg_ == 0) return;
    EvTimer te(st, stats ? &stats->emit : nullptr);
    uint64_t total = 0;
    for (auto& o : outs) total = std::max(total, o.out_off + o.bytes);
    if (((uintptr_t)d_out & 3u) != 0) throw StarchError(-2, "output buffer must be 4-byte aligned");
    if (out_base + total + 4 > out_cap) throw StarchError(-3, "output buffer too small");
    HIP_CHECK(hipMemsetAsync(d_out + out_base, 0, total, st));
    std::vector<uint64_t> bitoff(nsub_);
    std::vector<MemberOut> mo(nseg_);
    for (uint32_t s = 0; s < nseg_; ++s) {
        uint64_t pos = (out_base + outs[s].out_off + 10) * 8;
        mo[s].out_off = out_base + outs[s].out_off;
        mo[s].text_len = seg_len_[s];
        const uint64_t p0 = pos;
        for (uint32_t b = sub0_[s]; b < sub0_[s + 1]; ++b) { bitoff[b] = pos; pos += nbits_[b]; }
        mo[s].deflate_bits = pos - p0;
    }
    uint64_t* d_off = b_off.as<uint64_t>(nsub_);
    MemberOut* d_mo = b_mo.as<MemberOut>(nseg_);
    HIP_CHECK(hipMemcpyAsync(d_off, bitoff.data(), nsub_ * sizeof(uint64_t), hipMemcpyHostToDevice, st));
    HIP_CHECK(hipMemcpyAsync(d_mo, mo.data(), nseg_ * sizeof(MemberOut), hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_gz_concat, dim3(nsub_), dim3(256), 0, st, static_cast<const SubDesc*>(b_subs.p), nsub_,
                       static_cast<const uint32_t*>(b_bits.p), static_cast<const uint32_t*>(b_nbits.p), d_off,
                       reinterpret_cast<uint32_t*>(d_out));
    hipLaunchKernelGGL(k_gz_frame, dim3((nseg_ + 63) / 64), dim3(64), 0, st, d_mo,
                       static_cast<const uint32_t*>(b_crc.p) + nsub_, nseg_, d_out);
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipStreamSynchronize(st));          // host vectors leave scope
    te.stop();
}

}  // namespace gz
