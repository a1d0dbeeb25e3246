// starch_amd/csrc/bz2_decode.hip -- bzip2 decompression on MI355X (SURVEY §8
// f2; restates bzip2-1.0.6's decoder, bz:decompress.c:106-646,
// bz:huffman.c:170-200, bz:bzlib.c:621-708, data-parallel across blocks).
//
// Blocks of a stream are bit-aligned and back to back, so they are found by
// scanning every bit offset for the 48-bit block / end-of-stream magics
// (k_dec_scan, as bzip2recover does); the host walks the hits stream by stream
// ("BZh<level>" header, blocks, end magic + combined CRC).  Then per block:
//   k_dec_block   one wave per block, lane 0 sequential: header (CRC,
//                 origPtr, symbol map, selectors, delta-coded code lengths),
//                 Huffman decode (a 10-bit lookup table per group, the
//                 limit/base/perm search of hbCreateDecodeTables beyond it),
//                 RUNA/RUNB and inverse MTF (a register nibble list for <= 16
//                 symbols, an LDS byte list above); writes the last column as
//                 symbol ranks and the rank counts.  The block's data must end
//                 exactly at the next magic (a false magic inside coded data
//                 is caught here).
//   k_dec_tt      one workgroup per block: tt[cftab[c] + stable rank] = i << 8
//                 (bz:decompress.c:625-633), stable ranks by wave ballots
//   k_dec_walk    one workgroup per block: the inverse BWT walk
//                 (tPos = tt[tPos]; byte = tPos & 0xff; tPos >>= 8) split at
//                 sampled nodes: every lane walks from a sample to the next
//                 one, lane 0 chains the segments, the lanes write their bytes
//   k_dec_unrle   undo RLE1 (bz:bzlib.c:621-708): lane 0 counts the output and
//                 checkpoints its state 64 times, then 64 lanes write
//   CRC           block CRCs of the output (bz2_rle.hip's k_crc_chunks) and
//                 the streams' combined CRCs, checked against the stored ones.
// Randomised blocks (bzip2 < 0.9.5) are rejected.
#include "bz2_int.hpp"
#include "bz2_decode.hpp"

#include <algorithm>
#include <string.h>

namespace bz {
namespace {

constexpr uint64_t kMagicBlk = 0x314159265359ull, kMagicEnd = 0x177245385090ull;
constexpr uint32_t kDecStride = 900064;        // per-block scratch (>= 100000 * 9)
constexpr int kMaxCode = 23;                   // BZ_MAX_CODE_LEN
constexpr int kFastBits = 10;

enum : int32_t {
    E_OK = 0, E_RAND = -1, E_MAP = -2, E_GROUPS = -3, E_SEL = -4, E_LEN = -5, E_CODE = -6, E_OVER = -7,
    E_ORIG = -8, E_BITS = -9, E_WALK = -10, E_CRC = -11
};

struct DecBlk {
    uint64_t bit_beg;       // first bit after the block magic
    uint64_t bit_end;       // bit position of the next magic
    uint64_t out_off;
    uint32_t level;
    uint32_t stored_crc;
    uint32_t orig_ptr;
    uint32_t nblock;
    uint32_t out_len;
    int32_t status;
};

// ---------------------------------------------------------------------------
// magic scan: thread t checks the 64 bit offsets of bytes 8t .. 8t+7
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_dec_scan(const uint8_t* __restrict__ in, uint64_t n,
                                                  uint64_t* __restrict__ hits, uint32_t cap, uint32_t* __restrict__ cnt)
{
    const uint64_t base = ((uint64_t)blockIdx.x * 256 + threadIdx.x) * 8;
    if (base >= n) return;
    uint64_t hi = 0, lo = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        hi = (hi << 8) | (base + k < n ? in[base + k] : 0u);
        lo = (lo << 8) | (base + 8 + k < n ? in[base + 8 + k] : 0u);
    }
    for (uint32_t b = 0; b < 64; ++b) {
        if (base * 8 + b + 48 > n * 8) break;
        const uint64_t w = (b ? (hi << b) | (lo >> (64 - b)) : hi) >> 16;
        const bool blk = w == kMagicBlk, end = w == kMagicEnd;
        if (blk || end) {
            const uint32_t i = atomicAdd(cnt, 1u);
            if (i < cap) hits[i] = ((base * 8 + b) << 1) | (end ? 1u : 0u);
        }
    }
}

// ---------------------------------------------------------------------------
// block decode (lane 0 of one wave per block)
// ---------------------------------------------------------------------------
struct BitReader {                 // MSB-first bits from big-endian words, 64 B read ahead
    const uint4* src;              // 16-byte aligned
    uint4 q0, q1, q2, q3;
    uint32_t qi;                   // next word of q0
    uint64_t bb;                   // bits left-aligned
    uint32_t bn;                   // valid bits in bb
    uint64_t pos;                  // bits consumed since the start word
    __device__ __forceinline__ void init(const uint8_t* in, uint64_t bit)
    {
        const uint64_t w16 = bit >> 7;             // 16-byte unit holding the bit
        src = reinterpret_cast<const uint4*>(in) + w16;
        q0 = src[0]; q1 = src[1]; q2 = src[2]; q3 = src[3];
        src += 4;
        qi = 0; bb = 0; bn = 0; pos = 0;
        refill();
        const uint32_t skip = (uint32_t)(bit & 127u);
        for (uint32_t s = skip; s > 0;) {          // skip to the bit (<= 127)
            const uint32_t k = s > 32u ? 32u : s;
            bb <<= k; bn -= k; s -= k;
            refill();
        }
        pos = 0;
    }
    __device__ __forceinline__ uint32_t word()
    {
        const uint32_t w = qi == 0 ? q0.x : qi == 1 ? q0.y : qi == 2 ? q0.z : q0.w;
        if (++qi == 4) { q0 = q1; q1 = q2; q2 = q3; q3 = *src++; qi = 0; }
        return __builtin_bswap32(w);
    }
    __device__ __forceinline__ void refill()
    {
        if (bn < 32) { bb |= (uint64_t)word() << (32 - bn); bn += 32; }
    }
    __device__ __forceinline__ uint32_t get(uint32_t k)   // 1 <= k <= 32
    {
        refill();
        const uint32_t v = (uint32_t)(bb >> (64 - k));
        bb <<= k; bn -= k; pos += k;
        return v;
    }
};

struct DecShared {
    uint8_t sel[kMaxSelectors];
    uint8_t len[6][258];
    uint8_t seq2u[256];
    uint8_t list[256];
    uint16_t perm[6][258];
    int32_t limit[6][kMaxCode + 1], base[6][kMaxCode + 1];
    uint16_t fast[6][1 << kFastBits];
    uint32_t cnt[256];
    int32_t minlen[6];
    uint32_t usefast[6];
};

__global__ void __launch_bounds__(64) k_dec_block(const uint8_t* __restrict__ in, DecBlk* __restrict__ blks,
                                                   uint8_t* __restrict__ ll_all, uint32_t* __restrict__ cnt_all,
                                                   uint8_t* __restrict__ seq_all)
{
    __shared__ DecShared S;
    const uint32_t lane = threadIdx.x;
    DecBlk* B = blks + blockIdx.x;
    for (int i = lane; i < 256; i += 64) S.cnt[i] = 0;
    for (int i = lane; i < 6 * 258; i += 64) (&S.perm[0][0])[i] = 0;
    for (int i = lane; i < 6 * (1 << kFastBits); i += 64) (&S.fast[0][0])[i] = 0;
    __syncthreads();
    if (lane != 0) return;
    uint8_t* ll = ll_all + (uint64_t)blockIdx.x * kDecStride;
    int32_t st = E_OK;
    BitReader br;
    br.init(in, B->bit_beg);
    const uint32_t crc = br.get(32);
    const uint32_t rnd = br.get(1);
    const uint32_t orig = br.get(24);
    uint32_t nin = 0, nblock = 0;
    if (rnd) { st = E_RAND; goto done; }
    {
        const uint32_t in16 = br.get(16);
        for (uint32_t i = 0; i < 16; ++i) {
            if (!((in16 >> (15 - i)) & 1u)) continue;
            const uint32_t bits = br.get(16);
            for (uint32_t j = 0; j < 16; ++j)
                if ((bits >> (15 - j)) & 1u) S.seq2u[nin++] = (uint8_t)(i * 16 + j);
        }
    }
    if (nin == 0) { st = E_MAP; goto done; }
    {
        const uint32_t alpha = nin + 2;
        const uint32_t ng = br.get(3);
        if (ng < 2 || ng > 6) { st = E_GROUPS; goto done; }
        uint32_t nsel = br.get(15);
        if (nsel < 1) { st = E_SEL; goto done; }
        uint32_t pos6 = 0x543210u;                 // selector MTF list, 4 bits per entry
        for (uint32_t i = 0; i < nsel; ++i) {
            uint32_t j = 0;
            while (br.get(1)) {
                ++j;
                if (j >= ng) { st = E_SEL; goto done; }
            }
            if (i < 18002) {                       // BZ_MAX_SELECTORS; extra selectors are read, not used (1.0.8)
                const uint32_t v = (pos6 >> (4 * j)) & 15u;
                const uint32_t m = (4 * j + 4 >= 32) ? ~0u : ((1u << (4 * j + 4)) - 1u);
                pos6 = (pos6 & ~m) | (((pos6 << 4) & m) | v);
                S.sel[i] = (uint8_t)v;
            }
        }
        if (nsel > 18002) nsel = 18002;
        for (uint32_t t = 0; t < ng; ++t) {
            int32_t curr = (int32_t)br.get(5);
            for (uint32_t i = 0; i < alpha; ++i) {
                for (;;) {
                    if (curr < 1 || curr > 20) { st = E_LEN; goto done; }
                    if (!br.get(1)) break;
                    if (!br.get(1)) ++curr; else --curr;
                }
                S.len[t][i] = (uint8_t)curr;
            }
        }
        // decode tables (bz:huffman.c:170-200) + a 10-bit lookup table
        for (uint32_t t = 0; t < ng; ++t) {
            int32_t mn = 32, mx = 0;
            uint32_t kraft = 0;
            for (uint32_t i = 0; i < alpha; ++i) {
                const int32_t L = S.len[t][i];
                mn = L < mn ? L : mn;
                mx = L > mx ? L : mx;
                kraft += 1u << (20 - L);
            }
            int32_t* limit = S.limit[t];
            int32_t* base = S.base[t];
            uint32_t pp = 0;
            for (int32_t i = mn; i <= mx; ++i)
                for (uint32_t j = 0; j < alpha; ++j)
                    if (S.len[t][j] == i) S.perm[t][pp++] = (uint16_t)j;
            for (int i = 0; i <= kMaxCode; ++i) base[i] = 0;
            for (uint32_t i = 0; i < alpha; ++i) base[S.len[t][i] + 1]++;
            for (int i = 1; i <= kMaxCode; ++i) base[i] += base[i - 1];
            for (int i = 0; i <= kMaxCode; ++i) limit[i] = 0;
            int32_t vec = 0;
            for (int32_t i = mn; i <= mx; ++i) {
                vec += (base[i + 1] - base[i]);
                limit[i] = vec - 1;
                vec <<= 1;
            }
            for (int32_t i = mn + 1; i <= mx; ++i) base[i] = ((limit[i - 1] + 1) << 1) - base[i];
            S.minlen[t] = mn;
            // lookup table: canonical codes in (length, symbol) order, shortest
            // first; only for prefix codes (Kraft sum <= 1), else the search alone
            S.usefast[t] = kraft <= (1u << 20) ? 1u : 0u;
            if (S.usefast[t]) {
                uint32_t code = 0;
                for (int32_t L = mn; L <= mx; ++L) {
                    for (uint32_t j = 0; j < alpha; ++j) {
                        if (S.len[t][j] != L) continue;
                        if (L <= kFastBits) {
                            const uint32_t a = code << (kFastBits - L), e = (code + 1) << (kFastBits - L);
                            for (uint32_t x = a; x < e && x < (1u << kFastBits); ++x)
                                if (!S.fast[t][x]) S.fast[t][x] = (uint16_t)(((uint32_t)L << 9) | j);
                        }
                        ++code;
                    }
                    code <<= 1;
                }
            }
        }
        // data: Huffman symbols, RUNA/RUNB, inverse MTF (bz:decompress.c:510-600)
        const uint32_t eob = nin + 1;
        const uint32_t nmax = 100000u * B->level;
        int32_t gno = -1;
        uint32_t gpos = 0, g = 0;
        const bool nib = nin <= 16;
        uint64_t L = 0xFEDCBA9876543210ull;
        if (!nib) for (int i = 0; i < 256; ++i) S.list[i] = (uint8_t)i;
        uint32_t pack = 0;
        uint32_t es = 0, N = 1;
        bool inrun = false;
        auto put = [&](uint32_t v) {
            pack |= v << (8 * (nblock & 3u));
            if ((nblock & 3u) == 3u) { *reinterpret_cast<uint32_t*>(ll + (nblock & ~3u)) = pack; pack = 0; }
            ++nblock;
        };
        for (;;) {
            if (gpos == 0) {
                ++gno;
                if ((uint32_t)gno >= nsel) { st = E_SEL; goto done; }
                gpos = 50;
                g = S.sel[gno];
            }
            --gpos;
            br.refill();
            uint32_t sym, zn;
            const uint32_t e = S.usefast[g] ? S.fast[g][br.bb >> (64 - kFastBits)] : 0u;
            if (e) {
                sym = e & 511u;
                zn = e >> 9;
            } else {
                zn = (uint32_t)S.minlen[g];
                uint32_t zvec = (uint32_t)(br.bb >> (64 - zn));
                while ((int32_t)zvec > S.limit[g][zn]) {
                    ++zn;
                    if (zn > 20) { st = E_CODE; goto done; }
                    zvec = (uint32_t)(br.bb >> (64 - zn));
                }
                const int32_t ix = (int32_t)zvec - S.base[g][zn];
                if (ix < 0 || ix >= 258) { st = E_CODE; goto done; }
                sym = S.perm[g][ix];
            }
            br.bb <<= zn; br.bn -= zn; br.pos += zn;
            if (sym <= 1) {                         // RUNA / RUNB
                if (!inrun) { inrun = true; es = 0; N = 1; }
                if (N >= 2u * 1024u * 1024u) { st = E_OVER; goto done; }
                es += (sym + 1) * N;
                N <<= 1;
                continue;
            }
            if (inrun) {                            // flush the run of the front symbol
                inrun = false;
                const uint32_t uc = nib ? (uint32_t)(L & 15u) : S.list[0];
                if (nblock + es > nmax) { st = E_OVER; goto done; }
                S.cnt[uc] += es;
                for (uint32_t k = 0; k < es; ++k) put(uc);
            }
            if (sym == eob) break;
            if (nblock >= nmax) { st = E_OVER; goto done; }
            const uint32_t nn = sym - 1;
            uint32_t uc;
            if (nib) {
                uc = (uint32_t)(L >> (4 * nn)) & 15u;
                const uint64_t m = nn >= 15 ? ~0ull : ((1ull << (4 * nn + 4)) - 1ull);
                L = (L & ~m) | (((L << 4) & m) | uc);
            } else {
                uc = S.list[nn];
                for (uint32_t k = nn; k > 0; --k) S.list[k] = S.list[k - 1];
                S.list[0] = (uint8_t)uc;
            }
            S.cnt[uc]++;
            put(uc);
        }
        if (nblock & 3u) *reinterpret_cast<uint32_t*>(ll + (nblock & ~3u)) = pack;
        // the block's bits end exactly where the next magic starts
        if (B->bit_beg + br.pos != B->bit_end) st = E_BITS;
        if (orig >= nblock) st = E_ORIG;
    }
done:
    B->stored_crc = crc;
    B->orig_ptr = orig;
    B->nblock = nblock;
    B->status = st;
    uint32_t* cnt = cnt_all + (uint64_t)blockIdx.x * 256;
    for (int i = 0; i < 256; ++i) cnt[i] = S.cnt[i];
    uint8_t* seq = seq_all + (uint64_t)blockIdx.x * 256;
    for (uint32_t i = 0; i < 256; ++i) seq[i] = i < nin ? S.seq2u[i] : 0;
}

// ---------------------------------------------------------------------------
// tt vector: tt[cftab[c] + (rank of i among earlier equal symbols)] = i << 8
// (bz:decompress.c:625-633; the low byte, ll[j], stays in ll)
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_dec_tt(const DecBlk* __restrict__ blks, const uint8_t* __restrict__ ll_all,
                                                const uint32_t* __restrict__ cnt_all, uint32_t* __restrict__ tt_all)
{
    __shared__ uint32_t base[256];
    __shared__ uint32_t wc[4][256];
    __shared__ uint32_t scan_sh[8];
    const DecBlk& B = blks[blockIdx.x];
    if (B.status != E_OK) return;
    const uint32_t n = B.nblock;
    const uint8_t* ll = ll_all + (uint64_t)blockIdx.x * kDecStride;
    uint32_t* tt = tt_all + (uint64_t)blockIdx.x * kDecStride;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t c0 = cnt_all[(uint64_t)blockIdx.x * 256 + tid];
    base[tid] = block_excl_scan_add<uint32_t>(c0, scan_sh, (uint32_t*)nullptr);
    for (int w = 0; w < 4; ++w) wc[w][tid] = 0;
    __syncthreads();
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    for (uint32_t i0 = 0; i0 < n; i0 += 256) {
        const uint32_t i = i0 + tid;
        const bool valid = i < n;
        const uint32_t c = valid ? ll[i] : 0u;
        uint64_t m = __ballot(valid);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const bool bit = (c >> b) & 1u;
            const uint64_t bal = __ballot(bit);
            m &= bit ? bal : ~bal;
        }
        const uint32_t rk = (uint32_t)__popcll(m & lt), cn = (uint32_t)__popcll(m);
        const bool leader = valid && rk == 0;
        if (leader) wc[wave][c] = cn;
        __syncthreads();
        uint32_t pos = 0;
        if (valid) {
            pos = base[c] + rk;
            for (int w = 0; w < wave; ++w) pos += wc[w][c];
        }
        __syncthreads();
        if (leader) { atomicAdd(&base[c], cn); wc[wave][c] = 0; }
        __syncthreads();
        if (valid) tt[pos] = i << 8;
    }
}

// ---------------------------------------------------------------------------
// inverse BWT walk, split at sampled nodes (one workgroup of 1024 per block)
// ---------------------------------------------------------------------------
constexpr int kWalkT = 1024;
__global__ void __launch_bounds__(kWalkT) k_dec_walk(DecBlk* __restrict__ blks, const uint32_t* __restrict__ tt_all,
                                                     const uint8_t* __restrict__ ll_all, const uint8_t* __restrict__ seq_all,
                                                     uint8_t* __restrict__ rle_all)
{
    __shared__ uint32_t slen[kWalkT], snx[kWalkT], soff[kWalkT];
    __shared__ uint8_t seq[256];
    __shared__ int32_t bad;
    __shared__ uint32_t cyc;
    DecBlk& B = blks[blockIdx.x];
    if (B.status != E_OK) return;
    const uint32_t n = B.nblock;
    const uint32_t* tt = tt_all + (uint64_t)blockIdx.x * kDecStride;
    const uint8_t* ll = ll_all + (uint64_t)blockIdx.x * kDecStride;
    uint8_t* out = rle_all + (uint64_t)blockIdx.x * kDecStride;
    const int tid = threadIdx.x;
    if (tid < 256) seq[tid] = seq_all[(uint64_t)blockIdx.x * 256 + tid];
    if (tid == 0) bad = 0;
    const uint32_t p0 = tt[B.orig_ptr] >> 8;
    uint32_t G = 1;
    while ((uint64_t)G * (kWalkT - 1) < n) G <<= 1;   // samples: nodes p with p % G == 0, and p0
    const uint32_t ns = (n + G - 1) / G;
    const bool extra = (p0 & (G - 1)) != 0;
    const uint32_t total = ns + (extra ? 1u : 0u);
    auto is_s = [&](uint32_t p) { return (p & (G - 1)) == 0 || p == p0; };
    auto idx = [&](uint32_t p) { return (p & (G - 1)) == 0 ? p / G : ns; };
    __syncthreads();
    if ((uint32_t)tid < total) {
        const uint32_t s = (uint32_t)tid < ns ? (uint32_t)tid * G : p0;
        uint32_t p = s, len = 0;
        do {
            p = tt[p] >> 8;
            ++len;
        } while (!is_s(p) && len <= n);
        if (len > n || p >= n) bad = 1;
        slen[tid] = len;
        snx[tid] = idx(p);
    }
    __syncthreads();
    // lane 0 chains the segments from p0's sample.  A periodic block's
    // permutation has several cycles of equal length C | n; bzip2 walks n steps
    // around p0's cycle (bz:decompress.c:635-642), so its bytes repeat n / C times
    if (tid == 0 && !bad) {
        for (uint32_t k = 0; k < total; ++k) soff[k] = 0xFFFFFFFFu;
        const uint32_t k0 = idx(p0);
        uint32_t k = k0, o = 0, steps = 0;
        do {
            soff[k] = o;
            o += slen[k];
            k = snx[k];
            if (k >= total || ++steps > total) { bad = 1; break; }
        } while (k != k0);
        if (!bad && (o == 0 || n % o != 0)) bad = 1;
        cyc = o;
    }
    __syncthreads();
    if (bad) {
        if (tid == 0) B.status = E_WALK;
        return;
    }
    if ((uint32_t)tid < total && soff[tid] != 0xFFFFFFFFu) {
        uint32_t p = (uint32_t)tid < ns ? (uint32_t)tid * G : p0;
        const uint32_t o = soff[tid], len = slen[tid];
        for (uint32_t j = 0; j < len; ++j) {
            out[o + j] = seq[ll[p]];
            p = tt[p] >> 8;
        }
    }
    const uint32_t C = cyc;
    if (C < n) {                                    // periodic: repeat the cycle's bytes
        __threadfence();
        __syncthreads();
        for (uint32_t j = C + tid; j < n; j += kWalkT) out[j] = out[j % C];
    }
}

// ---------------------------------------------------------------------------
// undo RLE1 (bz:bzlib.c:621-708): 4 equal bytes are followed by a count byte
// (0..251) of further copies.  Mode 0: lane 0 counts the block's output and
// checkpoints (input position, output offset, equal-run state) at 64 points;
// mode 1: lane l decodes from checkpoint l and writes.
// ---------------------------------------------------------------------------
struct UnrleCk { uint32_t in, out, run, last; };

__global__ void __launch_bounds__(64) k_dec_unrle(DecBlk* __restrict__ blks, const uint8_t* __restrict__ rle_all,
                                                   UnrleCk* __restrict__ cks, uint8_t* __restrict__ out, uint32_t mode)
{
    DecBlk& B = blks[blockIdx.x];
    if (B.status != E_OK) return;
    const uint32_t n = B.nblock, lane = threadIdx.x;
    const uint8_t* r = rle_all + (uint64_t)blockIdx.x * kDecStride;
    UnrleCk* ck = cks + (uint64_t)blockIdx.x * 64;
    if (mode == 0) {
        if (lane != 0) return;
        const uint32_t step = (n + 63) / 64;
        uint32_t o = 0, run = 0, last = 0, next_ck = 0, k = 0;
        const uint4* r4 = reinterpret_cast<const uint4*>(r);
        for (uint32_t i = 0; i < n; i += 16) {
            const uint4 v = r4[i >> 4];
            const uint32_t w[4] = {v.x, v.y, v.z, v.w};
            for (uint32_t j = 0; j < 16 && i + j < n; ++j) {
                if (i + j == next_ck) {
                    ck[k++] = UnrleCk{i + j, o, run, last};
                    next_ck += step;
                }
                const uint32_t c = (w[j >> 2] >> (8 * (j & 3))) & 0xffu;
                if (run == 4) { o += c; run = 0; continue; }        // count byte
                if (run && c == last) ++run; else { run = 1; last = c; }
                ++o;
            }
        }
        for (; k < 64; ++k) ck[k] = UnrleCk{n, o, run, last};
        B.out_len = o;
        return;
    }
    // mode 1: lane l decodes [ck[l].in, ck[l+1].in)
    const UnrleCk c0 = ck[lane];
    const uint32_t end = lane + 1 < 64 ? ck[lane + 1].in : n;
    uint8_t* dst = out + B.out_off;
    uint32_t o = c0.out, run = c0.run, last = c0.last;
    for (uint32_t i = c0.in; i < end; ++i) {
        const uint32_t c = r[i];
        if (run == 4) {
            for (uint32_t q = 0; q < c; ++q) dst[o + q] = (uint8_t)last;
            o += c;
            run = 0;
            continue;
        }
        if (run && c == last) ++run; else { run = 1; last = c; }
        dst[o++] = (uint8_t)c;
    }
}

__global__ void k_dec_crc_desc(const DecBlk* __restrict__ blks, uint32_t nb, BlockDesc* __restrict__ bd)
{
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nb) return;
    BlockDesc d{};
    d.in_beg = blks[b].out_off;
    d.in_end = blks[b].status == E_OK ? blks[b].out_off + blks[b].out_len : blks[b].out_off;
    bd[b] = d;
}

}  // namespace

// ---------------------------------------------------------------------------
// host driver
// ---------------------------------------------------------------------------
static inline uint32_t rotl1(uint32_t x) { return (x << 1) | (x >> 31); }

uint64_t Decoder::decode(const uint8_t* d_in, uint64_t n, const uint8_t* h_in, hipStream_t st, DevBuf& out,
                         std::vector<DecStream>& streams)
{
    upload_crc_constants();
    streams.clear();
    if (n == 0) return 0;
    auto fail = [](const std::string& m) -> void { throw StarchError(-12, "bzip2 decode: " + m); };
    // 1. magic hits
    const uint32_t cap = (uint32_t)std::min<uint64_t>(n / 8 + 1024, 1u << 26);
    uint64_t* d_hits = b_hits.as<uint64_t>(cap);
    uint32_t* d_cnt = b_cnt.as<uint32_t>(4);
    HIP_CHECK(hipMemsetAsync(d_cnt, 0, 4 * sizeof(uint32_t), st));
    hipLaunchKernelGGL(k_dec_scan, dim3((unsigned)ceil_div(ceil_div(n, 8), 256)), dim3(256), 0, st, d_in, n, d_hits,
                       cap, d_cnt);
    HIP_CHECK(hipGetLastError());
    uint32_t nh = 0;
    HIP_CHECK(hipMemcpyAsync(&nh, d_cnt, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    if (nh > cap) fail("too many magic candidates");
    std::vector<uint64_t> hits(nh);
    if (nh) HIP_CHECK(hipMemcpyAsync(hits.data(), d_hits, nh * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    std::sort(hits.begin(), hits.end());
    auto bytes_at = [&](uint64_t off, uint32_t len, uint8_t* dst) {
        const uint64_t m = off + len <= n ? len : (off < n ? n - off : 0);
        memset(dst, 0, len);
        if (!m) return;
        if (h_in) memcpy(dst, h_in + off, m);
        else {
            HIP_CHECK(hipMemcpyAsync(dst, d_in + off, m, hipMemcpyDeviceToHost, st));
            HIP_CHECK(hipStreamSynchronize(st));
        }
    };
    auto bits_at = [&](uint64_t bit, uint32_t k) -> uint32_t {   // k <= 32
        uint8_t b[8];
        bytes_at(bit >> 3, 8, b);
        uint64_t w = 0;
        for (int i = 0; i < 8; ++i) w = (w << 8) | b[i];
        return (uint32_t)((w << (bit & 7)) >> (64 - k));
    };
    // 2. walk streams: header, block hits, end hit + combined CRC
    std::vector<DecBlk> blk;
    size_t h = 0;
    uint64_t sb = 0;
    while (sb < n) {
        uint8_t hdr[4];
        bytes_at(sb, 4, hdr);
        if (hdr[0] != 'B' || hdr[1] != 'Z' || hdr[2] != 'h' || hdr[3] < '1' || hdr[3] > '9')
            fail("no stream header at byte " + std::to_string(sb));
        DecStream s{};
        s.in_beg = sb;
        s.level = (uint32_t)(hdr[3] - '0');
        s.n_blocks = 0;
        uint64_t expect = (sb + 4) * 8;
        while (h < nh && (hits[h] >> 1) < expect) ++h;   // hits inside an earlier stream's trailer/padding
        for (;;) {
            if (h >= nh || (hits[h] >> 1) != expect) fail("block / end-of-stream magic missing at bit " +
                                                          std::to_string(expect));
            const uint64_t pos = hits[h] >> 1;
            if (hits[h] & 1u) {                         // end of stream
                s.stored_crc = bits_at(pos + 48, 32);
                s.in_end = (pos + 48 + 32 + 7) / 8;
                ++h;
                break;
            }
            if (h + 1 >= nh) fail("stream ends without its trailer");
            DecBlk d{};
            d.bit_beg = pos + 48;
            d.bit_end = hits[h + 1] >> 1;
            d.level = s.level;
            blk.push_back(d);
            ++s.n_blocks;
            expect = d.bit_end;
            ++h;
        }
        streams.push_back(s);
        sb = s.in_end;
    }
    const uint32_t nb = (uint32_t)blk.size();
    uint64_t total = 0;
    if (nb) {
        // 3. per-block pipeline in batches (scratch 6 B + 256 B per block slot)
        const uint32_t batch = std::min<uint32_t>(nb, 2048);
        DecBlk* d_blk = b_blocks.as<DecBlk>(nb);
        HIP_CHECK(hipMemcpyAsync(d_blk, blk.data(), nb * sizeof(DecBlk), hipMemcpyHostToDevice, st));
        uint8_t* d_ll = b_ll.as<uint8_t>((uint64_t)batch * kDecStride + 64);
        uint32_t* d_tt = b_tt.as<uint32_t>((uint64_t)batch * kDecStride + 64);
        uint8_t* d_rle = b_rle.as<uint8_t>((uint64_t)nb * kDecStride + 64);
        uint32_t* d_cntb = b_meta.as<uint32_t>((uint64_t)nb * 256 * 2);
        uint8_t* d_seq = reinterpret_cast<uint8_t*>(d_cntb + (uint64_t)nb * 256);
        UnrleCk* d_ck = reinterpret_cast<UnrleCk*>(b_crc.as<uint8_t>((uint64_t)nb * 64 * sizeof(UnrleCk)));
        for (uint32_t b0 = 0; b0 < nb; b0 += batch) {
            const uint32_t cnt = std::min(batch, nb - b0);
            hipLaunchKernelGGL(k_dec_block, dim3(cnt), dim3(64), 0, st, d_in, d_blk + b0, d_ll, d_cntb + 256ull * b0,
                               d_seq + 256ull * b0);
            hipLaunchKernelGGL(k_dec_tt, dim3(cnt), dim3(256), 0, st, d_blk + b0, d_ll, d_cntb + 256ull * b0, d_tt);
            hipLaunchKernelGGL(k_dec_walk, dim3(cnt), dim3(kWalkT), 0, st, d_blk + b0, d_tt, d_ll, d_seq + 256ull * b0,
                               d_rle + (uint64_t)b0 * kDecStride);
            HIP_CHECK(hipGetLastError());
        }
        hipLaunchKernelGGL(k_dec_unrle, dim3(nb), dim3(64), 0, st, d_blk, d_rle, d_ck, nullptr, 0u);
        HIP_CHECK(hipGetLastError());
        HIP_CHECK(hipMemcpyAsync(blk.data(), d_blk, nb * sizeof(DecBlk), hipMemcpyDeviceToHost, st));
        HIP_CHECK(hipStreamSynchronize(st));
        static const char* what[] = {"ok", "randomised block (unsupported)", "empty symbol map", "bad group count",
                                     "bad selectors", "bad code lengths", "bad Huffman code", "block overrun",
                                     "origPtr out of range", "block data does not end at the next magic",
                                     "BWT permutation is not one cycle", "CRC mismatch"};
        for (uint32_t b = 0; b < nb; ++b) {
            if (blk[b].status != E_OK) fail(std::string("block ") + std::to_string(b) + ": " + what[-blk[b].status]);
            blk[b].out_off = total;
            total += blk[b].out_len;
        }
        HIP_CHECK(hipMemcpyAsync(d_blk, blk.data(), nb * sizeof(DecBlk), hipMemcpyHostToDevice, st));
        uint8_t* d_out = out.as<uint8_t>(total + 64);
        hipLaunchKernelGGL(k_dec_unrle, dim3(nb), dim3(64), 0, st, d_blk, d_rle, d_ck, d_out, 1u);
        // 4. block CRCs of the output
        BlockDesc* d_bd = b_bd.as<BlockDesc>(nb);
        hipLaunchKernelGGL(k_dec_crc_desc, dim3((nb + 255) / 256), dim3(256), 0, st, d_blk, nb, d_bd);
        rle_crc(d_out, d_bd, nb, nullptr, reinterpret_cast<uint32_t*>(d_tt), st);
        HIP_CHECK(hipGetLastError());
        std::vector<BlockDesc> bd(nb);
        HIP_CHECK(hipMemcpyAsync(bd.data(), d_bd, nb * sizeof(BlockDesc), hipMemcpyDeviceToHost, st));
        HIP_CHECK(hipStreamSynchronize(st));
        uint32_t b = 0;
        for (auto& s : streams) {
            s.out_off = s.n_blocks ? blk[b].out_off : total;
            s.combined_crc = 0;
            uint64_t len = 0;
            for (uint32_t k = 0; k < s.n_blocks; ++k, ++b) {
                if (bd[b].crc != blk[b].stored_crc)
                    fail("block " + std::to_string(b) + ": CRC mismatch");
                s.combined_crc = rotl1(s.combined_crc) ^ bd[b].crc;
                len += blk[b].out_len;
            }
            s.out_len = len;
            if (s.combined_crc != s.stored_crc) fail("stream combined CRC mismatch");
        }
    } else {
        for (auto& s : streams) {
            s.out_off = 0;
            s.out_len = 0;
            s.combined_crc = 0;
            if (s.stored_crc != 0) fail("stream combined CRC mismatch");
        }
        out.as<uint8_t>(64);
    }
    return total;
}

}  // namespace bz
