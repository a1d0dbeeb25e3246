// starch_amd/csrc/bz2_rle.hip -- RLE1, block cut and block CRC on MI355X.
//
// Restates bzip2-1.0.6's input side (bz:bzlib.c:224-338, 369-412) as
// data-parallel passes over 4 KiB tiles of a stream's bytes.  A byte's RLE1
// chunk position t = (position in its run) mod 255 decides its output: a
// chunk of L bytes emits min(L,4) copies + one count byte when L >= 4, so t < 3
// weighs 1, t == 3 weighs 2 (its copy + the count), t > 3 nothing.
//   1. k_rle_sum    per-tile run summary (first/last byte, uniform, trailing
//                   run, the leading run's length) and the RLE1 size of the
//                   bytes from the tile's first change on (their run positions
//                   are known inside the tile)
//   2. k_rle_carry  per-stream fold -> run position entering each tile, and
//                   the tile's RLE1 size (its leading run's weight in closed
//                   form from that position)
//   3. k_cut        per-stream greedy block cut over the RLE1 size prefix:
//                   chunk k joins the block iff the block holds < nblockMAX
//                   bytes before it (bz:bzlib.c:307,399-402); the final chunk
//                   joins a full block only when it is a single byte supplied
//                   with the finishing call (bz:bzlib.c:393-397)
//   4. k_rle_emit   materialise each block's RLE1 bytes + inUse map
//   5. k_crc_chunks + k_crc_final
//                   CRC-32/BZIP2 of each block's input bytes: slice-by-4 CRC of
//                   16-byte strips, GF(2) combine of strips -> chunks -> block
// The per-byte chunk positions are never stored: k_cut (one tile per block)
// and k_rle_emit recompute them from the text and the tile's entering run
// position.  Every lane handles one 16-byte strip, loaded with one or two
// aligned 16-B loads (any text alignment).
#include "bz2_int.hpp"
#include <atomic>
#include <string.h>

namespace bz {

__constant__ uint32_t c_pow8[64];   // x^(8*2^k) mod P, P = 0x04c11db7 (MSB-first)
__constant__ uint32_t c_crc_tab[256];
__constant__ uint32_t c_crc_tab4[4][256];   // [k][i]: register after byte i then k zero bytes
__constant__ uint32_t c_lane[64];           // x^(8*128*(63-i)): lane i's line shifted to the end of its 8 KB span

void upload_crc_constants()
{
    // __constant__ data is per device: upload once for every device used
    static std::atomic<uint64_t> done{0};
    int dev = 0;
    HIP_CHECK(hipGetDevice(&dev));
    const uint64_t bit = 1ull << (dev & 63);
    if (done.load() & bit) return;
    uint32_t tab[256];
    for (uint32_t b = 0; b < 256; ++b) {
        uint32_t c = b << 24;
        for (int k = 0; k < 8; ++k) c = (c & 0x80000000u) ? (c << 1) ^ 0x04c11db7u : (c << 1);
        tab[b] = c;
    }
    uint32_t pw[64];
    pw[0] = 0x100u;   // x^8
    for (int k = 1; k < 64; ++k) pw[k] = host_mulmod(pw[k - 1], pw[k - 1]);
    HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(c_pow8), pw, sizeof(pw)));
    HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(c_crc_tab), tab, sizeof(tab)));
    uint32_t tab4[4][256];
    for (uint32_t i = 0; i < 256; ++i) {
        uint32_t r = tab[i];
        tab4[0][i] = r;
        for (int k = 1; k < 4; ++k) { r = (r << 8) ^ tab[r >> 24]; tab4[k][i] = r; }
    }
    HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(c_crc_tab4), tab4, sizeof(tab4)));
    uint32_t cl[64];
    cl[63] = 1u;                                  // x^0
    for (int i = 62; i >= 0; --i) cl[i] = host_mulmod(cl[i + 1], pw[7]);   // pw[7] = x^(8*128)
    HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(c_lane), cl, sizeof(cl)));
    done.fetch_or(bit);
}

__device__ __forceinline__ uint32_t mulmod(uint32_t a, uint32_t b)
{
    uint32_t r = 0;
#pragma unroll 8
    for (int i = 31; i >= 0; --i) {
        r = (r & 0x80000000u) ? ((r << 1) ^ 0x04c11db7u) : (r << 1);
        if ((b >> i) & 1u) r ^= a;
    }
    return r;
}

// x^(8*len) mod P
__device__ __forceinline__ uint32_t xpow8(uint64_t len)
{
    uint32_t r = 0x1u;  // x^0
    int k = 0;
    while (len) {
        if (len & 1u) r = mulmod(r, c_pow8[k]);
        len >>= 1;
        ++k;
    }
    return r;
}

// ---------------------------------------------------------------------------
__global__ void k_tiles(const uint64_t* __restrict__ seg_tile0, const StreamIn* __restrict__ streams,
                        uint32_t nstreams, uint64_t ntiles, TileDesc* __restrict__ tiles)
{
    uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ntiles) return;
    uint32_t lo = 0, hi = nstreams;            // last s with seg_tile0[s] <= t
    while (hi - lo > 1) {
        uint32_t mid = (lo + hi) >> 1;
        if (seg_tile0[mid] <= t) lo = mid; else hi = mid;
    }
    uint32_t s = lo;
    while (s + 1 < nstreams && seg_tile0[s + 1] <= t) ++s;   // skip empty streams
    uint64_t k = t - seg_tile0[s];
    TileDesc d;
    d.beg = streams[s].text_off + k * kTB;
    uint64_t end = streams[s].text_off + streams[s].text_len;
    d.len = (uint32_t)((end - d.beg) < (uint64_t)kTB ? (end - d.beg) : (uint64_t)kTB);
    d.stream = s;
    d.first = (k == 0);
    tiles[t] = d;
}

// 16 bytes at p (any alignment): one aligned 16-B load, plus the next one only
// when it holds needed bytes below `lim` (so nothing past the data is touched).
__device__ __forceinline__ uint4 load16u(const uint8_t* p, const uint8_t* lim)
{
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    const uint4* q = reinterpret_cast<const uint4*>(a & ~(uintptr_t)15);
    const uint32_t sh = (uint32_t)(a & 15u);
    const uint4 x = q[0];
    if (sh == 0) return x;
    const uint4 y = (reinterpret_cast<const uint8_t*>(q + 1) < lim) ? q[1] : make_uint4(0, 0, 0, 0);
    const uint32_t w0 = x.x, w1 = x.y, w2 = x.z, w3 = x.w, w4 = y.x, w5 = y.y, w6 = y.z, w7 = y.w;
    const uint32_t bi = sh & 3u;
    uint32_t a0, a1, a2, a3, a4;
    switch (sh >> 2) {
    case 0: a0 = w0; a1 = w1; a2 = w2; a3 = w3; a4 = w4; break;
    case 1: a0 = w1; a1 = w2; a2 = w3; a3 = w4; a4 = w5; break;
    case 2: a0 = w2; a1 = w3; a2 = w4; a3 = w5; a4 = w6; break;
    default: a0 = w3; a1 = w4; a2 = w5; a3 = w6; a4 = w7; break;
    }
    return make_uint4(__builtin_amdgcn_alignbyte(a1, a0, bi), __builtin_amdgcn_alignbyte(a2, a1, bi),
                      __builtin_amdgcn_alignbyte(a3, a2, bi), __builtin_amdgcn_alignbyte(a4, a3, bi));
}

__device__ __forceinline__ uint32_t byte16(const uint4& v, int k)
{
    const uint32_t w = k < 4 ? v.x : k < 8 ? v.y : k < 12 ? v.z : v.w;
    return (w >> (8 * (k & 3))) & 0xffu;
}

// Runs inside a tile are located by their change positions: byte y > 0 of a
// tile starts a new run iff it differs from byte y - 1.  A lane holds one
// 16-byte strip; chg_mask marks its changed bytes (the byte before the strip
// comes from the previous strip's last byte; the tile's first byte is never a
// change) and the last change at or before a byte, a prefix maximum, gives
// every run length -- one integer max-scan instead of a scan of run summaries.
__device__ __forceinline__ uint32_t nonzero_bytes(uint32_t x)   // 0x80 in each nonzero byte (exact)
{
    return (((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x) & 0x80808080u;
}

// per-word masks of changed bytes among the strip's first cnt bytes
__device__ __forceinline__ void chg_mask(const uint4& v, uint32_t pb, int cnt, uint32_t (&m)[4])
{
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    uint32_t carry = pb;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t sh = (w[i] << 8) | carry;          // byte k of sh = byte k - 1 of the strip
        carry = w[i] >> 24;
        const int lim = cnt - 4 * i;                      // valid bytes of this word
        const uint32_t keep = lim >= 4 ? 0x80808080u : (lim <= 0 ? 0u : (0x80808080u >> (8 * (4 - lim))));
        m[i] = nonzero_bytes(w[i] ^ sh) & keep;
    }
}

// index (0..15) of the strip's last changed byte, or -1
__device__ __forceinline__ int last_change(const uint32_t (&m)[4])
{
    return m[3] ? 12 + ((31 - __clz((int)m[3])) >> 3)
         : m[2] ? 8 + ((31 - __clz((int)m[2])) >> 3)
         : m[1] ? 4 + ((31 - __clz((int)m[1])) >> 3)
         : m[0] ? ((31 - __clz((int)m[0])) >> 3) : -1;
}

// the strip of this lane and the byte before it (the strip's own first byte
// at the tile start, so that position 0 is never a change)
__device__ __forceinline__ void load_strip(const uint8_t* text, const TileDesc& d, int off, int cnt, uint4& v,
                                           uint32_t& pb)
{
    v = cnt > 0 ? load16u(text + d.beg + off, text + d.beg + d.len) : make_uint4(0, 0, 0, 0);
    pb = off > 0 && cnt > 0 ? (uint32_t)text[d.beg + off - 1] : (v.x & 0xffu);
}

__device__ __forceinline__ int first_change(const uint32_t (&m)[4])   // index (0..15) of the first changed byte, or -1
{
    return m[0] ? ((__builtin_ctz(m[0]) - 7) >> 3)
         : m[1] ? 4 + ((__builtin_ctz(m[1]) - 7) >> 3)
         : m[2] ? 8 + ((__builtin_ctz(m[2]) - 7) >> 3)
         : m[3] ? 12 + ((__builtin_ctz(m[3]) - 7) >> 3) : -1;
}

__device__ __forceinline__ uint32_t rle_w(uint32_t t) { return t < 3 ? 1u : (t == 3 ? 2u : 0u); }

// Chunk positions t of a lane's strip (bytes off .. off + cnt - 1 of a tile),
// packed 4 per word into tw; returns the strip's RLE1 weight.  ex = the
// tile's last change before the strip + 1 (0: none); the bytes before the
// tile's first change continue the run entering the tile at position c
// (KNOWN), or (!KNOWN) are left out of the weight.  One modulo per strip,
// then t steps by one (wrapping at 255) or restarts at a change.
template <bool KNOWN>
__device__ __forceinline__ uint32_t strip_t(const uint32_t (&m)[4], uint32_t off, int cnt, uint32_t ex, uint32_t c,
                                            uint32_t (&tw)[4])
{
    uint32_t tp = ex ? (off - ex) % 255u : (KNOWN ? (c + off + 254u) % 255u : 0u);   // t of byte off - 1
    bool lead = ex == 0;
    uint32_t w = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) tw[q] = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        if (k < cnt) {
            const bool chg = ((m[k >> 2] >> (8 * (k & 3) + 7)) & 1u) != 0;
            lead = lead && !chg;
            const uint32_t t = chg ? 0u : (tp == 254u ? 0u : tp + 1u);
            tw[k >> 2] |= t << (8 * (k & 3));
            if (KNOWN || !lead) w += rle_w(t);
            tp = t;
        }
    }
    return w;
}

// the tile's last change before this lane's strip + 1 (0: none), from every
// lane's last change (x = position + 1, 0: none); msh: 4 words of LDS.  Ends
// with a barrier.
__device__ __forceinline__ uint32_t tile_ex(uint32_t x, uint32_t* msh)
{
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint32_t incl = wave_incl_scan_max<uint32_t>(x);
    uint32_t ex = (uint32_t)__shfl_up((int)incl, 1, 64);
    if (lane == 0) ex = 0;
    if (lane == 63) msh[wid] = incl;
    __syncthreads();
    for (int w = 0; w < wid; ++w) ex = msh[w] > ex ? msh[w] : ex;
    return ex;
}

// One wave per tile, 64 bytes per lane: the lane's change masks, the tile's
// last change before the lane (a wave max-scan), its first change (the
// leading run) and the chunk positions of the bytes from the first change on
// -- wave scans only, no workgroup barriers.
constexpr int SUM_WPG = 4;                       // tiles (waves) per workgroup

__global__ void __launch_bounds__(64 * SUM_WPG) k_rle_sum(const uint8_t* __restrict__ text,
                                                         const TileDesc* __restrict__ tiles, uint64_t ntiles,
                                                         TileSum* __restrict__ sums)
{
    const uint64_t tile = (uint64_t)blockIdx.x * SUM_WPG + (threadIdx.x >> 6);
    if (tile >= ntiles) return;                  // wave-uniform
    const int lane = threadIdx.x & 63;
    const TileDesc d = tiles[tile];
    const uint32_t a = 64u * (uint32_t)lane;     // the lane's first byte, tile offset
    const int cnt = d.len > a ? (d.len - a < 64u ? (int)(d.len - a) : 64) : 0;
    uint32_t w[16];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t p = a + 16u * i;
        const uint4 v = p < d.len ? load16u(text + d.beg + p, text + d.beg + d.len) : make_uint4(0, 0, 0, 0);
        w[4 * i] = v.x; w[4 * i + 1] = v.y; w[4 * i + 2] = v.z; w[4 * i + 3] = v.w;
    }
    uint32_t carry = (uint32_t)__shfl_up((int)(w[15] >> 24), 1, 64);
    if (lane == 0) carry = w[0] & 0xffu;         // the tile's first byte is never a change
    uint32_t m[16];
    int lc = -1, fc = -1;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const uint32_t sh = (w[i] << 8) | carry;
        carry = w[i] >> 24;
        const int lim = cnt - 4 * i;
        const uint32_t keep = lim >= 4 ? 0x80808080u : (lim <= 0 ? 0u : (0x80808080u >> (8 * (4 - lim))));
        m[i] = nonzero_bytes(w[i] ^ sh) & keep;
    }
#pragma unroll
    for (int i = 15; i >= 0; --i)
        if (lc < 0 && m[i]) lc = 4 * i + ((31 - __clz((int)m[i])) >> 3);
#pragma unroll
    for (int i = 0; i < 16; ++i)
        if (fc < 0 && m[i]) fc = 4 * i + ((__builtin_ctz(m[i]) - 7) >> 3);
    const uint32_t incl = wave_incl_scan_max<uint32_t>(lc >= 0 ? a + (uint32_t)lc + 1u : 0u);
    uint32_t ex = (uint32_t)__shfl_up((int)incl, 1, 64);
    if (lane == 0) ex = 0;
    const uint32_t plast = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);   // last change + 1 (0: none)
    const uint32_t finv = wave_incl_scan_max<uint32_t>(fc >= 0 ? ~(a + (uint32_t)fc) : 0u);
    const uint32_t ffirst = ~(uint32_t)__builtin_amdgcn_readlane((int)finv, 63);  // first change (~0: none)
    // chunk positions of the bytes from the tile's first change on, and their weight
    uint32_t tp = ex ? (a - ex) % 255u : 0u;     // t of the byte before the lane's first
    bool lead = ex == 0;
    uint32_t wt = 0;
#pragma unroll
    for (int k = 0; k < 64; ++k) {
        if (k < cnt) {
            const bool chg = ((m[k >> 2] >> (8 * (k & 3) + 7)) & 1u) != 0;
            lead = lead && !chg;
            const uint32_t t = chg ? 0u : (tp == 254u ? 0u : tp + 1u);
            if (!lead) wt += rle_w(t);
            tp = t;
        }
    }
    const uint32_t wsum = (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan_add<uint32_t>(wt), 63);
    if (lane == 0) {
        TileSum o;
        o.len = d.len;
        o.first = d.len ? (uint8_t)(w[0] & 0xffu) : (uint8_t)0xff;
        o.last = d.len ? text[d.beg + d.len - 1] : (uint8_t)0xff;
        o.uni = plast == 0 ? 1 : 0;
        o.trail = plast == 0 ? d.len : d.len - (plast - 1);
        o.pad = 0;
        o.lead = ffirst == 0xFFFFFFFFu ? d.len : ffirst;
        o.wrest = wsum;
        sums[tile] = o;
    }
}

// RLE1 size of a run's L bytes starting at chunk position c: how many of
// them sit at positions 0, 1, 2 (weight 1) and 3 (weight 2) mod 255
__device__ __forceinline__ uint32_t lead_w(uint32_t c, uint32_t L)
{
    const uint32_t q = L / 255u, r = L % 255u;
    uint32_t w = 5u * q;
#pragma unroll
    for (uint32_t v = 0; v < 4; ++v) {
        const uint32_t dv = (v + 255u - c) % 255u;   // offset of the first byte at position v
        if (dv < r) w += v == 3 ? 2u : 1u;
    }
    return w;
}

// one 256-thread workgroup per stream: run length entering each tile, via an
// inclusive scan of tile run summaries (the run-summary combine is associative)
struct RunSum64 {
    uint64_t len, trail;
    int first, last, uni, pad;
};
__device__ __forceinline__ RunSum64 rs64_combine(const RunSum64& A, const RunSum64& B)
{
    if (A.len == 0) return B;
    if (B.len == 0) return A;
    RunSum64 R;
    R.first = A.first;
    R.last = B.last;
    R.len = A.len + B.len;
    R.uni = A.uni && B.uni && A.last == B.first;
    R.trail = (B.uni && B.first == A.last) ? B.len + A.trail : B.trail;
    R.pad = 0;
    return R;
}

// one 1024-thread workgroup per stream: each thread folds a run of tiles,
// one workgroup scan of the run summaries, then each thread re-walks its run
// (the run-summary combine is associative) -- two passes over the tile
// summaries instead of a barrier-bound scan per 256 tiles
constexpr int CT = 1024;
__global__ void __launch_bounds__(CT) k_rle_carry(const uint64_t* __restrict__ seg_tile0, uint32_t nstreams,
                                                   const TileSum* __restrict__ sums, uint32_t* __restrict__ carry,
                                                   uint32_t* __restrict__ tile_w)
{
    __shared__ RunSum64 sh[CT];
    const uint32_t s = blockIdx.x;
    const int tid = threadIdx.x;
    const uint64_t t0 = seg_tile0[s], t1 = seg_tile0[s + 1];
    const uint64_t per = (t1 - t0 + CT - 1) / CT;
    const uint64_t a = t0 + (uint64_t)tid * per, e = a + per < t1 ? a + per : t1;
    auto load = [&](uint64_t t) {
        const TileSum x = sums[t];
        RunSum64 S;
        S.len = x.len; S.trail = x.trail; S.first = x.first; S.last = x.last; S.uni = x.uni; S.pad = 0;
        return S;
    };
    RunSum64 agg;
    agg.len = 0; agg.trail = 0; agg.first = agg.last = -1; agg.uni = 1; agg.pad = 0;
    for (uint64_t t = a; t < e; ++t) agg = rs64_combine(agg, load(t));
    sh[tid] = agg;
    __syncthreads();
    for (int d = 1; d < CT; d <<= 1) {                  // inclusive scan of the run folds
        const RunSum64 v = (tid >= d) ? rs64_combine(sh[tid - d], sh[tid]) : sh[tid];
        __syncthreads();
        sh[tid] = v;
        __syncthreads();
    }
    RunSum64 P;
    if (tid) P = sh[tid - 1];
    else { P.len = 0; P.trail = 0; P.first = P.last = -1; P.uni = 1; P.pad = 0; }
    for (uint64_t t = a; t < e; ++t) {
        const RunSum64 S = load(t);
        const uint32_t c = (t > t0 && P.len > 0 && P.last == S.first) ? (uint32_t)(P.trail % 255u) : 0u;
        carry[t] = c;
        tile_w[t] = sums[t].wrest + lead_w(c, sums[t].lead);
        P = rs64_combine(P, S);
    }
}

__global__ void k_stream_w(const uint64_t* __restrict__ seg_tile0, const uint64_t* __restrict__ tile_wpre,
                           uint32_t nstreams, uint64_t* __restrict__ out)
{
    uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s < nstreams) out[s] = tile_wpre[seg_tile0[s + 1]] - tile_wpre[seg_tile0[s]];
}

// Chunk positions t of K consecutive bytes per lane (lane l: bytes p0 + K*l +
// k, packed 4 per word), one wave: tin = t of byte p0 - 1 and bin its value
// (p0 starting a stream: tin 254, bin = text[p0]).  Bytes at or past lim get
// t = 1 (no chunk starts there; the callers give them no weight).
template <int K>
__device__ __forceinline__ void run_t(const uint8_t* __restrict__ text, uint64_t p0, uint64_t lim, uint32_t tin,
                                      uint32_t bin, uint32_t (&tw)[K / 4])
{
    const int lane = threadIdx.x & 63;
    const uint64_t a = p0 + (uint64_t)K * (uint64_t)lane;
    uint32_t w[K / 4];
    if constexpr (K >= 16) {
#pragma unroll
        for (int i = 0; i < K / 16; ++i) {
            const uint64_t p = a + 16u * (uint64_t)i;
            const uint4 v = p < lim ? load16u(text + p, text + lim) : make_uint4(0, 0, 0, 0);
            w[4 * i] = v.x; w[4 * i + 1] = v.y; w[4 * i + 2] = v.z; w[4 * i + 3] = v.w;
        }
    } else {
        static_assert(K == 4, "run_t: K = 4 or a multiple of 16");
        w[0] = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (a + k < lim) w[0] |= (uint32_t)text[a + k] << (8 * k);
    }
    uint32_t carry = (uint32_t)__shfl_up((int)(w[K / 4 - 1] >> 24), 1, 64);
    if (lane == 0) carry = bin & 0xffu;
    uint32_t m[K / 4];
    int lc = -1;
#pragma unroll
    for (int i = 0; i < K / 4; ++i) {
        const uint32_t sh = (w[i] << 8) | carry;
        carry = w[i] >> 24;
        const uint64_t pi = a + 4u * (uint64_t)i;
        const int lim_i = pi >= lim ? 0 : (lim - pi >= 4 ? 4 : (int)(lim - pi));
        const uint32_t keep = lim_i >= 4 ? 0x80808080u : (lim_i <= 0 ? 0u : (0x80808080u >> (8 * (4 - lim_i))));
        m[i] = nonzero_bytes(w[i] ^ sh) & keep;
        if (m[i]) lc = 4 * i + ((31 - __clz((int)m[i])) >> 3);
    }
    const uint32_t x = lc >= 0 ? (uint32_t)(K * lane + lc + 1) : 0u;   // last change + 1, relative to p0
    const uint32_t incl = wave_incl_scan_max<uint32_t>(x);
    uint32_t ex = (uint32_t)__shfl_up((int)incl, 1, 64);
    if (lane == 0) ex = 0;
    uint32_t tp = ex ? ((uint32_t)(K * lane) - ex) % 255u : (tin + (uint32_t)(K * lane)) % 255u;   // t of byte a - 1
#pragma unroll
    for (int q = 0; q < K / 4; ++q) tw[q] = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const bool chg = ((m[k >> 2] >> (8 * (k & 3) + 7)) & 1u) != 0;
        const uint32_t t = chg ? 0u : (tp == 254u ? 0u : tp + 1u);
        tw[k >> 2] |= (a + k < lim ? t : 1u) << (8 * (k & 3));
        tp = t;
    }
}

// Block-cut tables.  The cut is a chain -- block k + 1 starts at the first
// chunk start whose RLE1 offset W reaches W_k + nblockMAX -- so one wave per
// stream walks it; walking it by searching the text per block left the GPU
// idle for ~8 us per block.  Since W_{k+1} - W_k - nblockMAX is 0..4 (a chunk
// weighs at most 5), W_k = k * nblockMAX + e_k with a slowly growing e_k, and
// every block's end can be tabulated in parallel beforehand for e in
// [0, CUT_E): one wave per (stream, k) finds the chunk starts c whose W(c) -
// T0 lies in [0, CUT_E), T0 = (k + 1) * nblockMAX, in the tile where W
// crosses T0 and the next one, and stores for every e the first of them at or
// past T0 + e (its offset in dtab, its text position in ptab).  254: none
// before the stream ends; 255: not within the two tiles (the walk then
// searches the text as before).  The walk itself becomes one table read per
// block, the next row already loaded.
constexpr int CUT_E = 128;
constexpr int CUT_WPG = 4;                       // (stream, k) waves per workgroup

__global__ void __launch_bounds__(64 * CUT_WPG) k_cut_tab(const StreamIn* __restrict__ streams,
                                                         const uint64_t* __restrict__ seg_tile0,
                                                         const uint64_t* __restrict__ tile_wpre,
                                                         const uint8_t* __restrict__ text,
                                                         const uint32_t* __restrict__ carry, uint32_t nblock_max,
                                                         const uint64_t* __restrict__ slot0, uint8_t* __restrict__ dtab,
                                                         uint64_t* __restrict__ ptab)
{
    __shared__ uint64_t pos_sh[CUT_WPG][CUT_E];
    const uint32_t s = blockIdx.y;
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint64_t k = (uint64_t)blockIdx.x * CUT_WPG + (uint64_t)wv;
    if (k >= slot0[s + 1] - slot0[s]) return;                  // wave-uniform from here on
    const uint64_t beg = streams[s].text_off, end = beg + streams[s].text_len;
    const uint64_t t0 = seg_tile0[s], t1 = seg_tile0[s + 1];
    if (t1 == t0) return;
    const uint64_t w0 = tile_wpre[t0], wend = tile_wpre[t1] - w0;
    const uint64_t T0 = (k + 1) * (uint64_t)nblock_max;
    if (T0 > wend) return;                                      // the walk reads no such row
    // tile lo with W(lo) < T0 <= W(lo + 1) (tile starts; W(t1) = wend): a
    // 64-tile window around T0 / kTB (a byte weighs about one), bisection otherwise
    uint64_t lo = t0, hi = t1;
    {
        const uint64_t g = t0 + T0 / kTB;
        uint64_t a = g > t0 + 32 ? g - 32 : t0;
        if (a + 64 > hi) a = hi > t0 + 64 ? hi - 64 : t0;
        const uint64_t t = a + (uint64_t)lane;
        const uint64_t ball = __ballot(t <= hi && tile_wpre[t] - w0 >= T0);
        const bool below_all = (tile_wpre[a] - w0) < T0;
        if (ball && below_all) {
            hi = a + (uint64_t)(__ffsll((unsigned long long)ball) - 1);
            lo = hi - 1;
        } else if (ball) {
            hi = a;
        } else if (a + 63 < hi) {
            lo = a + 63;
        }
    }
    while (hi - lo > 1) {
        const uint64_t mid = (lo + hi) >> 1;
        if (tile_wpre[mid] - w0 < T0) lo = mid; else hi = mid;
    }
    // chunk starts of tiles lo and lo + 1 with W - T0 in [0, CUT_E): a bit each
    uint32_t mk[CUT_E / 32];
#pragma unroll
    for (int i = 0; i < CUT_E / 32; ++i) mk[i] = 0;
    bool to_end = false;                                        // the two tiles reach the stream's end
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const uint64_t tj = lo + (uint64_t)j;
        if (tj >= t1) { to_end = true; break; }                 // (uniform)
        const uint64_t tstart = beg + (tj - t0) * kTB;
        const uint64_t tend = tstart + kTB < end ? tstart + kTB : end;
        if (tend == end) to_end = true;
        uint32_t tw[16];
        run_t<64>(text, tstart, tend, (carry[tj] + 254u) % 255u, text[tstart], tw);
        uint32_t ls = 0;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const uint32_t l3 = ~nonzero_bytes(tw[q] & 0xFCFCFCFCu) & 0x80808080u;   // t <= 3
            const uint32_t e3 = ~nonzero_bytes(tw[q] ^ 0x03030303u) & 0x80808080u;  // t == 3
            ls += (uint32_t)(__popc(l3) + __popc(e3));
        }
        // (bytes past tend carry t = 1: weight 1, after every real byte of the lane)
        uint64_t W = tile_wpre[tj] - w0 + (wave_incl_scan_add<uint32_t>(ls) - ls);
        const uint64_t a = tstart + 64u * (uint64_t)lane;
#pragma unroll
        for (int b = 0; b < 64; ++b) {
            const uint32_t t = (tw[b >> 2] >> (8 * (b & 3))) & 0xffu;
            if (t == 0 && a + b < tend && W >= T0 && W - T0 < (uint64_t)CUT_E) {
                const uint32_t o = (uint32_t)(W - T0);
#pragma unroll
                for (int i = 0; i < CUT_E / 32; ++i)
                    if ((o >> 5) == (uint32_t)i) mk[i] |= 1u << (o & 31u);
                pos_sh[wv][o] = a + (uint64_t)b;
            }
            W += rle_w(t);
        }
    }
#pragma unroll
    for (int i = 0; i < CUT_E / 32; ++i)
        mk[i] = (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan_or(mk[i]), 63);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint64_t row = (slot0[s] + k) * (uint64_t)CUT_E;
#pragma unroll
    for (int h = 0; h < CUT_E / 64; ++h) {
        const uint32_t e = (uint32_t)lane + 64u * h;
        int b = -1;                                             // first bit >= e
#pragma unroll
        for (int i = 0; i < CUT_E / 32; ++i) {
            const uint32_t lo_bit = (uint32_t)i * 32u;
            const uint32_t mm = e <= lo_bit ? mk[i] : (e < lo_bit + 32u ? mk[i] & (~0u << (e - lo_bit)) : 0u);
            if (b < 0 && mm) b = (int)lo_bit + __builtin_ctz(mm);
        }
        dtab[row + e] = b >= 0 ? (uint8_t)b : (to_end ? (uint8_t)254 : (uint8_t)255);
        ptab[row + e] = b >= 0 ? pos_sh[wv][b] : end;
    }
}

// one wave per stream: greedy cut (see file header).  Per block: binary search
// of the tile where the RLE1 size crosses nblockMAX, the chunk positions of
// that tile (run_t, from its entering run position) and a 64-lane scan of
// their weights for the crossing byte q, then a ballot over the next 256
// bytes for the first chunk start p >= q (chunks are at most 255 bytes).
__global__ void __launch_bounds__(64) k_cut(const StreamIn* __restrict__ streams, const uint64_t* __restrict__ seg_tile0,
                                             const uint64_t* __restrict__ tile_wpre, const uint8_t* __restrict__ text,
                                             const uint32_t* __restrict__ carry, uint32_t nstreams, uint32_t nblock_max,
                                             const uint64_t* __restrict__ slot0, const uint8_t* __restrict__ dtab,
                                             const uint64_t* __restrict__ ptab, BlockDesc* __restrict__ tmp,
                                             uint32_t* __restrict__ nblk)
{
    const uint32_t s = blockIdx.x;
    const int lane = threadIdx.x;
    const uint64_t beg = streams[s].text_off, end = beg + streams[s].text_len;
    const uint64_t t0 = seg_tile0[s], t1 = seg_tile0[s + 1];
    const uint64_t w0 = tile_wpre[t0], wend = tile_wpre[t1] - w0;
    const bool frj = streams[s].final_run_joins != 0;
    const uint64_t nrow = slot0[s + 1] - slot0[s];
    uint64_t bs = beg, wbs = 0;
    uint32_t k = 0;
    // table rows (k_cut_tab): lane l holds entries l and l + 64, the next row in flight
    uint32_t da = 255u, db = 255u;
    uint64_t pa = 0, pb = 0;
    auto row = [&](uint32_t kk, uint32_t& xa, uint32_t& xb, uint64_t& ya, uint64_t& yb) {
        xa = xb = 255u;
        ya = yb = 0;
        if (dtab && kk < nrow) {
            const uint64_t r = (slot0[s] + kk) * (uint64_t)CUT_E;
            xa = dtab[r + lane];
            xb = dtab[r + 64 + lane];
            ya = ptab[r + lane];
            yb = ptab[r + 64 + lane];
        }
    };
    row(0, da, db, pa, pb);
    while (bs < end) {
        const uint64_t target = wbs + nblock_max;
        uint64_t block_end = end, wblock_end = wend;
        uint32_t na, nb2;
        uint64_t qa, qb;
        row(k + 1, na, nb2, qa, qb);
        if (wend >= target) {
          // this block's end from its table row when W_k - k * nblockMAX is tabulated
          const uint64_t e = wbs - (uint64_t)k * nblock_max;
          uint32_t d = 255u;
          if (e < (uint64_t)CUT_E)
              d = (uint32_t)__builtin_amdgcn_readlane((int)(e < 64 ? da : db), (int)(e & 63u));
          uint64_t p = end, Wp = wend;
          if (d < 254u) {
              const uint64_t pp = e < 64 ? pa : pb;
              const uint32_t plo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)pp, (int)(e & 63u));
              const uint32_t phi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(pp >> 32), (int)(e & 63u));
              p = ((uint64_t)phi << 32) | plo;
              Wp = (uint64_t)(k + 1) * nblock_max + d;
          } else if (d == 255u) {   // not tabulated: search the text
            uint64_t lo = t0 + (bs - beg) / kTB, hi = t1;   // Wstart(lo) <= wbs < target <= Wstart(hi)
            // RLE1 sizes run close to text sizes (a byte weighs 0..2), so the
            // crossing tile sits near lo + (target - W(lo)) / kTB: one window of
            // 64 tiles around that guess, one round trip; bisection otherwise
            {
                const uint64_t wl = tile_wpre[lo] - w0;
                uint64_t g = lo + (target > wl ? (target - wl) / kTB : 0);
                uint64_t a = g > lo + 32 ? g - 32 : lo;
                if (a + 64 > hi) a = hi > lo + 64 ? hi - 64 : lo;
                const uint64_t t = a + (uint64_t)lane;
                const bool ge = t < hi && tile_wpre[t] - w0 >= target;
                const uint64_t ball = __ballot(ge);
                const bool below_all = (tile_wpre[a] - w0) < target;   // the window starts below the target
                if (ball && below_all) {         // crossing inside the window: adjacent (lo, hi)
                    const uint64_t f = a + (uint64_t)(__ffsll((unsigned long long)ball) - 1);
                    hi = f;
                    lo = f - 1;
                } else if (ball) {               // W(a) >= target: before the window (a > lo)
                    hi = a;
                } else if (a + 63 < hi) {        // after the window
                    lo = a + 63;
                }
            }
            while (hi - lo > 1) {
                uint64_t mid = (lo + hi) >> 1;
                if (tile_wpre[mid] - w0 < target) lo = mid; else hi = mid;
            }
            uint64_t q = 0, Wq = 0;
            uint32_t tq = 0;                 // chunk position of byte q - 1
            for (;;) {   // normally one iteration
                const uint64_t tstart = beg + (lo - t0) * kTB;
                uint64_t tend = tstart + kTB;
                if (tend > end) tend = end;
                const uint64_t y0 = tstart < bs ? bs : tstart;
                const uint64_t W0 = tstart < bs ? wbs : tile_wpre[lo] - w0;
                // each lane: 64 bytes of the tile and their chunk positions in
                // registers; bytes outside [y0, tend) weigh 0
                const uint64_t a = tstart + (uint64_t)lane * 64;
                uint32_t tw[16];
                run_t<64>(text, tstart, tend, (carry[lo] + 254u) % 255u, text[tstart], tw);
                uint32_t ssum = 0;
#pragma unroll
                for (int k = 0; k < 64; ++k) {
                    const uint64_t y = a + (uint64_t)k;
                    if (y >= y0 && y < tend) ssum += rle_w((tw[k >> 2] >> (8 * (k & 3))) & 0xffu);
                }
                const uint32_t incl = wave_incl_scan_add(ssum);
                const uint64_t ball = __ballot(a < tend && W0 + incl >= target);
                if (ball) {
                    const int L = __ffsll((unsigned long long)ball) - 1;
                    uint64_t x = a < y0 ? y0 : a, Wx = W0 + incl - ssum;
                    uint32_t tx = 0;
                    {   // the crossing byte, from the registers: per-word weights
                        // by SWAR (rle_w = [t <= 3] + [t == 3]), then a walk over
                        // 16 words and 4 bytes instead of 64 bytes
                        const int kq = y0 > a ? (y0 - a < 64 ? (int)(y0 - a) : 64) : 0;
                        const int kt = tend > a ? (tend - a < 64 ? (int)(tend - a) : 64) : 0;
                        auto upto = [](int n) { return n >= 4 ? 0x80808080u : (n <= 0 ? 0u : (0x80808080u >> (8 * (4 - n)))); };
                        uint32_t need = (uint32_t)(target - Wx);   // > 0 in lane L
                        uint32_t le = 0, eq = 0;
                        int wsel = -1;
#pragma unroll
                        for (int i = 0; i < 16; ++i) {
                            const uint32_t vm = upto(kt - 4 * i) & ~upto(kq - 4 * i);
                            const uint32_t l3 = ~nonzero_bytes(tw[i] & 0xFCFCFCFCu) & vm;
                            const uint32_t e3 = ~nonzero_bytes(tw[i] ^ 0x03030303u) & vm;
                            const uint32_t wi = (uint32_t)(__popc(l3) + __popc(e3));
                            if (wsel < 0) {
                                if (wi < need) need -= wi;
                                else { wsel = i; le = l3; eq = e3; }
                            }
                        }
                        if (wsel >= 0) {
                            int jsel = 3;
#pragma unroll
                            for (int j = 3; j >= 0; --j) {   // first byte j whose prefix weight reaches need
                                const uint32_t c = (uint32_t)(__popc(le & upto(j + 1)) + __popc(eq & upto(j + 1)));
                                if (c >= need) jsel = j;
                            }
                            const uint32_t cj = (uint32_t)(__popc(le & upto(jsel + 1)) + __popc(eq & upto(jsel + 1)));
                            x = a + (uint64_t)(4 * wsel + jsel) + 1;
                            Wx = target - need + cj;
                            tx = (tw[wsel] >> (8 * jsel)) & 0xffu;
                        }
                    }
                    q = __shfl(x, L, 64);
                    Wq = __shfl(Wx, L, 64);
                    tq = (uint32_t)__shfl((int)tx, L, 64);
                    break;
                }
                ++lo;   // cannot happen when the tile search is exact; stay safe
                if (lo >= t1) { q = end; Wq = wend; break; }
            }
            // the first chunk start p >= q (within 255 bytes) and the weight of
            // [q, p): the chunk positions of the 256 bytes after q, four per lane
            uint32_t part = 0;
            if (q < end) {
                uint32_t tv[1];
                run_t<4>(text, q, end, tq, text[q - 1], tv);
                const uint32_t zb = ~nonzero_bytes(tv[0]) & 0x80808080u;   // bytes with t == 0
                const uint64_t hit = __ballot(zb != 0);
                if (hit) {
                    const int L = __ffsll((unsigned long long)hit) - 1;
                    const uint32_t zl = (uint32_t)__shfl((int)zb, L, 64);
                    p = q + 4u * (uint64_t)L + (uint64_t)((__builtin_ctz(zl) - 7) >> 3);
                }
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const uint64_t pos = q + 4u * (uint64_t)lane + k;
                    if (pos < p) part += rle_w((tv[0] >> (8 * k)) & 0xffu);
                }
            }
            Wp = Wq + wave_reduce_add(part);
          }
          if (p < end && !(frj && p == end - 1)) { block_end = p; wblock_end = Wp; }
        }
        if (lane == 0) {
            BlockDesc b;
            b.in_beg = bs; b.in_end = block_end; b.w_beg = wbs; b.n = (uint32_t)(wblock_end - wbs); b.stream = s;
            tmp[slot0[s] + k] = b;
        }
        ++k;
        bs = block_end;
        wbs = wblock_end;
        da = na; db = nb2; pa = qa; pb = qb;
    }
    if (lane == 0) nblk[s] = k;
}

// first block index of every stream (exclusive scan of the per-stream block
// counts k_cut left) and the block total, on the device: one workgroup
__global__ void __launch_bounds__(1024) k_block_first(const uint32_t* __restrict__ nblk, uint32_t ns,
                                                       uint32_t* __restrict__ first, uint32_t* __restrict__ total)
{
    __shared__ uint32_t sh[1024 / 64 + 1];
    uint32_t carry = 0;
    for (uint32_t s0 = 0; s0 < ns; s0 += 1024) {
        const uint32_t s = s0 + threadIdx.x;
        uint32_t tot = 0;
        const uint32_t ex = block_excl_scan_add<uint32_t>(s < ns ? nblk[s] : 0u, sh, &tot);
        if (s < ns) first[s] = carry + ex;
        carry += tot;
    }
    if (threadIdx.x == 0) *total = carry;
}

// also maps every tile to the block holding its first byte (tile_block)
__global__ void k_compact_blocks(const BlockDesc* __restrict__ tmp, const uint64_t* __restrict__ slot0,
                                 const uint32_t* __restrict__ nblk, const uint32_t* __restrict__ first,
                                 uint32_t nstreams, BlockDesc* __restrict__ out, const StreamIn* __restrict__ streams,
                                 const uint64_t* __restrict__ seg_tile0, uint32_t* __restrict__ tile_block)
{
    uint32_t s = blockIdx.x;
    if (s >= nstreams) return;
    const uint64_t beg = streams[s].text_off, t0 = seg_tile0[s];
    for (uint32_t k = threadIdx.x; k < nblk[s]; k += blockDim.x) {
        BlockDesc b = tmp[slot0[s] + k];
        const uint64_t ta = (b.in_beg - beg + kTB - 1) / kTB, te = (b.in_end - beg + kTB - 1) / kTB;
        for (uint64_t t = ta; t < te; ++t) tile_block[t0 + t] = first[s] + k;
        b.bits = 0; b.bit_off = 0; b.crc = 0; b.orig_ptr = 0; b.n_in_use = 0; b.n_mtf = 0; b.flags = 0;
        b.n_groups = 0; b.n_sel = 0;
        for (int j = 0; j < 8; ++j) b.in_use[j] = 0;
        out[first[s] + k] = b;
    }
}

// cooperative LDS -> global byte copy by the workgroup: head bytes up to a
// 4-byte aligned destination, 4-byte stores, then the tail (the word stores
// stay inside [dst, dst + len), so neighbouring tiles never overlap)
__device__ __forceinline__ void copy_out(uint8_t* dst, const uint8_t* src, uint32_t len)
{
    const uint32_t head0 = (uint32_t)((4u - ((uintptr_t)dst & 3u)) & 3u);
    const uint32_t head = head0 < len ? head0 : len;
    if (threadIdx.x < head) dst[threadIdx.x] = src[threadIdx.x];
    const uint32_t nw = (len - head) / 4u;
    uint32_t* d4 = reinterpret_cast<uint32_t*>(dst + head);
    for (uint32_t w = threadIdx.x; w < nw; w += blockDim.x) {
        const uint32_t q = head + 4u * w;
        d4[w] = (uint32_t)src[q] | ((uint32_t)src[q + 1] << 8) | ((uint32_t)src[q + 2] << 16) |
                ((uint32_t)src[q + 3] << 24);
    }
    for (uint32_t k = head + 4u * nw + threadIdx.x; k < len; k += blockDim.x) dst[k] = src[k];
}

// materialise RLE1 block bytes (bz:bzlib.c:224-256) + inUse (bz:bzlib.c:232,247)
__global__ void __launch_bounds__(256) k_rle_emit(const uint8_t* __restrict__ text, const TileDesc* __restrict__ tiles,
                                                   const uint64_t* __restrict__ tile_wpre,
                                                   const uint64_t* __restrict__ seg_tile0,
                                                   const uint32_t* __restrict__ carry, const StreamIn* __restrict__ streams,
                                                   const uint32_t* __restrict__ sfirst, const uint32_t* __restrict__ snblk,
                                                   const uint32_t* __restrict__ tile_block,
                                                   BlockDesc* __restrict__ blocks, uint8_t* __restrict__ blk,
                                                   uint64_t stride)
{
    __shared__ uint32_t wsh[5], msh[4];
    __shared__ uint8_t ob[kTB + kTB / 4 + 16];      // the tile's RLE1 output (<= 5/4 of its bytes)
    // inUse bits per lane ([slot][word][lane]: no two lanes share a word, so no
    // serialised LDS atomics on the few words a text's bytes fall in)
    __shared__ uint32_t ul[2][8][256];
    TileDesc d = tiles[blockIdx.x];
    const uint32_t s = d.stream;
    const uint64_t send = streams[s].text_off + streams[s].text_len;
#pragma unroll
    for (int q = 0; q < 16; ++q) ul[q >> 3][q & 7][threadIdx.x] = 0;
    const uint32_t bsel = tile_block[blockIdx.x];   // block holding the tile's first byte
    int off = threadIdx.x * 16;
    int cnt = (int)d.len - off;
    cnt = cnt < 0 ? 0 : (cnt > 16 ? 16 : cnt);
    // the strip's chunk positions, from the tile's changes and its entering run position
    uint4 xv;
    uint32_t pb;
    load_strip(text, d, off, cnt, xv, pb);
    uint32_t m[4];
    chg_mask(xv, pb, cnt, m);
    const int lc = last_change(m);
    const uint32_t ex = tile_ex(lc >= 0 ? (uint32_t)(off + lc + 1) : 0u, msh);
    uint32_t twd[4];
    const uint32_t w = strip_t<true>(m, (uint32_t)off, cnt, ex, carry[blockIdx.x], twd);
    const uint4 tv = make_uint4(twd[0], twd[1], twd[2], twd[3]);
    uint32_t tot = 0;
    const uint32_t pre = block_excl_scan_add<uint32_t>(w, wsh, &tot);   // contains __syncthreads
    const uint32_t b0 = bsel;
    const uint32_t bl = sfirst[s] + snblk[s];
    // the tile's output is built in LDS at its scan offsets, then copied out
    // with coalesced stores into at most two blocks (blocks are cut at chunk
    // starts, so a chunk's bytes never straddle two blocks; a block holds far
    // more than one tile)
    const uint64_t Wt = tile_wpre[blockIdx.x] - tile_wpre[seg_tile0[s]];   // stream W of the tile's first byte
    const uint64_t wb0 = blocks[b0].w_beg;
    const uint64_t wnext = b0 + 1 < bl ? blocks[b0 + 1].w_beg : ~0ull;
    // the strip's changes as 16 bits (bit p: byte p differs from the one before),
    // the bytes past the strip counted as changes: a chunk length (t == 3) whose
    // run ends inside the strip is read off the mask, without loading the text
    uint32_t cm = cnt < 16 ? (0xffffu << cnt) & 0xffffu : 0u;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t x = m[i] >> 7;
        cm |= ((x | (x >> 7) | (x >> 14) | (x >> 21)) & 0xfu) << (4 * i);
    }
    uint32_t o = pre;
    for (int k = 0; k < cnt; ++k) {
        const uint32_t t = byte16(tv, k);
        const uint8_t c = (uint8_t)byte16(xv, k);
        const int slot = (Wt + o >= wnext) ? 1 : 0;
        if (t < 3) {
            ob[o] = c;
            // an LDS OR with no return (ds_or_b32): no read-modify-write chain
            // through the byte loop
            if (t == 0) atomicOr(&ul[slot][c >> 5][threadIdx.x], 1u << (c & 31));
        } else if (t == 3) {
            // the chunk's length: its bytes go on while they equal c, up to 255
            // (its start i - 3 plus 254)
            const uint64_t i = d.beg + off + k;
            const uint32_t rest = (cm >> (k + 1)) | 0x10000u;   // bit 16 - k - 1: past the strip
            const uint32_t p = (uint32_t)k + 1u + (uint32_t)__builtin_ctz(rest);   // first change after k
            uint64_t j = i + (p - (uint32_t)k);
            if (p >= (uint32_t)cnt) {                          // the run reaches the strip's end
                const uint64_t jl = i + 252 < send ? i + 252 : send;
                j = d.beg + off + cnt;
                while (j < jl && text[j] == c) ++j;
            }
            const uint32_t L = (uint32_t)(j - i) + 3;
            const uint8_t cnt_byte = (uint8_t)(L - 4);
            ob[o] = c;
            ob[o + 1] = cnt_byte;
            atomicOr(&ul[slot][cnt_byte >> 5][threadIdx.x], 1u << (cnt_byte & 31));
        }
        o += rle_w(t);
    }
    __syncthreads();
    const uint32_t split = wnext > Wt ? (wnext - Wt < tot ? (uint32_t)(wnext - Wt) : tot) : 0u;
    copy_out(blk + (uint64_t)b0 * stride + (Wt - wb0), ob, split);
    if (split < tot) copy_out(blk + (uint64_t)(b0 + 1) * stride, ob + split, tot - split);
    {   // OR of the 256 lanes' words: 16 threads per (slot, word), each ORs 16
        // lanes' words (four 16-B LDS reads), then DPP row shifts OR the 16
        // threads into the row's last lane, which publishes the word
        const int pr = threadIdx.x >> 4, r = threadIdx.x & 15;
        const uint4* row = reinterpret_cast<const uint4*>(&ul[pr >> 3][pr & 7][r * 16]);
        uint32_t v = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) { const uint4 x = row[i]; v |= x.x | x.y | x.z | x.w; }
        v |= dpp_up(v, 1);
        v |= dpp_up(v, 2);
        v |= dpp_up(v, 4);
        v |= dpp_up(v, 8);
        const uint32_t bb = b0 + (uint32_t)(pr >> 3);
        if (r == 15 && v && bb < bl) atomicOr(&blocks[bb].in_use[pr & 7], v);
    }
}

// CRC-32/BZIP2 of [in_beg, in_end) per block (bz:bzlib_private.h:155-172).
// R(A||B) = R(A)*x^(8|B|) + R(B) (mod P); crc = ~(0xffffffff*x^(8n) + R(all)).
// k_crc_chunks: each wave takes one chunk of a block (up to CRC_MAXC chunks,
// whole 8 KB spans); every lane runs slice-by-4 over its own 128-byte line of
// a span (eight 16-B loads in flight); then R(span) = XOR_i R(line_i) *
// x^(8 * bytes after line i): each lane shifts its own register (a constant
// per lane for a full span) and one XOR reduction over the wave combines them
// -- one multiplication deep instead of a six-level tree of them.
// k_crc_final: one wave per block combines the chunk registers the same way.
constexpr uint32_t CRC_LANE = 128;                // bytes per lane per span
constexpr uint32_t CRC_SPAN = 64 * CRC_LANE;      // 8 KB per wave per span
constexpr uint32_t CRC_MAXC = 128;
constexpr int CRC_WPB = 4;                        // chunks (waves) per workgroup

__device__ __forceinline__ uint64_t crc_chunk_bytes(uint64_t span)
{
    uint64_t c = (span + CRC_MAXC - 1) / CRC_MAXC;
    c = (c + CRC_SPAN - 1) / CRC_SPAN * CRC_SPAN;
    return c < CRC_SPAN ? CRC_SPAN : c;
}

__global__ void __launch_bounds__(64 * CRC_WPB) k_crc_chunks(const uint8_t* __restrict__ text,
                                                             const BlockDesc* __restrict__ blocks,
                                                             uint32_t* __restrict__ creg, const uint32_t* __restrict__ nbd)
{
    if (nbd && blockIdx.y >= *nbd) return;           // grid sized by the host's upper bound
    __shared__ uint32_t t4[4][256];
    for (int i = threadIdx.x; i < 1024; i += 64 * CRC_WPB) (&t4[0][0])[i] = (&c_crc_tab4[0][0])[i];
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const uint32_t c = blockIdx.x * CRC_WPB + (threadIdx.x >> 6), b = blockIdx.y;
    const uint64_t beg = blocks[b].in_beg, end = blocks[b].in_end;
    const uint64_t csz = crc_chunk_bytes(end - beg);
    const uint64_t cb = beg + (uint64_t)c * csz;
    if (c >= CRC_MAXC || cb >= end) return;          // per wave; no barriers below
    const uint64_t ce = cb + csz < end ? cb + csz : end;
    uint32_t acc = 0;
    for (uint64_t c0 = cb; c0 < ce; c0 += CRC_SPAN) {
        const uint64_t a = c0 + (uint64_t)lane * CRC_LANE;
        const uint32_t n = a < ce ? (uint32_t)(ce - a < CRC_LANE ? ce - a : CRC_LANE) : 0u;
        uint4 v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k)
            v[k] = (16u * k < n) ? load16u(text + a + 16 * k, text + ce) : make_uint4(0, 0, 0, 0);
        uint32_t r = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t m = n > 16u * k ? (n - 16u * k < 16u ? n - 16u * k : 16u) : 0u;
            if (m == 16) {
                const uint32_t ws[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const uint32_t x = r ^ __builtin_bswap32(ws[q]);   // bytes in stream order, MSB-first
                    r = t4[3][x >> 24] ^ t4[2][(x >> 16) & 255u] ^ t4[1][(x >> 8) & 255u] ^ t4[0][x & 255u];
                }
            } else {
                for (uint32_t q = 0; q < m; ++q) r = (r << 8) ^ t4[0][(r >> 24) ^ byte16(v[k], (int)q)];
            }
        }
        const uint32_t slen = ce - c0 < CRC_SPAN ? (uint32_t)(ce - c0) : CRC_SPAN;
        const uint32_t lend = (uint32_t)(lane + 1) * CRC_LANE;
        uint32_t x = 0;
        if (n) x = mulmod(r, slen == CRC_SPAN ? c_lane[lane] : xpow8(slen - (lend < slen ? lend : slen)));
#pragma unroll
        for (int l = 1; l < 64; l <<= 1) x ^= __shfl_xor(x, l, 64);
        if (lane == 0) acc = mulmod(acc, slen == CRC_SPAN ? c_pow8[13] : xpow8(slen)) ^ x;
    }
    if (lane == 0) creg[(uint64_t)b * CRC_MAXC + c] = acc;
}

__global__ void __launch_bounds__(64) k_crc_final(const uint32_t* __restrict__ creg, BlockDesc* __restrict__ blocks,
                                                   const uint32_t* __restrict__ nbd)
{
    const uint32_t b = blockIdx.x;
    if (nbd && b >= *nbd) return;
    const int lane = threadIdx.x;
    const uint64_t beg = blocks[b].in_beg, end = blocks[b].in_end;
    const uint64_t csz = crc_chunk_bytes(end - beg);
    const uint32_t nch = (uint32_t)((end - beg + csz - 1) / csz);
    // lane l holds chunks 2l, 2l+1 (CRC_MAXC = 128 = 2 * 64), shifted by the
    // bytes after them; one XOR reduction combines the lanes
    uint32_t r = 0;
    uint64_t pend = beg;                              // end of this lane's chunks
    for (int q = 0; q < 2; ++q) {
        const uint32_t k = 2u * lane + q;
        if (k < nch) {
            const uint64_t cb = beg + (uint64_t)k * csz;
            const uint64_t cl = (end - cb) < csz ? end - cb : csz;
            r = (q ? mulmod(r, xpow8(cl)) : 0u) ^ creg[(uint64_t)b * CRC_MAXC + k];
            pend = cb + cl;
        }
    }
    uint32_t x = 0;
    if (2u * lane < nch) x = mulmod(r, xpow8(end - pend));
    for (int l = 1; l < 64; l <<= 1) x ^= __shfl_xor(x, l, 64);
    if (lane == 0) blocks[b].crc = ~(mulmod(0xffffffffu, xpow8(end - beg)) ^ x);
}

// ---------------------------------------------------------------------------
// launch wrappers (host)
// ---------------------------------------------------------------------------
static inline unsigned g1(uint64_t n, unsigned b) { return (unsigned)((n + b - 1) / b); }

void rle_tiles(const uint64_t* tile0, const StreamIn* streams, uint32_t ns, uint64_t ntiles, TileDesc* tiles,
               hipStream_t st)
{
    hipLaunchKernelGGL(k_tiles, dim3(g1(ntiles, 256)), dim3(256), 0, st, tile0, streams, ns, ntiles, tiles);
}
void rle_sum(const uint8_t* text, const TileDesc* tiles, uint64_t ntiles, TileSum* sums, hipStream_t st)
{
    hipLaunchKernelGGL(k_rle_sum, dim3((unsigned)((ntiles + SUM_WPG - 1) / SUM_WPG)), dim3(64 * SUM_WPG), 0, st, text,
                       tiles, ntiles, sums);
}
void rle_carry(const uint64_t* tile0, uint32_t ns, const TileSum* sums, uint32_t* carry, uint32_t* tile_w,
               hipStream_t st)
{
    hipLaunchKernelGGL(k_rle_carry, dim3(ns), dim3(CT), 0, st, tile0, ns, sums, carry, tile_w);
}
void rle_stream_w(const uint64_t* tile0, const uint64_t* wpre, uint32_t ns, uint64_t* out, hipStream_t st)
{
    hipLaunchKernelGGL(k_stream_w, dim3(g1(ns, 64)), dim3(64), 0, st, tile0, wpre, ns, out);
}
uint64_t rle_cut_tab_bytes(uint64_t nslots) { return nslots * CUT_E * (1 + sizeof(uint64_t)) + 64; }

void rle_cut(const StreamIn* streams, const uint64_t* tile0, const uint64_t* wpre, const uint8_t* text,
             const uint32_t* carry, uint32_t ns, uint32_t nblock_max, const uint64_t* slot0, uint64_t nslots,
             uint64_t max_slots, void* tab, BlockDesc* tmp, uint32_t* nblk, hipStream_t st)
{
    // STARCH_CUT_TAB=0: the walk searches the text for every block
    static const bool tab_off = [] { const char* e = getenv("STARCH_CUT_TAB"); return e && !strcmp(e, "0"); }();
    uint64_t* ptab = nullptr;
    uint8_t* dtab = nullptr;
    if (!tab_off && tab && max_slots) {
        ptab = static_cast<uint64_t*>(tab);
        dtab = reinterpret_cast<uint8_t*>(ptab + nslots * CUT_E);
        hipLaunchKernelGGL(k_cut_tab, dim3((unsigned)((max_slots + CUT_WPG - 1) / CUT_WPG), ns), dim3(64 * CUT_WPG), 0, st,
                           streams, tile0, wpre, text, carry, nblock_max, slot0, dtab, ptab);
    }
    hipLaunchKernelGGL(k_cut, dim3(ns), dim3(64), 0, st, streams, tile0, wpre, text, carry, ns, nblock_max, slot0,
                       dtab, ptab, tmp, nblk);
}
void rle_compact(const BlockDesc* tmp, const uint64_t* slot0, const uint32_t* nblk, const uint32_t* first, uint32_t ns,
                 BlockDesc* out, const StreamIn* streams, const uint64_t* tile0, uint32_t* tile_block, hipStream_t st)
{
    hipLaunchKernelGGL(k_compact_blocks, dim3(ns), dim3(256), 0, st, tmp, slot0, nblk, first, ns, out, streams, tile0,
                       tile_block);
}
void rle_emit(const uint8_t* text, const TileDesc* tiles, uint64_t ntiles, const uint64_t* wpre, const uint64_t* tile0,
              const uint32_t* carry, const StreamIn* streams, const uint32_t* first, const uint32_t* nblk,
              const uint32_t* tile_block, BlockDesc* blocks, uint8_t* blk, uint64_t stride, hipStream_t st)
{
    hipLaunchKernelGGL(k_rle_emit, dim3((unsigned)ntiles), dim3(256), 0, st, text, tiles, wpre, tile0, carry, streams,
                       first, nblk, tile_block, blocks, blk, stride);
}
void rle_block_first(const uint32_t* nblk, uint32_t ns, uint32_t* first, uint32_t* total, hipStream_t st)
{
    hipLaunchKernelGGL(k_block_first, dim3(1), dim3(1024), 0, st, nblk, ns, first, total);
}
void rle_crc(const uint8_t* text, BlockDesc* blocks, uint32_t nb_max, const uint32_t* nb_dev, uint32_t* creg,
             hipStream_t st)
{
    if (!nb_max) return;
    hipLaunchKernelGGL(k_crc_chunks, dim3(CRC_MAXC / CRC_WPB, nb_max), dim3(64 * CRC_WPB), 0, st, text, blocks, creg,
                       nb_dev);
    hipLaunchKernelGGL(k_crc_final, dim3(nb_max), dim3(64), 0, st, creg, blocks, nb_dev);
}

}  // namespace bz
