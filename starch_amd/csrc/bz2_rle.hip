// starch_amd/csrc/bz2_rle.hip -- RLE1, block cut and block CRC on MI355X.
//
// Restates bzip2-1.0.6's input side (bz:bzlib.c:224-338, 369-412) as
// data-parallel passes over 4 KiB tiles of a stream's bytes:
//   1. k_rle_sum    per-tile run summary (first/last byte, uniform, trailing run)
//   2. k_rle_carry  per-stream sequential fold -> run length entering each tile
//   3. k_rle_pos    per-byte RLE1 chunk position t = (position in run) mod 255
//                   and per-tile RLE1 output size (a chunk of L bytes emits
//                   min(L,4) copies + one count byte when L >= 4)
//   4. k_cut        per-stream greedy block cut over the RLE1 size prefix:
//                   chunk k joins the block iff the block holds < nblockMAX
//                   bytes before it (bz:bzlib.c:307,399-402); the final chunk
//                   joins a full block only when it is a single byte supplied
//                   with the finishing call (bz:bzlib.c:393-397)
//   5. k_rle_emit   materialise each block's RLE1 bytes + inUse map
//   6. k_block_crc  CRC-32/BZIP2 of each block's input bytes via GF(2) combine
#include "bz2_int.hpp"

namespace bz {

__constant__ uint32_t c_pow8[64];   // x^(8*2^k) mod P, P = 0x04c11db7 (MSB-first)
__constant__ uint32_t c_crc_tab[256];

void upload_crc_constants()
{
    static bool done = false;
    if (done) return;
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
    done = true;
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

struct RunSum {
    uint32_t len, trail;
    int first, last;
    bool uni;
};
__device__ __forceinline__ RunSum rs_combine(const RunSum& A, const RunSum& B)
{
    if (A.len == 0) return B;
    if (B.len == 0) return A;
    RunSum R;
    R.first = A.first;
    R.last = B.last;
    R.len = A.len + B.len;
    R.uni = A.uni && B.uni && A.last == B.first;
    R.trail = (B.uni && B.first == A.last) ? B.len + A.trail : B.trail;
    return R;
}

__device__ __forceinline__ RunSum strip_summary(const uint8_t* p, int cnt)
{
    RunSum r;
    r.len = 0; r.trail = 0; r.first = -1; r.last = -1; r.uni = true;
    if (cnt <= 0) return r;
    r.len = cnt;
    r.first = p[0];
    int last = p[0];
    uint32_t tr = 1;
    for (int k = 1; k < cnt; ++k) {
        int c = p[k];
        if (c == last) ++tr; else { tr = 1; r.uni = false; }
        last = c;
    }
    r.last = last;
    r.trail = tr;
    return r;
}

__global__ void __launch_bounds__(256) k_rle_sum(const uint8_t* __restrict__ text, const TileDesc* __restrict__ tiles,
                                                  TileSum* __restrict__ sums)
{
    __shared__ RunSum sh[256];
    TileDesc d = tiles[blockIdx.x];
    int off = threadIdx.x * 16;
    int cnt = (int)d.len - off;
    cnt = cnt < 0 ? 0 : (cnt > 16 ? 16 : cnt);
    sh[threadIdx.x] = strip_summary(text + d.beg + off, cnt);
    __syncthreads();
    if (threadIdx.x == 0) {
        RunSum acc = sh[0];
        for (int k = 1; k < 256; ++k) acc = rs_combine(acc, sh[k]);
        TileSum o;
        o.first = (uint8_t)acc.first;
        o.last = (uint8_t)acc.last;
        o.uni = acc.uni ? 1 : 0;
        o.len = acc.len;
        o.trail = acc.trail;
        sums[blockIdx.x] = o;
    }
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

__global__ void __launch_bounds__(256) k_rle_carry(const uint64_t* __restrict__ seg_tile0, uint32_t nstreams,
                                                    const TileSum* __restrict__ sums, uint32_t* __restrict__ carry)
{
    __shared__ RunSum64 sh[256];
    const uint32_t s = blockIdx.x;
    const int tid = threadIdx.x;
    const uint64_t t0 = seg_tile0[s], t1 = seg_tile0[s + 1];
    RunSum64 acc;
    acc.len = 0; acc.trail = 0; acc.first = acc.last = -1; acc.uni = 1; acc.pad = 0;
    for (uint64_t c0 = t0; c0 < t1; c0 += 256) {
        const uint64_t t = c0 + tid;
        RunSum64 S;
        S.len = 0; S.trail = 0; S.first = S.last = -1; S.uni = 1; S.pad = 0;
        if (t < t1) {
            TileSum x = sums[t];
            S.len = x.len; S.trail = x.trail; S.first = x.first; S.last = x.last; S.uni = x.uni;
        }
        sh[tid] = S;
        __syncthreads();
        for (int d = 1; d < 256; d <<= 1) {
            RunSum64 v = (tid >= d) ? rs64_combine(sh[tid - d], sh[tid]) : sh[tid];
            __syncthreads();
            sh[tid] = v;
            __syncthreads();
        }
        RunSum64 P = tid ? rs64_combine(acc, sh[tid - 1]) : acc;
        if (t < t1)
            carry[t] = (t > t0 && P.len > 0 && P.last == S.first) ? (uint32_t)(P.trail % 255u) : 0u;
        acc = rs64_combine(acc, sh[255]);
        __syncthreads();
    }
}

__device__ __forceinline__ uint32_t rle_w(uint32_t t) { return t < 3 ? 1u : (t == 3 ? 2u : 0u); }

__global__ void __launch_bounds__(256) k_rle_pos(const uint8_t* __restrict__ text, const TileDesc* __restrict__ tiles,
                                                  const uint32_t* __restrict__ carry, uint8_t* __restrict__ tpos,
                                                  uint32_t* __restrict__ tile_w)
{
    __shared__ RunSum sh[256];
    __shared__ uint32_t inc[256];
    __shared__ uint32_t wsh[5];
    TileDesc d = tiles[blockIdx.x];
    int off = threadIdx.x * 16;
    int cnt = (int)d.len - off;
    cnt = cnt < 0 ? 0 : (cnt > 16 ? 16 : cnt);
    const uint8_t* p = text + d.beg + off;
    sh[threadIdx.x] = strip_summary(p, cnt);
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t c = carry[blockIdx.x];
        RunSum acc;
        acc.len = c; acc.trail = c; acc.uni = true;
        acc.first = acc.last = (d.len ? text[d.beg] : -1);
        for (int k = 0; k < 256; ++k) {
            RunSum S = sh[k];
            inc[k] = (acc.len > 0 && S.len > 0 && acc.last == S.first) ? acc.trail : 0;
            acc = rs_combine(acc, S);
        }
    }
    __syncthreads();
    uint32_t run = inc[threadIdx.x];
    uint32_t w = 0;
    int prev = -1;
    for (int k = 0; k < cnt; ++k) {
        int c = p[k];
        if (k > 0) run = (c == prev) ? run + 1 : 0;
        prev = c;
        uint32_t t = run % 255u;
        tpos[d.beg + off + k] = (uint8_t)t;
        w += rle_w(t);
    }
    uint32_t tot;
    (void)block_excl_scan_add<uint32_t>(w, wsh, &tot);
    if (threadIdx.x == 0) tile_w[blockIdx.x] = tot;
}

// RLE1 size prefix (stream-relative) at text position x of stream s
struct WView {
    const uint64_t* tile_wpre;
    const uint8_t* tpos;
    uint64_t beg, end, t0, w0;
    __device__ uint64_t tile_w_at(uint64_t t) const { return tile_wpre[t] - w0; }
};

__global__ void k_stream_w(const uint64_t* __restrict__ seg_tile0, const uint64_t* __restrict__ tile_wpre,
                           uint32_t nstreams, uint64_t* __restrict__ out)
{
    uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s < nstreams) out[s] = tile_wpre[seg_tile0[s + 1]] - tile_wpre[seg_tile0[s]];
}

// one wave per stream: greedy cut (see file header).  Per block: binary search
// of the tile where the RLE1 size crosses nblockMAX, a 64-lane scan of that
// tile's byte weights for the crossing byte q, then a ballot over the next 256
// bytes for the first chunk start p >= q (chunks are at most 255 bytes).
__global__ void __launch_bounds__(64) k_cut(const StreamIn* __restrict__ streams, const uint64_t* __restrict__ seg_tile0,
                                             const uint64_t* __restrict__ tile_wpre, const uint8_t* __restrict__ tpos,
                                             uint32_t nstreams, uint32_t nblock_max, const uint64_t* __restrict__ slot0,
                                             BlockDesc* __restrict__ tmp, uint32_t* __restrict__ nblk)
{
    const uint32_t s = blockIdx.x;
    const int lane = threadIdx.x;
    const uint64_t beg = streams[s].text_off, end = beg + streams[s].text_len;
    const uint64_t t0 = seg_tile0[s], t1 = seg_tile0[s + 1];
    const uint64_t w0 = tile_wpre[t0], wend = tile_wpre[t1] - w0;
    const bool frj = streams[s].final_run_joins != 0;
    uint64_t bs = beg, wbs = 0;
    uint32_t k = 0;
    while (bs < end) {
        const uint64_t target = wbs + nblock_max;
        uint64_t block_end = end, wblock_end = wend;
        if (wend >= target) {
            uint64_t lo = t0 + (bs - beg) / kTB, hi = t1;   // Wstart(lo) <= wbs < target <= Wstart(hi)
            while (hi - lo > 1) {
                uint64_t mid = (lo + hi) >> 1;
                if (tile_wpre[mid] - w0 < target) lo = mid; else hi = mid;
            }
            uint64_t q = 0, Wq = 0;
            for (;;) {   // normally one iteration
                const uint64_t tstart = beg + (lo - t0) * kTB;
                uint64_t tend = tstart + kTB;
                if (tend > end) tend = end;
                const uint64_t y0 = tstart < bs ? bs : tstart;
                const uint64_t W0 = tstart < bs ? wbs : tile_wpre[lo] - w0;
                const uint64_t a = y0 + (uint64_t)lane * 64;
                const uint64_t e = (a + 64 < tend) ? a + 64 : tend;
                uint32_t ssum = 0;
                for (uint64_t y = a; y < e; ++y) ssum += rle_w(tpos[y]);
                const uint32_t incl = wave_incl_scan_add(ssum);
                const uint64_t ball = __ballot(a < tend && W0 + incl >= target);
                if (ball) {
                    const int L = __ffsll((unsigned long long)ball) - 1;
                    uint64_t x = a, Wx = W0 + incl - ssum;
                    if (lane == L) {
                        while (Wx < target) { Wx += rle_w(tpos[x]); ++x; }
                    }
                    q = __shfl(x, L, 64);
                    Wq = __shfl(Wx, L, 64);
                    break;
                }
                ++lo;   // cannot happen when the tile search is exact; stay safe
                if (lo >= t1) { q = end; Wq = wend; break; }
            }
            uint64_t p = end;
            for (int r = 0; r < 4; ++r) {
                const uint64_t pos = q + (uint64_t)r * 64 + lane;
                const uint64_t hit = __ballot(pos < end && tpos[pos] == 0);
                if (hit) { p = q + (uint64_t)r * 64 + (__ffsll((unsigned long long)hit) - 1); break; }
                if (q + (uint64_t)(r + 1) * 64 >= end) break;
            }
            uint32_t part = 0;
            for (int r = 0; r < 4; ++r) {
                const uint64_t pos = q + (uint64_t)r * 64 + lane;
                if (pos < p) part += rle_w(tpos[pos]);
            }
            const uint64_t Wp = Wq + wave_reduce_add(part);
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
    }
    if (lane == 0) nblk[s] = k;
}

__global__ void k_compact_blocks(const BlockDesc* __restrict__ tmp, const uint64_t* __restrict__ slot0,
                                 const uint32_t* __restrict__ nblk, const uint32_t* __restrict__ first,
                                 uint32_t nstreams, BlockDesc* __restrict__ out)
{
    uint32_t s = blockIdx.x;
    if (s >= nstreams) return;
    for (uint32_t k = threadIdx.x; k < nblk[s]; k += blockDim.x) {
        BlockDesc b = tmp[slot0[s] + k];
        b.bits = 0; b.bit_off = 0; b.crc = 0; b.orig_ptr = 0; b.n_in_use = 0; b.n_mtf = 0; b.flags = 0;
        b.n_groups = 0; b.n_sel = 0;
        for (int j = 0; j < 8; ++j) b.in_use[j] = 0;
        out[first[s] + k] = b;
    }
}

// materialise RLE1 block bytes (bz:bzlib.c:224-256) + inUse (bz:bzlib.c:232,247)
__global__ void __launch_bounds__(256) k_rle_emit(const uint8_t* __restrict__ text, const TileDesc* __restrict__ tiles,
                                                   const uint64_t* __restrict__ tile_wpre,
                                                   const uint64_t* __restrict__ seg_tile0,
                                                   const uint8_t* __restrict__ tpos, const StreamIn* __restrict__ streams,
                                                   const uint32_t* __restrict__ sfirst, const uint32_t* __restrict__ snblk,
                                                   BlockDesc* __restrict__ blocks, uint8_t* __restrict__ blk,
                                                   uint64_t stride)
{
    __shared__ uint32_t used[2][8];
    __shared__ uint32_t wsh[5];
    __shared__ uint32_t bsel;
    TileDesc d = tiles[blockIdx.x];
    const uint32_t s = d.stream;
    const uint64_t send = streams[s].text_off + streams[s].text_len;
    if (threadIdx.x < 16) used[threadIdx.x >> 3][threadIdx.x & 7] = 0;
    if (threadIdx.x == 0) {   // block holding the tile's first byte
        uint32_t lo = sfirst[s], hi = sfirst[s] + snblk[s];
        while (hi - lo > 1) {
            uint32_t mid = (lo + hi) >> 1;
            if (blocks[mid].in_beg <= d.beg) lo = mid; else hi = mid;
        }
        bsel = lo;
    }
    int off = threadIdx.x * 16;
    int cnt = (int)d.len - off;
    cnt = cnt < 0 ? 0 : (cnt > 16 ? 16 : cnt);
    uint32_t w = 0;
    for (int k = 0; k < cnt; ++k) w += rle_w(tpos[d.beg + off + k]);
    uint32_t pre = block_excl_scan_add<uint32_t>(w, wsh, (uint32_t*)nullptr);   // contains __syncthreads
    const uint32_t b0 = bsel;
    const uint32_t bl = sfirst[s] + snblk[s];
    uint64_t W = tile_wpre[blockIdx.x] - tile_wpre[seg_tile0[s]] + pre;
    uint32_t b = b0;
    uint64_t bend = blocks[b].in_end, wb = blocks[b].w_beg;
    for (int k = 0; k < cnt; ++k) {
        uint64_t i = d.beg + off + k;
        while (i >= bend && b + 1 < bl) { ++b; bend = blocks[b].in_end; wb = blocks[b].w_beg; }
        uint32_t t = tpos[i];
        uint8_t c = text[i];
        uint8_t* o = blk + (uint64_t)b * stride + (W - wb);
        int slot = (b == b0) ? 0 : 1;
        if (t < 3) {
            o[0] = c;
            if (t == 0) atomicOr(&used[slot][c >> 5], 1u << (c & 31));
        } else if (t == 3) {
            uint64_t j = i + 1;
            while (j < send && tpos[j] != 0) ++j;
            uint32_t L = (uint32_t)(j - i) + 3;
            uint8_t cnt_byte = (uint8_t)(L - 4);
            o[0] = c;
            o[1] = cnt_byte;
            atomicOr(&used[slot][cnt_byte >> 5], 1u << (cnt_byte & 31));
        }
        W += rle_w(t);
    }
    __syncthreads();
    if (threadIdx.x < 16) {
        int slot = threadIdx.x >> 3, j = threadIdx.x & 7;
        uint32_t bb = b0 + slot;
        if (used[slot][j] && bb < bl) atomicOr(&blocks[bb].in_use[j], used[slot][j]);
    }
}

// CRC-32/BZIP2 of [in_beg, in_end) per block; one 256-thread workgroup per block.
// R(A||B) = R(A)*x^(8|B|) + R(B) (mod P); crc = ~(0xffffffff*x^(8n) + R(all)).
__global__ void __launch_bounds__(256) k_block_crc(const uint8_t* __restrict__ text, BlockDesc* __restrict__ blocks)
{
    __shared__ uint32_t tab[256];
    __shared__ uint32_t rr[256];
    __shared__ uint32_t ll[256];
    tab[threadIdx.x] = c_crc_tab[threadIdx.x];
    const BlockDesc bd = blocks[blockIdx.x];
    const uint64_t beg = bd.in_beg, end = bd.in_end;
    __syncthreads();
    uint32_t acc = 0;   // raw register over processed prefix
    for (uint64_t c0 = beg; c0 < end; c0 += 4096) {
        uint64_t a = c0 + threadIdx.x * 16;
        uint64_t e = a + 16;
        if (e > end) e = end;
        uint32_t r = 0, n = 0;
        for (uint64_t i = a; i < e; ++i) { r = (r << 8) ^ tab[(r >> 24) ^ text[i]]; ++n; }
        rr[threadIdx.x] = r;
        ll[threadIdx.x] = (a < end) ? n : 0;
        __syncthreads();
        for (int step = 1; step < 256; step <<= 1) {
            if ((threadIdx.x & (2 * step - 1)) == 0) {
                uint32_t j = threadIdx.x + step;
                uint32_t lb = ll[j];
                if (lb) {
                    uint32_t m = (lb == (uint32_t)(16 * step)) ? c_pow8[4 + __builtin_ctz(step)] : xpow8(lb);
                    rr[threadIdx.x] = mulmod(rr[threadIdx.x], m) ^ rr[j];
                    ll[threadIdx.x] += lb;
                }
            }
            __syncthreads();
        }
        if (threadIdx.x == 0) {
            uint32_t lc = ll[0];
            uint32_t m = (lc == 4096u) ? c_pow8[12] : xpow8(lc);
            acc = mulmod(acc, m) ^ rr[0];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        uint32_t m = xpow8(end - beg);
        blocks[blockIdx.x].crc = ~(mulmod(0xffffffffu, m) ^ acc);
    }
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
    hipLaunchKernelGGL(k_rle_sum, dim3((unsigned)ntiles), dim3(256), 0, st, text, tiles, sums);
}
void rle_carry(const uint64_t* tile0, uint32_t ns, const TileSum* sums, uint32_t* carry, hipStream_t st)
{
    hipLaunchKernelGGL(k_rle_carry, dim3(ns), dim3(256), 0, st, tile0, ns, sums, carry);
}
void rle_pos(const uint8_t* text, const TileDesc* tiles, uint64_t ntiles, const uint32_t* carry, uint8_t* tpos,
             uint32_t* tile_w, hipStream_t st)
{
    hipLaunchKernelGGL(k_rle_pos, dim3((unsigned)ntiles), dim3(256), 0, st, text, tiles, carry, tpos, tile_w);
}
void rle_stream_w(const uint64_t* tile0, const uint64_t* wpre, uint32_t ns, uint64_t* out, hipStream_t st)
{
    hipLaunchKernelGGL(k_stream_w, dim3(g1(ns, 64)), dim3(64), 0, st, tile0, wpre, ns, out);
}
void rle_cut(const StreamIn* streams, const uint64_t* tile0, const uint64_t* wpre, const uint8_t* tpos, uint32_t ns,
             uint32_t nblock_max, const uint64_t* slot0, BlockDesc* tmp, uint32_t* nblk, hipStream_t st)
{
    hipLaunchKernelGGL(k_cut, dim3(ns), dim3(64), 0, st, streams, tile0, wpre, tpos, ns, nblock_max, slot0, tmp,
                       nblk);
}
void rle_compact(const BlockDesc* tmp, const uint64_t* slot0, const uint32_t* nblk, const uint32_t* first, uint32_t ns,
                 BlockDesc* out, hipStream_t st)
{
    hipLaunchKernelGGL(k_compact_blocks, dim3(ns), dim3(256), 0, st, tmp, slot0, nblk, first, ns, out);
}
void rle_emit(const uint8_t* text, const TileDesc* tiles, uint64_t ntiles, const uint64_t* wpre, const uint64_t* tile0,
              const uint8_t* tpos, const StreamIn* streams, const uint32_t* first, const uint32_t* nblk,
              BlockDesc* blocks, uint8_t* blk, uint64_t stride, hipStream_t st)
{
    hipLaunchKernelGGL(k_rle_emit, dim3((unsigned)ntiles), dim3(256), 0, st, text, tiles, wpre, tile0, tpos, streams,
                       first, nblk, blocks, blk, stride);
}
void rle_crc(const uint8_t* text, BlockDesc* blocks, uint32_t nb, hipStream_t st)
{
    if (nb) hipLaunchKernelGGL(k_block_crc, dim3(nb), dim3(256), 0, st, text, blocks);
}

}  // namespace bz
