// starch_amd/csrc/bz2_emit.hip -- bit emission straight into the archive.
//
// Restates the writing half of sendMTFValues / BZ2_compressBlock
// (bz:compress.c:494-598, 602-667) and the MSB-first bit writer
// (bz:compress.c:37-97).  Every block already knows its absolute bit offset
// (blocks are bit-concatenated inside a stream, bz:compress.c:609), so all
// 50-symbol groups of all blocks are written in parallel: a lane owns a bit
// range, plain-stores the 32-bit big-endian words fully inside it and ORs
// (atomically) the two words it may share with its neighbours.  The output
// buffer is zeroed beforehand.
#include "bz2_bwt.hpp"

namespace bz {

struct BitOut {
    uint32_t* w;
    uint64_t word;
    uint64_t acc;
    int nb;
    bool first;
    __device__ void init(uint32_t* out, uint64_t pos)
    {
        w = out;
        word = pos >> 5;
        nb = (int)(pos & 31);
        acc = 0;
        first = nb != 0;
    }
    __device__ __forceinline__ void flush_word(uint32_t v)
    {
        uint32_t be = __builtin_bswap32(v);
        if (first) atomicOr(&w[word], be); else w[word] = be;
        first = false;
        ++word;
    }
    __device__ __forceinline__ void put(int len, uint32_t code)
    {
        acc = (acc << len) | (uint64_t)code;
        nb += len;
        if (nb >= 32) {
            nb -= 32;
            flush_word((uint32_t)(acc >> nb));
            acc &= nb ? ((1ull << nb) - 1ull) : 0ull;
        }
    }
    __device__ void finish()
    {
        if (nb > 0) atomicOr(&w[word], __builtin_bswap32((uint32_t)(acc << (32 - nb))));
        nb = 0;
    }
};

constexpr int ET = 1024;

// One workgroup per block.  Thread 0 writes the fixed header (magic, CRC,
// origPtr, inUse map, nGroups, nSelectors); the selectors' unary MTF codes
// are written in parallel (contiguous selector ranges per thread, bit offsets
// by a block scan); thread 0 writes the delta-coded lengths; then the bit
// offsets of the data groups (k_emit_data writes them).
__global__ void __launch_bounds__(ET) k_emit_block(const BlockDesc* __restrict__ blocks,
                                                    const uint16_t* __restrict__ mtfv_all, uint64_t mtf_stride,
                                                    const Tables* __restrict__ tabs, const uint8_t* __restrict__ sel_all,
                                                    const uint32_t* __restrict__ gbits_all, uint32_t* __restrict__ gpre_all,
                                                    const uint32_t* __restrict__ src_of, uint32_t* __restrict__ out32)
{
    __shared__ uint8_t len[6][258];
    __shared__ uint32_t code[6][258];
    __shared__ uint32_t scan_sh[ET / 64 + 1];
    const int tid = threadIdx.x;
    const uint32_t b = blockIdx.x;
    const uint32_t d = src_of ? src_of[b] : b;          // data index (bz2_dedupe.hip)
    const BlockDesc bd = blocks[b];
    const int alpha = (int)bd.n_in_use + 2;
    const int ng = (int)bd.n_groups;
    for (int i = tid; i < 6 * 258; i += ET) {
        int t = i / 258, v = i % 258;
        if (t < ng && v < alpha) { len[t][v] = tabs[d].len[t][v]; code[t][v] = tabs[d].code[t][v]; }
    }
    const uint8_t* sel = sel_all + (uint64_t)d * (2 * kMaxSelectors);
    const uint8_t* selmtf = sel + kMaxSelectors;
    const uint32_t* gbits = gbits_all + (uint64_t)d * kMaxSelectors;

    uint32_t used16 = 0;
    for (int i = 0; i < 16; ++i) {
        const uint32_t w = bd.in_use[i >> 1];
        const uint32_t half = (i & 1) ? (w >> 16) : (w & 0xffffu);
        if (half) used16 |= 1u << (15 - i);
    }
    const uint64_t sel0 = bd.bit_off + 48 + 32 + 1 + 24 + 16 + 16ull * __popc(used16) + 3 + 15;
    if (tid == 0) {   // block header, mapping table, counts (bz:compress.c:496-544, 611-621)
        BitOut o;
        o.init(out32, bd.bit_off);
        o.put(24, 0x314159u);
        o.put(24, 0x265359u);
        o.put(32, bd.crc);
        o.put(1, 0);
        o.put(24, bd.orig_ptr);
        o.put(16, used16);
        for (int i = 0; i < 16; ++i) {
            if (!(used16 & (1u << (15 - i)))) continue;
            const uint32_t w = bd.in_use[i >> 1];
            const uint32_t half = (i & 1) ? (w >> 16) : (w & 0xffffu);
            uint32_t bits = 0;
            for (int j = 0; j < 16; ++j) if (half & (1u << j)) bits |= 1u << (15 - j);
            o.put(16, bits);
        }
        o.put(3, (uint32_t)ng);
        o.put(15, bd.n_sel);
        o.finish();
    }
    // selectors, MTF-coded in unary (bz:compress.c:546-556)
    const uint32_t per = (bd.n_sel + ET - 1) / ET;
    const uint32_t sa = tid * per, se = sa + per < bd.n_sel ? sa + per : bd.n_sel;
    uint32_t sb = 0;
    for (uint32_t i = sa; i < se; ++i) sb += selmtf[i] + 1u;
    uint32_t stot;
    const uint32_t spre = block_excl_scan_add<uint32_t>(sb, scan_sh, &stot);
    if (sa < se) {
        BitOut o;
        o.init(out32, sel0 + spre);
        for (uint32_t i = sa; i < se; ++i) {
            const uint32_t j = selmtf[i];
            o.put((int)j + 1, ((1u << j) - 1u) << 1);
        }
        o.finish();
    }
    if (tid == 0) {   // coding tables, delta-coded lengths (bz:compress.c:558-575)
        BitOut o;
        o.init(out32, sel0 + stot);
        for (int t = 0; t < ng; ++t) {
            int cur = len[t][0];
            o.put(5, (uint32_t)cur);
            for (int i = 0; i < alpha; ++i) {
                while (cur < len[t][i]) { o.put(2, 2); ++cur; }
                while (cur > len[t][i]) { o.put(2, 3); --cur; }
                o.put(1, 0);
            }
        }
        o.finish();
    }
    // bit offsets of the coded 50-symbol groups: exclusive scan of their sizes
    // (k_emit_data writes the groups themselves, flat over all blocks)
    uint32_t* gpre = gpre_all + (uint64_t)b * kMaxSelectors;
    uint32_t run = 0;
    for (uint32_t g0 = 0; g0 < bd.n_sel; g0 += ET) {
        const uint32_t g = g0 + tid;
        const uint32_t gb = (g < bd.n_sel) ? gbits[g] : 0u;
        uint32_t tot;
        const uint32_t pre = block_excl_scan_add<uint32_t>(gb, scan_sh, &tot);
        if (g < bd.n_sel) gpre[g] = run + pre;
        run += tot;
    }
}

// Coded data: one 50-symbol group per lane, over (block, 256-group tile).
// The tile's MTF values are staged in LDS with coalesced loads; each lane
// codes its group (lengths and codes packed len << 24 | code, one LDS read
// per symbol) into an LDS image of the tile's output words (LDS atomic ORs:
// neighbouring groups share words), and the image is stored with coalesced
// writes -- plain stores inside, global atomic ORs for the two edge words
// shared with the neighbouring tiles / the block header.  A tile whose output
// does not fit the image writes straight to global memory (BitOut).
constexpr int DT = 256;
constexpr uint32_t EI_WORDS = DT * 50 / 2;       // staged MTF values (u16 pairs)
constexpr uint32_t EO_WORDS = 2048;              // staged output words

struct BitOutL {                                 // MSB-first bits into LDS words [w0, ...)
    uint32_t* ob;
    uint32_t w0, word;
    uint64_t acc;
    int nb;
    __device__ __forceinline__ void init(uint32_t* o, uint32_t wbase, uint64_t pos)
    {
        ob = o;
        w0 = wbase;
        word = (uint32_t)(pos >> 5);
        nb = (int)(pos & 31);
        acc = 0;
    }
    __device__ __forceinline__ void put(int len, uint32_t code)
    {
        acc = (acc << len) | (uint64_t)code;
        nb += len;
        if (nb >= 32) {
            nb -= 32;
            atomicOr(&ob[word - w0], (uint32_t)(acc >> nb));
            ++word;
            acc &= nb ? ((1ull << nb) - 1ull) : 0ull;
        }
    }
    __device__ __forceinline__ void finish()
    {
        if (nb > 0) atomicOr(&ob[word - w0], (uint32_t)(acc << (32 - nb)));
    }
};

__global__ void __launch_bounds__(DT) k_emit_data(const BlockDesc* __restrict__ blocks,
                                                  const uint16_t* __restrict__ mtfv_all, uint64_t mtf_stride,
                                                  const Tables* __restrict__ tabs, const uint8_t* __restrict__ sel_all,
                                                  const uint32_t* __restrict__ gbits_all,
                                                  const uint32_t* __restrict__ gpre_all,
                                                  const uint32_t* __restrict__ src_of, uint32_t* __restrict__ out32)
{
    __shared__ uint32_t lc[6][258];
    __shared__ uint32_t mv[EI_WORDS];
    __shared__ uint32_t ob[EO_WORDS];
    const uint32_t b = blockIdx.y;
    const uint32_t n_sel = blocks[b].n_sel;
    const uint32_t d = src_of ? src_of[b] : b;          // data index (bz2_dedupe.hip)
    const uint32_t g0 = blockIdx.x * DT;
    if (g0 >= n_sel) return;                                // uniform
    const int tid = threadIdx.x;
    const uint32_t gcnt = n_sel - g0 < (uint32_t)DT ? n_sel - g0 : (uint32_t)DT;
    const int alpha = (int)blocks[b].n_in_use + 2;
    const int ng = (int)blocks[b].n_groups;
    for (int i = tid; i < ng * 258; i += DT) {
        const int t = i / 258, v = i % 258;
        if (v < alpha) lc[t][v] = ((uint32_t)tabs[d].len[t][v] << 24) | tabs[d].code[t][v];
    }
    const uint32_t n_mtf = blocks[b].n_mtf;
    const uint32_t s0 = g0 * 50;
    const uint32_t s1 = (g0 + gcnt) * 50 < n_mtf ? (g0 + gcnt) * 50 : n_mtf;
    // alphabets <= 32 store their MTF values as bytes (bz2_mtf.hip Out8), larger ones as u16
    const bool v8 = alpha <= 32;                            // uniform
    const uint32_t nwi = v8 ? (s1 - s0 + 3) / 4 : (s1 - s0 + 1) / 2;
    const uint32_t* src = v8 ? reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(mtfv_all + (uint64_t)d * mtf_stride) + s0)
                             : reinterpret_cast<const uint32_t*>(mtfv_all + (uint64_t)d * mtf_stride + s0);
    for (uint32_t i = tid; i < nwi; i += DT) mv[i] = src[i];
    const uint32_t* gpre = gpre_all + (uint64_t)b * kMaxSelectors;
    const uint64_t base = blocks[b].bit_off + blocks[b].hdr_bits;
    const uint64_t tb0 = base + gpre[g0];
    const uint64_t tb1 = base + gpre[g0 + gcnt - 1] + gbits_all[(uint64_t)d * kMaxSelectors + g0 + gcnt - 1];
    const uint32_t w0 = (uint32_t)(tb0 >> 5), nwo = (uint32_t)((tb1 + 31) >> 5) - w0;
    const bool staged = nwo <= EO_WORDS;                    // uniform
    if (staged) for (uint32_t i = tid; i < nwo; i += DT) ob[i] = 0;
    __syncthreads();
    if ((uint32_t)tid < gcnt) {
        const uint32_t g = g0 + tid;
        const uint32_t gs = g * 50;
        const uint32_t ge = gs + 50 < n_mtf ? gs + 50 : n_mtf;
        const uint32_t* row = lc[sel_all[(uint64_t)d * (2 * kMaxSelectors) + g]];
        const uint32_t* m = mv + (gs - s0) / 2;                // gs, s0 even
        auto code_group = [&](auto& o) {
            if (v8) {   // bytes: the group starts at an even byte (50 g); 4 per LDS word after the first 2
                uint32_t i = gs, off = gs - s0;
                auto sym = [&](uint32_t v) {
                    const uint32_t c = row[v];
                    o.put((int)(c >> 24), c & 0xFFFFFFu);
                };
                if (off & 2u) {
                    const uint32_t w = mv[off >> 2] >> 16;
                    sym(w & 0xffu);
                    if (i + 1 < ge) sym(w >> 8);
                    i += 2;
                    off += 2;
                }
                for (; i < ge; i += 4, off += 4) {
                    const uint32_t w = mv[off >> 2];
                    sym(w & 0xffu);
                    if (i + 1 < ge) sym((w >> 8) & 0xffu);
                    if (i + 2 < ge) sym((w >> 16) & 0xffu);
                    if (i + 3 < ge) sym(w >> 24);
                }
            } else {
                for (uint32_t i = gs; i < ge; i += 2) {
                    const uint32_t w = m[(i - gs) >> 1];
                    const uint32_t c0 = row[w & 0xffffu];
                    o.put((int)(c0 >> 24), c0 & 0xFFFFFFu);
                    if (i + 1 < ge) {
                        const uint32_t c1 = row[w >> 16];
                        o.put((int)(c1 >> 24), c1 & 0xFFFFFFu);
                    }
                }
            }
            o.finish();
        };
        if (staged) {
            BitOutL o;
            o.init(ob, w0, base + gpre[g]);
            code_group(o);
        } else {
            BitOut o;
            o.init(out32, base + gpre[g]);
            code_group(o);
        }
    }
    if (!staged) return;
    __syncthreads();
    for (uint32_t i = tid; i < nwo; i += DT) {
        const uint32_t v = __builtin_bswap32(ob[i]);
        if (i == 0 || i + 1 == nwo) atomicOr(&out32[w0 + i], v);
        else out32[w0 + i] = v;
    }
}

// stream header "BZh"+level and trailer (end magic, combined CRC, byte pad)
__global__ void k_stream_frame(const StreamOut* __restrict__ souts, const BlockDesc* __restrict__ blocks,
                               uint32_t nstreams, int bs100k, uint64_t out_base, uint32_t* __restrict__ out32)
{
    uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= nstreams) return;
    const StreamOut so = souts[s];
    uint64_t pos = (out_base + so.out_off) * 8 + ((so.frame >> 8) & 7u);   // a piece may start mid-byte
    BitOut o;
    if (so.frame & 1u) {
        o.init(out32, pos);
        o.put(8, 'B');
        o.put(8, 'Z');
        o.put(8, 'h');
        o.put(8, (uint32_t)('0' + bs100k));
        o.finish();
        pos += 32;
    }
    if (!(so.frame & 2u)) return;                  // an open piece: the stream goes on
    uint32_t comb = so.combined_crc;               // blocks of earlier pieces
    uint64_t end = pos;
    for (uint32_t k = 0; k < so.n_blocks; ++k) {
        const BlockDesc& bd = blocks[so.first_block + k];
        comb = ((comb << 1) | (comb >> 31)) ^ bd.crc;                   // bz:compress.c:606-608
        end += bd.bits;
    }
    o.init(out32, end);
    o.put(24, 0x177245u);
    o.put(24, 0x385090u);
    o.put(32, comb);
    o.finish();
}

void launch_emit_blocks(const BlockDesc* blocks, uint32_t nb, const uint16_t* mtfv, uint64_t mtf_stride,
                        const Tables* tabs, const uint8_t* sel, const uint32_t* gbits, uint32_t* gpre,
                        const uint32_t* src_of, uint32_t* out32, hipStream_t st)
{
    if (!nb) return;
    hipLaunchKernelGGL(k_emit_block, dim3(nb), dim3(ET), 0, st, blocks, mtfv, mtf_stride, tabs, sel, gbits, gpre,
                       src_of, out32);
    hipLaunchKernelGGL(k_emit_data, dim3((kMaxSelectors + DT - 1) / DT, nb), dim3(DT), 0, st, blocks, mtfv,
                       mtf_stride, tabs, sel, gbits, gpre, src_of, out32);
    HIP_CHECK(hipGetLastError());
}

void launch_stream_frame(const StreamOut* souts, const BlockDesc* blocks, uint32_t nstreams, int bs100k,
                         uint64_t out_base, uint32_t* out32, hipStream_t st)
{
    if (!nstreams) return;
    hipLaunchKernelGGL(k_stream_frame, dim3((nstreams + 63) / 64), dim3(64), 0, st, souts, blocks, nstreams, bs100k,
                       out_base, out32);
    HIP_CHECK(hipGetLastError());
}

}  // namespace bz
