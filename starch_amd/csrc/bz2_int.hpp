// starch_amd/csrc/bz2_int.hpp -- internal types shared by the bzip2 stage files.
#pragma once
#include "bz2.hpp"

namespace bz {

constexpr int kTB = 4096;             // tile bytes for the RLE1 passes

struct TileDesc {                     // a <= 4 KiB slice of one stream
    uint64_t beg;
    uint32_t len;
    uint32_t stream;
    uint32_t first;
    uint32_t pad;
};

struct TileSum {                      // run summary of a tile
    uint32_t len, trail;
    uint8_t first, last, uni, pad;
    uint32_t lead;                    // bytes before its first change (the run it continues)
    uint32_t wrest;                   // RLE1 size of the bytes from its first change on
};

struct Tables {                       // per-block Huffman state (bz:compress.c:238-598)
    uint8_t len[6][258];
    uint8_t pad[4];
    uint32_t code[6][258];
    uint32_t freq[258];               // mtfFreq
    uint32_t pad2[2];
};

static inline uint32_t host_mulmod(uint32_t a, uint32_t b)
{
    uint32_t r = 0;
    for (int i = 31; i >= 0; --i) {
        r = (r & 0x80000000u) ? ((r << 1) ^ 0x04c11db7u) : (r << 1);
        if ((b >> i) & 1u) r ^= a;
    }
    return r;
}

// ---- per-XCD work queues (placement is a speed matter only) ----
// A persistent workgroup reads the XCD it runs on and takes work from that
// XCD's queue first, then steals from the others, so every queue drains
// whatever the dispatcher does; work whose data should share an L2 (one
// bzip2 block) is put in one queue.  MI355X_MICROARCH.md "Workgroup dispatch".
__device__ __forceinline__ uint32_t xcc_id()
{
    return (uint32_t)__builtin_amdgcn_s_getreg(20 | (0 << 6) | (3 << 11)) & 7u;   // hwreg(HW_REG_XCC_ID, 0, 4)
}

// Queue y's head word sits at head[y * XQ_STRIDE]: one 128-B line per head, so
// the XCDs' atomics never share a line.
constexpr uint32_t XQ_STRIDE = 32;

// qsize[y] = items in queue y; returns (y << 28) | index, or ~0u when all are
// drained.  Called by one lane.
__device__ __forceinline__ uint32_t xq_pop(uint32_t* head, const uint32_t* qsize, uint32_t x)
{
    for (uint32_t t = 0; t < 8; ++t) {
        const uint32_t y = (x + t) & 7u;
        const uint32_t sz = qsize[y];
        if (__hip_atomic_load(head + y * XQ_STRIDE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= sz) continue;
        const uint32_t i = atomicAdd(head + y * XQ_STRIDE, 1u);
        if (i < sz) return (y << 28) | i;
    }
    return 0xFFFFFFFFu;
}

// Chunked pop: up to k consecutive items; cnt = how many.  Called by one lane.
__device__ __forceinline__ uint32_t xq_pop_n(uint32_t* head, const uint32_t* qsize, uint32_t x, uint32_t k,
                                             uint32_t& cnt)
{
    for (uint32_t t = 0; t < 8; ++t) {
        const uint32_t y = (x + t) & 7u;
        const uint32_t sz = qsize[y];
        if (__hip_atomic_load(head + y * XQ_STRIDE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= sz) continue;
        const uint32_t i = atomicAdd(head + y * XQ_STRIDE, k);
        if (i < sz) {
            cnt = sz - i < k ? sz - i : k;
            return (y << 28) | i;
        }
    }
    cnt = 0;
    return 0xFFFFFFFFu;
}

// A wave's walk over per-XCD queues of a segmented list (seg[y] = start of
// queue y in the list): items come in list order per XCD, so the waves of one
// XCD stay on neighbouring items (one block's data in that XCD's L2) however
// uneven the items' costs.  next() is wave-uniform; ~0u when drained.
template <uint32_t K>
struct WaveQueue {
    uint32_t a = 0, r = 0;
    __device__ __forceinline__ uint32_t next(uint32_t* head, const uint32_t* qsize, const uint32_t* seg, uint32_t x)
    {
        if (r == 0) {
            uint32_t j = 0, cnt = 0;
            if ((threadIdx.x & 63) == 0) j = xq_pop_n(head, qsize, x, K, cnt);
            j = (uint32_t)__shfl((int)j, 0, 64);
            cnt = (uint32_t)__shfl((int)cnt, 0, 64);
            if (j == 0xFFFFFFFFu) return 0xFFFFFFFFu;
            a = seg[j >> 28] + (j & 0x0FFFFFFFu);
            r = cnt;
        }
        --r;
        return a++;
    }
};

// ---- move-to-front on a list of <= 16 symbols kept as nibbles of a u64 ----
struct NibState {          // transform L -> list ++ (L \ set)
    uint64_t list;         // nibble i = i-th symbol
    uint32_t set;          // 16-bit symbol set
    uint32_t cnt;
};

__device__ __forceinline__ NibState nib_compose(const NibState& c, const NibState& d)   // apply c, then d
{
    NibState r;
    r.list = d.list;
    r.cnt = d.cnt;
    for (uint32_t i = 0; i < c.cnt; ++i) {
        uint32_t sym = (uint32_t)(c.list >> (4 * i)) & 15u;
        if (!((d.set >> sym) & 1u)) { r.list |= (uint64_t)sym << (4 * r.cnt); ++r.cnt; }
    }
    r.set = c.set | d.set;
    return r;
}

__device__ __forceinline__ uint64_t lowmask4(uint32_t k)   // k nibbles
{
    return k >= 16 ? ~0ull : ((1ull << (4 * k)) - 1ull);
}

// one MTF step on the nibble list; returns the index of s.  s must be in the
// list (unused high nibbles are 0: the first match is the real position of 0).
// Zero-nibble search on 32-bit halves, then a bit-select moves nibbles 0..k-1
// up by one and puts s in front.
__device__ __forceinline__ uint32_t nib_mtf(uint64_t& L, uint32_t s)
{
    const uint32_t pat = s * 0x11111111u;
    uint32_t xl = (uint32_t)L ^ pat, xh = (uint32_t)(L >> 32) ^ pat;
    xl |= xl >> 1;
    xl |= xl >> 2;
    xh |= xh >> 1;
    xh |= xh >> 2;
    const uint32_t zl = ~xl & 0x11111111u, zh = ~xh & 0x11111111u;
    const uint32_t k = zl ? ((uint32_t)__builtin_ctz(zl) >> 2) : 8u + ((uint32_t)__builtin_ctz(zh) >> 2);
    const uint64_t m = (k >= 15u) ? ~0ull : ((1ull << (4u * k + 4u)) - 1ull);
    L = (((L << 4) | (uint64_t)s) & m) | (L & ~m);
    return k;
}

void upload_crc_constants();

// bz2_rle.hip launch wrappers
void rle_tiles(const uint64_t* tile0, const StreamIn* streams, uint32_t ns, uint64_t ntiles, TileDesc* tiles,
               hipStream_t st);
void rle_sum(const uint8_t* text, const TileDesc* tiles, uint64_t ntiles, TileSum* sums, hipStream_t st);
void rle_carry(const uint64_t* tile0, uint32_t ns, const TileSum* sums, uint32_t* carry, uint32_t* tile_w,
               hipStream_t st);
void rle_stream_w(const uint64_t* tile0, const uint64_t* wpre, uint32_t ns, uint64_t* out, hipStream_t st);
// tab: rle_cut_tab_bytes(nslots) of scratch for the cut tables (k_cut_tab);
// max_slots: the most block slots of one stream
uint64_t rle_cut_tab_bytes(uint64_t nslots);
void rle_cut(const StreamIn* streams, const uint64_t* tile0, const uint64_t* wpre, const uint8_t* text,
             const uint32_t* carry, uint32_t ns, uint32_t nblock_max, const uint64_t* slot0, uint64_t nslots,
             uint64_t max_slots, void* tab, BlockDesc* tmp, uint32_t* nblk, hipStream_t st);
void rle_compact(const BlockDesc* tmp, const uint64_t* slot0, const uint32_t* nblk, const uint32_t* first, uint32_t ns,
                 BlockDesc* out, const StreamIn* streams, const uint64_t* tile0, uint32_t* tile_block, hipStream_t st);
void rle_emit(const uint8_t* text, const TileDesc* tiles, uint64_t ntiles, const uint64_t* wpre, const uint64_t* tile0,
              const uint32_t* carry, const StreamIn* streams, const uint32_t* first, const uint32_t* nblk,
              const uint32_t* tile_block, BlockDesc* blocks, uint8_t* blk, uint64_t stride, hipStream_t st);
constexpr uint32_t kCrcMaxChunks = 128;       // per block (k_crc_chunks)
void rle_block_first(const uint32_t* nblk, uint32_t ns, uint32_t* first, uint32_t* total, hipStream_t st);
// nb_max: grid bound; nb_dev (nullable): the device's block count (blocks past it are skipped)
void rle_crc(const uint8_t* text, BlockDesc* blocks, uint32_t nb_max, const uint32_t* nb_dev, uint32_t* creg,
             hipStream_t st);

}  // namespace bz
