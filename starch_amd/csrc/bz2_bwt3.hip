// starch_amd/csrc/bz2_bwt3.hip -- block sort v3 (the default): a batch-wide
// segmented sort of every rotation of every block, then refinement of the
// rotations whose packed prefix keys tie.
//
// Contract (same as k_bwt, bz2_bwt.hip): SA = the exact sorted order of the
// cyclic rotations of every non-periodic block (BZ2_blockSort's ptr[],
// bz:blocksort.c:1031-1089; unique because all rotations differ), origPtr =
// rank of rotation 0; periodic blocks are flagged (flags bit0) for
// k_fallback_exact, which reproduces fallbackSort's tie order.
//
// Why this shape: a 900 KB transformed-BED block almost never needs more than
// its packed D-symbol prefix (D = 64 / B symbols of B = ceil(log2 nInUse)
// bits in a u64 key; 16 for BED3 text): measured on cfg2 blocks, ~5 tied
// pairs per 900k rotations; cfg4 (narrowPeak) ~0.8 %.  So the work is a
// segmented sort of (block, 64-bit key) pairs, done for ALL blocks of a batch
// at once:
//
//   k3_pss      packed symbol stream (PSS) of every block: its symbols as
//               B-bit fields, MSB first, in u64 words, wrapped past the end;
//               the key of rotation r is bits [rB, rB+KB) -- two word loads
//               and a shift, so keys are never stored
//   k3_hist     per 32k-rotation tile: 4096-bucket histogram of the top 12 bits
//   k3_scan     per block: bucket starts, per-tile cursors, size-class lists
//   k3_scatter  rotations -> bucket order in SA.  Persistent, per-XCD queues:
//               each XCD streams ITS blocks one at a time, so the scattered
//               4-B writes of a block meet in that XCD's 4 MB L2
//   k3_bin_*    every work list is binned by block into 8 per-XCD segments
//               (blocks x, x+8, ... in order), so the persistent kernels below
//               touch ~one block's PSS per XCD at a time (L2-resident)
//   k3_part_l   buckets > 4096: MSD partition on the next 8 key bits, repeated
//   k3_sort_w   buckets <= 64: one wave, rank by comparison
//   k3_sort_lds buckets <= 256: one wave; <= 1024/2048/4096: one workgroup;
//               one MSD digit then ranking by comparison (LSD radix when a
//               sub-bucket is large), keys in registers, LDS exchange
//   -- every sort writes SA and lists the groups of equal keys --
//   text rounds a tied group is re-sorted by its NEXT D' = 52/B symbols, read
//               from the PSS at an offset (12 key bits stay free for the packed
//               group index); enough for BED text, where ties are short
//   k3_rk_*     blocks still tied after the text rounds (long repeats,
//               periodic blocks): dense RK = head position of every
//               rotation's group, then prefix doubling --
//   k3_gather   doubling round r: key(q) = RK[(SA[q] + h0*2^(r-1)) mod n] for
//               the tied rotations only (K2); the same kernels re-sort the
//               groups and update RK.  A round in which no group of a block
//               splits proves the block periodic.
//
// Scratch (BwtScratch, per batch slot, stride S elements): SA/V = rotations in
// bucket order (V: partition ping-pong); K = PSS + per-tile cursors (round 0,
// text rounds), key ping-pong while doubling; K2 = doubling keys; RK ranks;
// U = wave-class list; U2/V2 = tie-group lists of consecutive rounds (u64).
#include "bz2_int.hpp"
#include "bz2_bwt.hpp"

#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <type_traits>
#include <vector>

namespace bz {
namespace {

constexpr int PT = 256;                 // hist threads
constexpr int PTILE = 32768;            // rotations per partition tile
constexpr int PDIG = 12;
constexpr int PNB = 1 << PDIG;          // 4096 top-level buckets per block (binary digit)
// Blocks of 17..20 symbols (B = 5: narrowPeak / BED6+ text) take a mixed-radix
// top-level digit instead: their first 3 symbols, s0*nin^2 + s1*nin + s2 <
// 8000, so every bucket shares 15 key bits (the binary digit covers 2.4
// symbols there and leaves buckets ~6x larger).  Batches holding such blocks
// run the top-level kernels with 8192 bins.
constexpr int PNB_WIDE = 8192;
static_assert(PTILE <= 32768 && PNB_WIDE <= 8192, "k3_scatter_lds packs (digit << 15) | rotation-in-tile");
constexpr int MAXT = (900064 + PTILE - 1) / PTILE;   // tiles per block (bs <= 9)
// size classes: W rank-by-compare (one wave), S wave-private LDS sort,
// M1..M3 workgroup LDS sort, L MSD partition
constexpr uint32_t W_MAX = 64, S1_MAX = 128, S_MAX = 256, M0_MAX = 512, M1_MAX = 1024, M2_MAX = 2048, M3_MAX = 4096;
// groups above L_MIN are MSD-partitioned (k3_part_l) instead of sorted whole
#ifndef STARCH_L_MIN
#define STARCH_L_MIN 4096
#endif
constexpr uint32_t L_MIN = STARCH_L_MIN;
constexpr uint32_t GB_MIN = 16384;      // doubling: tie groups above this are gathered by the whole grid
constexpr uint32_t GB_MAXN = 8192;      // (two per block of a 2,048-block batch of near-periodic blocks, and spare)
constexpr uint32_t HG_MIN_PUSH = 32768;  // (= HG_MIN) L groups above it are partitioned by the whole grid
constexpr uint32_t RBITS = 20;          // rank bits (n <= 899,985 < 2^20)
constexpr uint32_t TEXT_ROUNDS = 4;     // max text-extension rounds before doubling

// counters (u32) in the meta buffer
enum { C_W = 0, C_S, C_S2, C_M1, C_M2, C_M3, C_L0, C_L1, C_T0, C_T1, C_TIE_ELEMS, C_ERR, C_TS0, C_TS1, C_H, C_DBG2,
       C_DBGL, C_M0, C_STG, C_STA, C_STW, C_STE, C_STLP, C_STH, C_HG, C_HGC, C_GB, C_LM0, C_LM1, C_N = 30 };

// item = slot[63:52] | start[51:32] | size[31:12] | parity[7] | shift[6:0]
__device__ __forceinline__ uint64_t mk_item(uint32_t slot, uint32_t s, uint32_t m, uint32_t shift, uint32_t par)
{
    return ((uint64_t)slot << 52) | ((uint64_t)s << 32) | ((uint64_t)m << 12) | ((uint64_t)par << 7) | shift;
}
__device__ __forceinline__ uint32_t it_slot(uint64_t x) { return (uint32_t)(x >> 52); }
__device__ __forceinline__ uint32_t it_start(uint64_t x) { return (uint32_t)(x >> 32) & 0xFFFFFu; }
__device__ __forceinline__ uint32_t it_size(uint64_t x) { return (uint32_t)(x >> 12) & 0xFFFFFu; }
__device__ __forceinline__ uint32_t it_par(uint64_t x) { return (uint32_t)(x >> 7) & 1u; }
__device__ __forceinline__ uint32_t it_shift(uint64_t x) { return (uint32_t)x & 127u; }

struct Geo {                   // per block key geometry
    uint32_t B;                // bits per symbol
    uint32_t D;                // symbols per round-0 key (KB = D*B bits)
    uint32_t Dp;               // symbols per text-round key (52/B)
    uint32_t KB;
    uint32_t nin;              // symbols in use
    uint32_t D1;               // top-level digit: 3 = mixed radix over 3 symbols, 0 = top PDIG key bits
    uint32_t SH;               // key bits every top-level bucket shares (3*B or PDIG)
    uint32_t pad;
};

// top-level bucket of a rotation from its 64-bit key window (MSB first)
__device__ __forceinline__ uint32_t top_digit(uint64_t v, const Geo& g)
{
    if (!g.D1) return (uint32_t)(v >> (64 - PDIG));
    const uint32_t mask = (1u << g.B) - 1u;
    const uint32_t s0 = (uint32_t)(v >> (64 - g.B)) & mask;
    const uint32_t s1 = (uint32_t)(v >> (64 - 2 * g.B)) & mask;
    const uint32_t s2 = (uint32_t)(v >> (64 - 3 * g.B)) & mask;
    return (s0 * g.nin + s1) * g.nin + s2;
}

__host__ __device__ constexpr uint64_t pss_words(uint64_t stride) { return stride / 8 + 64; }

struct Lists {
    uint32_t* ctr;          // C_N counters
    uint64_t* w;            // m <= 64
    uint64_t* s;            // m <= 128
    uint64_t* s2;           // m <= 256
    uint64_t* m0;           // m <= 512
    uint64_t* m1;           // m <= 1024
    uint64_t* m2;           // m <= 2048
    uint64_t* m3;           // m <= 4096
    uint64_t* l[2];         // m > 4096 (MSD partition), ping-pong by level
    uint64_t* t[2];         // tie groups, ping-pong by round
    Geo* geo;               // per slot
    uint32_t* gin;          // per slot: groups entering this round
    uint32_t* runs;         // per slot: runs produced this round
    uint32_t* periodic;     // per slot
    uint32_t* rounds;       // per slot: doubling rounds with work
    uint32_t* tied;         // per slot: still tied when doubling starts
    uint64_t* hg;           // huge groups of the current partition level (k3_hg_*), HG_MAXN
    uint32_t* hg_info;      // [HG_MAXN][512]: bin start | final flag; bin totals -> scatter cursors
    uint32_t* hg_pre;       // [HG_MAXN + 1]: chunk prefix of the huge groups (k3_hg_prefix)
    uint64_t* hg_vary;      // [HG_MAXN]: key bits that differ inside the group (OR of key ^ first key)
    uint32_t* hg_flag;      // [HG_MAXN]: HG_SKIP_* / HG_THREE (k3_hg_scan)
    uint32_t* hg_eqlt;      // [HG_MAXN][2]: elements equal to / below the group's first key
    uint32_t* hg_mc;        // [HG_MAXN][6]: in-place three-way: movers to / holes in each part
    uint32_t* hg_rank;      // [HG_MAXN]: in-place three-way: the equal part's rank (HG_KEEP: as it is)
    uint64_t* gb;           // doubling: tie groups gathered by the whole grid (k3_gather_big), GB_MAXN
    uint32_t* gb_h;         // ... their key offset h mod n
};

struct Ctx {
    BlockDesc* blocks;
    uint32_t b0;
    const uint8_t* blkbytes;
    uint64_t stride;        // block byte stride
    BwtScratch scr;
    Lists L;
    uint32_t nb;
    uint32_t lsel;          // L list that part/classify pushes into
    uint32_t tsel;          // tie list the sorts push into
    uint32_t mode;          // 0: SA only (round 0, text rounds); 1: doubling (RK, runs)
    uint32_t keysrc;        // 0: PSS at the text-round offset; 1: keys by group position (kA/kB)
    uint64_t* kA;           // keysrc 1: keys of parity-0 items (round 0: KM0, doubling: K2) ...
    uint64_t* kB;           // ... and of parity-1 items (round 0: KM1, doubling: K)
    uint8_t* lA;            // round 0: last-column symbols by position, parity 0 / 1 (LS0 / LS1);
    uint8_t* lB;            //   null while doubling (then read from the block bytes)
    uint32_t rtext;         // text round (0: round 0)
    uint32_t* qhead;        // 8 queue heads of the current persistent launch
    const uint32_t* qseg;   // 9 per-XCD segment offsets of the current binned list
    uint32_t nbins;         // top-level bins of this batch (PNB or PNB_WIDE)
    uint32_t sdig;          // round 0, first L level: the scatter wrote the L buckets' first digits into LL
};

__device__ __forceinline__ int bits_for3(uint32_t x) { return x ? 32 - __clz(x) : 0; }

__device__ __forceinline__ void wave_sync_lds3()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint64_t lanemask_lt()
{
    const int lane = threadIdx.x & 63;
    return lane ? (~0ull >> (64 - lane)) : 0ull;
}

// Rotation values (SA / V) and last-column bytes stream through the sorts:
// read once per group, written once.  Non-temporal access keeps them from
// evicting the blocks' packed symbol streams (the random key gathers) from
// the XCD's 4 MB L2.  STARCH_NT=0: plain accesses.
#ifndef STARCH_NT
#define STARCH_NT 0   // 1: non-temporal SA/LL/value streams (measured: cfg2 sort 23.5 -> 34.3 ms, cfg4 110 -> 130 ms)
#endif
#ifndef STARCH_W_UNROLL
#define STARCH_W_UNROLL 0   // k3_sort_w's rank loops unrolled by 4 (experiment)
#endif
template <class T>
__device__ __forceinline__ T ld_nt(const T* p)
{
    if constexpr (STARCH_NT != 0) return __builtin_nontemporal_load(p);
    else return *p;
}
template <class T>
__device__ __forceinline__ void st_nt(T* p, T v)
{
    if constexpr (STARCH_NT != 0) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// Append `item` for every lane with pred to list/ctr; one atomic per wave.
// Must be reached by all 64 lanes of the wave.
__device__ __forceinline__ void wave_push(uint32_t* ctr, uint64_t* list, bool pred, uint64_t item)
{
    const uint64_t m = __ballot(pred);
    if (!m) return;
    const int leader = __ffsll((unsigned long long)m) - 1;
    const int lane = threadIdx.x & 63;
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(ctr, (uint32_t)__popcll(m));
    base = __shfl(base, leader, 64);
    if (pred) list[base + __popcll(m & lanemask_lt())] = item;
}

// push a group [s, s+m) of slot with key bits [0, shift) still unsorted to its
// size class list (W, S, S2, M1, M2, M3, L).
// Pushes reserve their slots with LDS atomics and
// the workgroup takes ONE global atomic per class (the class counters are
// shared by every workgroup of the launch; per-wave global atomics on them
// serialise).  Every thread of the workgroup must call it; sh: 16 u32 of LDS.
__device__ __forceinline__ int size_class(uint32_t m)
{
    return m <= W_MAX ? 0 : m <= S1_MAX ? 1 : m <= S_MAX ? 2 : m > L_MIN ? 6 : m <= M0_MAX ? 7 : m <= M1_MAX ? 3 : m <= M2_MAX ? 4
         : m <= M3_MAX ? 5 : 6;
}
// class k's list and counter (0 W, 1 S, 2 S2, 3 M1, 4 M2, 5 M3, 6 L, 7 M0)
__device__ __forceinline__ uint64_t* class_list(const Ctx& c, int cls)
{
    return cls == 0 ? c.L.w : cls == 1 ? c.L.s : cls == 2 ? c.L.s2 : cls == 3 ? c.L.m1 : cls == 4 ? c.L.m2
         : cls == 5 ? c.L.m3 : cls == 7 ? c.L.m0 : c.L.l[c.lsel];
}
__device__ __forceinline__ uint32_t* class_ctr(const Ctx& c, int cls)
{
    return c.L.ctr + (cls == 0 ? C_W : cls == 1 ? C_S : cls == 2 ? C_S2 : cls == 3 ? C_M1 : cls == 4 ? C_M2
                      : cls == 5 ? C_M3 : cls == 7 ? C_M0 : C_L0 + c.lsel);
}

__device__ __forceinline__ void wg_classify(const Ctx& c, uint32_t* sh, bool pred, uint32_t slot, uint32_t s,
                                            uint32_t m, uint32_t shift, uint32_t par)
{
    const int cls = pred ? size_class(m) : -1;
    if (threadIdx.x < 8) sh[threadIdx.x] = 0;
    __syncthreads();
    uint32_t loff = 0;
    if (cls >= 0) loff = atomicAdd(&sh[cls], 1u);
    __syncthreads();
    if (threadIdx.x < 8 && sh[threadIdx.x]) sh[8 + threadIdx.x] = atomicAdd(class_ctr(c, (int)threadIdx.x), sh[threadIdx.x]);
    __syncthreads();
    if (cls >= 0) class_list(c, cls)[sh[8 + cls] + loff] = mk_item(slot, s, m, shift, par);
    if (cls == 6 && m > HG_MIN_PUSH) atomicMax(&c.L.ctr[C_LM0 + c.lsel], m);   // the host launches k3_hg_* only then
    __syncthreads();
}

// bits [bit, bit+nbits) of a packed symbol stream, right-aligned (1 <= nbits <= 64)
__device__ __forceinline__ uint64_t pss_bits(const uint64_t* __restrict__ w, uint64_t bit, uint32_t nbits)
{
    const uint64_t q = bit >> 6;
    const uint32_t p = (uint32_t)(bit & 63u);
    const uint64_t a = w[q];
    const uint64_t v = p ? ((a << p) | (w[q + 1] >> (64u - p))) : a;
    return v >> (64u - nbits);
}

// Key of a group element: rotation r (PSS modes) or group position q (K2/K).
struct KeySrc {
    const uint64_t* pss;
    const uint64_t* k;      // keys by position of this group's buffer (kA or kB by parity), slot base
    const uint8_t* l;       // last-column symbols by position (lA / lB by parity), slot base; or null
    uint32_t B, kbits, n, off, usek;
    __device__ __forceinline__ uint64_t operator()(uint64_t q, uint32_t r) const
    {
        if (usek) return k[q];
        uint32_t rr = r + off;
        if (rr >= n) rr -= n;
        return pss_bits(pss, (uint64_t)rr * B, kbits);
    }
    // PSS key of rotation r, branch-free (two word loads, a funnel shift)
    __device__ __forceinline__ uint64_t key_pss(uint32_t r) const
    {
        uint32_t rr = r + off;
        rr = rr >= n ? rr - n : rr;
#ifdef STARCH_EXP_NOGATHER   // timing experiment only: keys from a cache-resident window (wrong order)
        rr &= 4095u;
#endif
        const uint64_t bit = (uint64_t)rr * B;
        const uint64_t q = bit >> 6;
        const uint32_t p = (uint32_t)(bit & 63u);
        const uint64_t v = (pss[q] << p) | ((pss[q + 1] >> 1) >> (63u - p));
        return v >> (64u - kbits);
    }
    // ... and the last-column symbol of r (the symbol before it): its B bits sit
    // right before the key window, so three consecutive words cover both
    // (rotation 0 wraps: its symbol is the block's last)
    __device__ __forceinline__ uint64_t key_pss(uint32_t r, uint32_t& ls) const
    {
#ifdef STARCH_EXP_NOGATHER
        const uint32_t pr = r & 4095u;
#else
        const uint32_t pr = r ? r - 1u : n - 1u;
#endif
        uint32_t rr = r + off;
        rr = rr >= n ? rr - n : rr;
        if (off == 0 && r != 0) {
            const uint64_t bit0 = (uint64_t)pr * B;
            const uint64_t q0 = bit0 >> 6;
            const uint32_t p0 = (uint32_t)(bit0 & 63u);
            const uint64_t w0 = pss[q0], w1 = pss[q0 + 1], w2 = pss[q0 + 2];
            ls = (uint32_t)(((w0 << p0) | ((w1 >> 1) >> (63u - p0))) >> (64u - B));
            const uint32_t ps = p0 + B;                      // key start, relative to word q0
            const uint64_t a = ps >= 64 ? w1 : w0, b = ps >= 64 ? w2 : w1;
            const uint32_t p = ps & 63u;
            const uint64_t v = (a << p) | ((b >> 1) >> (63u - p));
            return v >> (64u - kbits);
        }
        const uint64_t pbit = (uint64_t)pr * B;
        const uint64_t pq = pbit >> 6;
        const uint32_t pp = (uint32_t)(pbit & 63u);
        const uint64_t pv = (pss[pq] << pp) | ((pss[pq + 1] >> 1) >> (63u - pp));
        ls = (uint32_t)(pv >> (64u - B));
        return key_pss(r);
    }
};

__device__ __forceinline__ KeySrc key_src(const Ctx& c, uint32_t slot, uint32_t par)
{
    KeySrc k;
    const uint64_t so = (uint64_t)slot * c.scr.stride;
    const Geo g = c.L.geo[slot];
    k.n = c.blocks[c.b0 + slot].n;
    k.B = g.B;
    k.usek = c.keysrc;
    k.pss = c.scr.K + so;
    k.k = (par ? c.kB : c.kA) + so;
    k.l = c.lA ? (par ? c.lB : c.lA) + so : nullptr;
    if (c.rtext == 0) {
        k.kbits = g.KB;
        k.off = 0;
    } else {
        k.kbits = g.Dp * g.B;
        k.off = (uint32_t)(((uint64_t)g.D + (uint64_t)(c.rtext - 1) * g.Dp) % k.n);
    }
    return k;
}

// Last-column symbol of rotation v: the rank (among the block's used byte
// values) of block[(v - 1) mod n] -- what the MTF consumes.  Rounds 0 and text
// rounds read it from the PSS; doubling rounds (PSS overwritten by keys) from
// the block text.  Written next to every final SA entry, so no separate
// gather pass over the block is needed.
__device__ __forceinline__ uint8_t last_sym(const Ctx& c, uint32_t slot, uint32_t v)
{
    const uint32_t b = c.b0 + slot;
    const uint32_t n = c.blocks[b].n;
    const uint32_t p = v ? v - 1u : n - 1u;
    if (!c.keysrc) {
        const uint32_t B = c.L.geo[slot].B;
        return (uint8_t)pss_bits(c.scr.K + (uint64_t)slot * c.scr.stride, (uint64_t)p * B, B);
    }
    const uint32_t byte = c.blkbytes[(uint64_t)b * c.stride + p];
    uint32_t r = __popc(c.blocks[b].in_use[byte >> 5] & ((1u << (byte & 31u)) - 1u));
    for (uint32_t j = 0; j < (byte >> 5); ++j) r += __popc(c.blocks[b].in_use[j]);
    return (uint8_t)r;
}

// key of the group element at position q holding rotation v: doubling keys
// (DBL) or the PSS; ls = its last-column symbol
template <bool DBL>
__device__ __forceinline__ uint64_t elem_key(const Ctx& c, const KeySrc& ks, uint32_t slot, uint64_t q, uint32_t v,
                                             uint32_t& ls)
{
    if constexpr (DBL) {
        ls = ks.l ? ks.l[q] : last_sym(c, slot, v);
        return ks.k[q];
    } else {
        return ks.key_pss(v, ls);
    }
}
template <bool DBL>
__device__ __forceinline__ uint64_t elem_key(const KeySrc& ks, uint64_t q, uint32_t v)
{
    if constexpr (DBL) return ks.k[q];
    else return ks.key_pss(v);
}

// symbol map of a block (rank among used byte values), >= 256 threads
__device__ __forceinline__ void load_sym(const BlockDesc& bd, uint8_t* sym, uint32_t* nin_out)
{
    const int tid = threadIdx.x;
    if (tid < 256) {
        uint32_t c = tid, below = 0;
        for (uint32_t j = 0; j < (c >> 5); ++j) below += __popc(bd.in_use[j]);
        below += __popc(bd.in_use[c >> 5] & ((1u << (c & 31)) - 1u));
        sym[c] = (uint8_t)below;
    }
    uint32_t nin = 0;
    for (int j = 0; j < 8; ++j) nin += __popc(bd.in_use[j]);
    *nin_out = nin;
}

// persistent-kernel job fetch: one lane pops, the value is broadcast
__device__ __forceinline__ uint32_t wg_pop(const Ctx& c, const uint32_t* qs, uint32_t* job_sh, uint32_t x)
{
    if (threadIdx.x == 0) *job_sh = xq_pop(c.qhead, qs, x);
    __syncthreads();
    const uint32_t j = *job_sh;
    __syncthreads();
    return j;
}

__device__ __forceinline__ uint32_t wave_pop(const Ctx& c, const uint32_t* qs, uint32_t x)
{
    uint32_t j = 0;
    if ((threadIdx.x & 63) == 0) j = xq_pop(c.qhead, qs, x);
    return (uint32_t)__shfl((int)j, 0, 64);
}

// queue sizes of a binned list (LDS), before the first pop
__device__ __forceinline__ void load_qsizes_binned(const Ctx& c, uint32_t* qs)
{
    if (threadIdx.x < 8) qs[threadIdx.x] = c.qseg[threadIdx.x + 1] - c.qseg[threadIdx.x];
    __syncthreads();
}

// ---------------------------------------------------------------------------
// k3_pss: packed symbol stream; also the block's key geometry and nInUse
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k3_pss(Ctx c)
{
    __shared__ uint8_t sym[256];
    const uint32_t slot = blockIdx.y, b = c.b0 + slot;
    const uint32_t n = c.blocks[b].n;
    uint32_t nin;
    load_sym(c.blocks[b], sym, &nin);
    const uint32_t B = nin > 1 ? (uint32_t)bits_for3(nin - 1) : 1u;
    const uint32_t nw = (uint32_t)(((uint64_t)(n + 128) * B + 63) / 64 + 1);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        Geo g;
        g.B = B;
        g.D = 64 / B;
        g.KB = g.D * B;
        g.Dp = (64 - PDIG) / B;
        g.nin = nin;
        g.D1 = (c.nbins == PNB_WIDE && B == 5 && nin <= 20) ? 3u : 0u;
        g.SH = g.D1 ? 3 * B : PDIG;
        g.pad = 0;
        c.L.geo[slot] = g;
        c.blocks[b].n_in_use = nin;
    }
    __syncthreads();
    const uint32_t w = blockIdx.x * 256 + threadIdx.x;
    if (w >= nw) return;
    const uint8_t* blk = c.blkbytes + (uint64_t)b * c.stride;
    const uint64_t bit0 = (uint64_t)w * 64;
    const uint64_t j0 = bit0 / B, j1 = (bit0 + 63) / B;
    uint64_t word = 0;
    if (B == 4 && j1 < n) {                      // 16 whole symbols: one aligned 16-B load
        const uint4 v = *reinterpret_cast<const uint4*>(blk + j0);
        const uint32_t q[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < 16; ++k) word = (word << 4) | sym[(q[k >> 2] >> (8 * (k & 3))) & 0xffu];
        c.scr.K[(uint64_t)slot * c.scr.stride + w] = word;
        return;
    }
    for (uint64_t j = j0; j <= j1; ++j) {
        const uint64_t s = sym[blk[j < n ? j : j % n]];
        const int sh = 64 - (int)B - (int)(j * B - bit0);
        word |= sh >= 0 ? (s << sh) : (s >> (-sh));
    }
    c.scr.K[(uint64_t)slot * c.scr.stride + w] = word;
}

// tile cursors / totals live in K after the PSS
__device__ __forceinline__ uint32_t* tile_hist(const Ctx& c, uint32_t slot)
{
    return reinterpret_cast<uint32_t*>(c.scr.K + (uint64_t)slot * c.scr.stride + pss_words(c.scr.stride));
}

// ---------------------------------------------------------------------------
// k3_hist: per-tile bucket histogram -> thist[slot][tile][NB]
// ---------------------------------------------------------------------------
template <int NB>
__global__ void __launch_bounds__(PT) k3_hist(Ctx c)
{
    __shared__ uint32_t cnt[NB];
    const uint32_t slot = blockIdx.y, b = c.b0 + slot, tile = blockIdx.x;
    const uint32_t n = c.blocks[b].n;
    const uint32_t t0 = tile * PTILE;
    if (t0 >= n) return;
    const Geo geo = c.L.geo[slot];
    const uint32_t B = geo.B;
    const uint64_t* pss = c.scr.K + (uint64_t)slot * c.scr.stride;
    for (int i = threadIdx.x; i < NB; i += PT) cnt[i] = 0;
    __syncthreads();
    const uint32_t e = n - t0 < (uint32_t)PTILE ? n - t0 : (uint32_t)PTILE;
    // 16 consecutive rotations per thread and step: their top-level digits all
    // come from four PSS words (funnel shifts), not two loads per rotation
    for (uint32_t k0 = threadIdx.x * 16u; k0 < e; k0 += PT * 16u) {
        const uint64_t bit0 = (uint64_t)(t0 + k0) * B;
        const uint64_t q0 = bit0 >> 6;
        const uint32_t p0 = (uint32_t)(bit0 & 63u);
        const uint64_t w[4] = {pss[q0], pss[q0 + 1], pss[q0 + 2], pss[q0 + 3]};
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const uint32_t bit = p0 + (uint32_t)k * B;      // < 64 + 15 * 8
            const uint32_t ix = bit >> 6, p = bit & 63u;
            const uint64_t a = ix == 0 ? w[0] : ix == 1 ? w[1] : w[2];
            const uint64_t nx = ix == 0 ? w[1] : ix == 1 ? w[2] : w[3];
            const uint64_t v = (a << p) | ((nx >> 1) >> (63u - p));
            if (k0 + k < e) atomicAdd(&cnt[top_digit(v, geo)], 1u);
        }
    }
    __syncthreads();
    uint32_t* th = tile_hist(c, slot) + (uint64_t)tile * NB;
    for (int i = threadIdx.x; i < NB; i += PT) th[i] = cnt[i];
}

// ---------------------------------------------------------------------------
// k3_scan: per block -- totals, bucket starts, per-tile cursors, class lists
// ---------------------------------------------------------------------------
constexpr int ST = 1024;              // k3_scan threads: NB/1024 consecutive buckets each

template <int NB>
__global__ void __launch_bounds__(ST) k3_scan(Ctx c)
{
    constexpr int Q = NB / (4 * ST);      // uint4 per thread
    __shared__ uint32_t scan_sh[ST / 64 + 1];
    __shared__ uint32_t cls_sh[16];
    const int tid = threadIdx.x;
    const uint32_t slot = blockIdx.x, b = c.b0 + slot;
    const uint32_t n = c.blocks[b].n;
    const uint32_t ntile = (n + PTILE - 1) / PTILE;
    uint4* th = reinterpret_cast<uint4*>(tile_hist(c, slot));   // [tile][NB/4]
    uint4* tot = th + (uint64_t)MAXT * (NB / 4);
    uint4 a[Q];
#pragma unroll
    for (int j = 0; j < Q; ++j) a[j] = make_uint4(0, 0, 0, 0);
#pragma unroll 4
    for (uint32_t k = 0; k < ntile; ++k) {
#pragma unroll
        for (int j = 0; j < Q; ++j) {
            const uint4 x = th[(uint64_t)k * (NB / 4) + tid * Q + j];
            a[j].x += x.x; a[j].y += x.y; a[j].z += x.z; a[j].w += x.w;
        }
    }
    uint32_t sum = 0;
#pragma unroll
    for (int j = 0; j < Q; ++j) { tot[tid * Q + j] = a[j]; sum += a[j].x + a[j].y + a[j].z + a[j].w; }
    const uint32_t pre = block_excl_scan_add<uint32_t>(sum, scan_sh, (uint32_t*)nullptr);
    uint4 run[Q];
    {
        uint32_t r = pre;
#pragma unroll
        for (int j = 0; j < Q; ++j) {
            run[j] = make_uint4(r, r + a[j].x, r + a[j].x + a[j].y, r + a[j].x + a[j].y + a[j].z);
            r += a[j].x + a[j].y + a[j].z + a[j].w;
        }
    }
#pragma unroll 4
    for (uint32_t k = 0; k < ntile; ++k) {
#pragma unroll
        for (int j = 0; j < Q; ++j) {
            uint4& x = th[(uint64_t)k * (NB / 4) + tid * Q + j];
            const uint4 v = x;
            x = run[j];
            run[j].x += v.x; run[j].y += v.y; run[j].z += v.z; run[j].w += v.w;
        }
    }
    const Geo geo = c.L.geo[slot];
    const uint32_t shift = geo.KB - geo.SH;
    uint32_t st = pre;
#pragma unroll
    for (int j = 0; j < Q; ++j) {
        const uint32_t cnt4[4] = {a[j].x, a[j].y, a[j].z, a[j].w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            wg_classify(c, cls_sh, cnt4[q] >= 2, slot, st, cnt4[q], shift, 0);
            st += cnt4[q];
        }
    }
}

// ---------------------------------------------------------------------------
// k3_scatter: rotations -> bucket order in SA (persistent, per-XCD block
// streams: queue x holds the tiles of blocks x, x+8, ... in order)
// ---------------------------------------------------------------------------
constexpr int SCT = 1024;

template <int NB>
__global__ void __launch_bounds__(SCT) k3_scatter(Ctx c)
{
    __shared__ uint32_t cur[NB], tot[NB];
    __shared__ uint32_t qs[8];
    __shared__ uint32_t job_sh;
    const int tid = threadIdx.x;
    const uint32_t x = xcc_id();
    if (tid < 8) qs[tid] = ((uint32_t)tid < c.nb ? (c.nb - tid + 7) / 8 : 0u) * MAXT;
    __syncthreads();
    for (;;) {
        const uint32_t job = wg_pop(c, qs, &job_sh, x);
        if (job == 0xFFFFFFFFu) break;
        const uint32_t y = job >> 28, k = job & 0x0FFFFFFFu;
        const uint32_t slot = y + 8u * (k / MAXT), tile = k % MAXT;
        const uint32_t b = c.b0 + slot;
        const uint32_t n = c.blocks[b].n;
        const uint32_t t0 = tile * PTILE;
        if (t0 >= n) continue;                       // uniform
        const uint64_t so = (uint64_t)slot * c.scr.stride;
        const uint32_t* th = tile_hist(c, slot);
        for (int i = tid; i < NB; i += SCT) { cur[i] = th[(uint64_t)tile * NB + i]; tot[i] = th[(uint64_t)MAXT * NB + i]; }
        __syncthreads();
        const Geo geo = c.L.geo[slot];
        const uint32_t B = geo.B;
        const uint64_t* pss = c.scr.K + so;
        uint32_t* SA = c.scr.SA + so;
        const uint32_t e = n - t0 < (uint32_t)PTILE ? n - t0 : (uint32_t)PTILE;
        // SU consecutive rotations per thread and step: digits from four PSS
        // words (funnel shifts), then the LDS cursor atomics, then the stores,
        // so each phase has SU in flight
        constexpr int SU = 16;
        for (uint32_t q0 = tid * SU; q0 < e; q0 += SU * SCT) {
            uint32_t d[SU], p[SU];
            {
                const uint64_t bit0 = (uint64_t)(t0 + q0) * B;
                const uint64_t qw = bit0 >> 6;
                const uint32_t p0 = (uint32_t)(bit0 & 63u);
                const uint64_t w[4] = {pss[qw], pss[qw + 1], pss[qw + 2], pss[qw + 3]};
#pragma unroll
                for (int u = 0; u < SU; ++u) {
                    const uint32_t bit = p0 + (uint32_t)u * B;  // < 64 + 15 * 8
                    const uint32_t ix = bit >> 6, pb = bit & 63u;
                    const uint64_t a = ix == 0 ? w[0] : ix == 1 ? w[1] : w[2];
                    const uint64_t nx = ix == 0 ? w[1] : ix == 1 ? w[2] : w[3];
                    d[u] = top_digit((a << pb) | ((nx >> 1) >> (63u - pb)), geo);
                }
            }
#pragma unroll
            for (int u = 0; u < SU; ++u) {
                const uint32_t q = q0 + u;
                p[u] = q < e ? atomicAdd(&cur[d[u]], 1u) : 0u;
            }
#pragma unroll
            for (int u = 0; u < SU; ++u) {
                const uint32_t q = q0 + u;
                if (q < e) {
                    const uint32_t r = t0 + q;
                    SA[p[u]] = r;
                    if (tot[d[u]] == 1u) {           // singleton bucket: final
                        c.scr.LL[so + p[u]] = (uint8_t)pss_bits(pss, (uint64_t)(r ? r - 1u : n - 1u) * B, B);
                        if (r == 0) c.blocks[b].orig_ptr = p[u];
                    }
                }
            }
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// k3_scatter_lds: the same scatter with the writes staged in LDS.  Each 32 K
// tile is handled in two 16 K halves: the half's rotations are counting-
// sorted by bucket inside LDS (entry = digit << 15 | rotation in the tile), then written
// out in local order, so consecutive threads store consecutive SA positions
// of a bucket's run instead of one scattered 4-byte store per rotation (the
// direct scatter's writes cost ~2.5-3.5x their bytes in HBM traffic).
// ---------------------------------------------------------------------------
template <int NB, bool MAT>
__global__ void __launch_bounds__(SCT) k3_scatter_lds(Ctx c)
{
    // rotations staged at a time: half a tile (4096 bins), a quarter (8192 bins: LDS)
    constexpr uint32_t SH_HALF = NB == PNB ? PTILE / 2 : PTILE / 4;
    constexpr int SU = (int)(SH_HALF / SCT);       // consecutive rotations per thread
    constexpr int BPT = NB / SCT;                  // bins per thread in the local scan
    __shared__ uint32_t cur[NB], tot[NB], lst[NB + 1];
    __shared__ uint32_t stage[SH_HALF];
    // the next 8 key bits below the top-level digit, staged beside each entry:
    // written next to the SA entries of the heavy (L-class) buckets, where
    // k3_part_l's first partition reads them instead of gathering each
    // rotation's key again (the plain instantiation only)
    __shared__ uint8_t stage8[MAT ? 4 : SH_HALF];
    __shared__ uint32_t scan_sh[SCT / 64 + 1];
    __shared__ uint32_t qs[8];
    __shared__ uint32_t job_sh;
    // round 0 writes every rotation's key window and last-column symbol next to
    // its SA entry (KM0 / LS0), from the stage's PSS words held in LDS
    // (MAT: bwt_kmat() only; the plain instantiation keeps no PSS window in LDS)
    constexpr uint32_t PWN = MAT ? (SH_HALF + 1) * 8 / 64 + 4 : 1;   // words for B <= 8
    __shared__ uint64_t pw[PWN];
    constexpr bool mat = MAT;
    const int tid = threadIdx.x;
    const uint32_t x = xcc_id();
    if (tid < 8) qs[tid] = ((uint32_t)tid < c.nb ? (c.nb - tid + 7) / 8 : 0u) * MAXT;
    __syncthreads();
    for (;;) {
        const uint32_t job = wg_pop(c, qs, &job_sh, x);
        if (job == 0xFFFFFFFFu) break;
        const uint32_t y = job >> 28, k = job & 0x0FFFFFFFu;
        const uint32_t slot = y + 8u * (k / MAXT), tile = k % MAXT;
        const uint32_t b = c.b0 + slot;
        const uint32_t n = c.blocks[b].n;
        const uint32_t t0 = tile * PTILE;
        if (t0 >= n) continue;                       // uniform
        const uint64_t so = (uint64_t)slot * c.scr.stride;
        const uint32_t* th = tile_hist(c, slot);
        for (int i = tid; i < NB; i += SCT) { cur[i] = th[(uint64_t)tile * NB + i]; tot[i] = th[(uint64_t)MAXT * NB + i]; }
        const Geo geo = c.L.geo[slot];
        const uint32_t B = geo.B;
        const uint64_t* pss = c.scr.K + so;
        uint32_t* SA = c.scr.SA + so;
        uint64_t* KM = c.kA + so;
        uint8_t* LS = c.lA ? c.lA + so : nullptr;
        const uint32_t e = n - t0 < (uint32_t)PTILE ? n - t0 : (uint32_t)PTILE;
        for (uint32_t h0 = 0; h0 < e; h0 += SH_HALF) {
            const uint32_t he = e - h0 < SH_HALF ? e - h0 : SH_HALF;
            for (int i = tid; i < NB; i += SCT) lst[i] = 0;
            // PSS words of this stage's keys and last symbols: rotations
            // [t0 + h0 - 1, t0 + h0 + he) plus one key window
            const uint32_t rs = t0 + h0;
            const uint64_t wbase = rs ? ((uint64_t)(rs - 1) * B) >> 6 : 0;
            if constexpr (mat) {
                const uint64_t wend = (((uint64_t)(rs + he) * B + 64) >> 6) + 2;
                for (uint64_t w = wbase + tid; w < wend; w += SCT) pw[w - wbase] = pss[w];
            }
            __syncthreads();
            // digits of SU consecutive rotations from four PSS words; local counts
            const uint32_t q0 = tid * SU;                // SCT * SU == SH_HALF
            uint32_t d[SU], p[SU];
            uint8_t sd[SU];
            {
                const uint64_t bit0 = (uint64_t)(t0 + h0 + q0) * B;
                const uint64_t qw = bit0 >> 6;
                const uint32_t p0 = (uint32_t)(bit0 & 63u);
                const uint64_t w[4] = {pss[qw], pss[qw + 1], pss[qw + 2], pss[qw + 3]};
                const uint32_t sds = 64u - geo.SH - 8u;       // (the key window's bits [SH, SH + 8))
#pragma unroll
                for (int u = 0; u < SU; ++u) {
                    const uint32_t bit = p0 + (uint32_t)u * B;
                    const uint32_t ix = bit >> 6, pb = bit & 63u;
                    const uint64_t a = ix == 0 ? w[0] : ix == 1 ? w[1] : w[2];
                    const uint64_t nx = ix == 0 ? w[1] : ix == 1 ? w[2] : w[3];
                    const uint64_t v = (a << pb) | ((nx >> 1) >> (63u - pb));
                    d[u] = top_digit(v, geo);
                    sd[u] = (uint8_t)(v >> sds);
                }
            }
#pragma unroll
            for (int u = 0; u < SU; ++u) p[u] = (q0 + u < he) ? atomicAdd(&lst[d[u]], 1u) : 0u;
            __syncthreads();
            // local bucket starts (exclusive scan, BPT bins per thread)
            {
                uint32_t v[BPT], sum = 0;
#pragma unroll
                for (int q = 0; q < BPT; ++q) { v[q] = lst[tid * BPT + q]; sum += v[q]; }
                uint32_t run = block_excl_scan_add<uint32_t>(sum, scan_sh, (uint32_t*)nullptr);
#pragma unroll
                for (int q = 0; q < BPT; ++q) { lst[tid * BPT + q] = run; run += v[q]; }
                if (tid == SCT - 1) lst[NB] = run;
            }
            __syncthreads();
#pragma unroll
            for (int u = 0; u < SU; ++u)
                if (q0 + u < he) {
                    const uint32_t j = lst[d[u]] + p[u];
                    stage[j] = (d[u] << 15) | (h0 + q0 + u);   // 13 + 15 bits
                    if constexpr (!MAT) stage8[j] = sd[u];
                }
            __syncthreads();
            // write out in local (bucket) order: runs of a bucket land on consecutive SA slots
            for (uint32_t j = tid; j < he; j += SCT) {
                const uint32_t v = stage[j];
                const uint32_t dg = v >> 15, r = t0 + (v & 0x7FFFu);
                const uint32_t pos = cur[dg] + (j - lst[dg]);
                st_nt(SA + pos, r);
                uint32_t ls = 0;
                if (mat && r) {   // (MAT: compile-time)
                    const uint64_t bit = (uint64_t)(r - 1) * B - (wbase << 6);
                    const uint32_t q = (uint32_t)(bit >> 6), p = (uint32_t)(bit & 63u);
                    ls = (uint32_t)(((pw[q] << p) | ((pw[q + 1] >> 1) >> (63u - p))) >> (64u - B));
                } else if (mat || tot[dg] == 1u) {
                    ls = (uint32_t)pss_bits(pss, (uint64_t)(r ? r - 1u : n - 1u) * B, B);
                }
                if (mat) {
                    const uint64_t bit = (uint64_t)r * B - (wbase << 6);
                    const uint32_t q = (uint32_t)(bit >> 6), p = (uint32_t)(bit & 63u);
                    KM[pos] = ((pw[q] << p) | ((pw[q + 1] >> 1) >> (63u - p))) >> (64u - geo.KB);
                    LS[pos] = (uint8_t)ls;
                }
                if (tot[dg] == 1u) {                   // singleton bucket: final
                    c.scr.LL[so + pos] = (uint8_t)ls;
                    if (r == 0) c.blocks[b].orig_ptr = pos;
                } else if (!mat && tot[dg] > L_MIN) {  // L class: its first partition digit (LL is free there until then)
                    c.scr.LL[so + pos] = stage8[j];
                }
            }
            __syncthreads();
            for (int i = tid; i < NB; i += SCT) cur[i] += lst[i + 1] - lst[i];
            __syncthreads();
        }
    }
}

// ---------------------------------------------------------------------------
// binning of a work list by block into per-XCD segments (blocks x, x+8, ...).
// A batch of few blocks (nb < 64) bins by (block, 64-item run mod 8) instead
// (vs = 3), so its groups spread over all XCDs: one block's PSS fits every
// L2, and binning by block alone would leave 7 of 8 XCDs idle.  Lists come
// out of the sorts mostly grouped by block: a wave whose 64 items share a bin
// counts / places them with one LDS atomic (one atomic per item serialised
// the wave on one address).
// ---------------------------------------------------------------------------
constexpr uint32_t BIN_CH = 4096;     // items per binning workgroup (at least)
constexpr uint32_t BIN_MAXWG = 128;

__device__ __forceinline__ uint32_t bin_of(uint64_t it, uint32_t i, uint32_t vs)
{
    return (it_slot(it) << vs) | ((i >> 6) & ((1u << vs) - 1u));
}

// chunks are multiples of 64 items, so every wave's 64 items share i >> 6
__global__ void __launch_bounds__(256) k3_bin_hist(const uint64_t* __restrict__ in, uint32_t n, uint32_t nb,
                                                    uint32_t ch, uint32_t* __restrict__ hist,
                                                    uint32_t* __restrict__ colsum, uint32_t vs)
{
    __shared__ uint32_t h[4096];
    for (uint32_t i = threadIdx.x; i < nb; i += 256) h[i] = 0;
    __syncthreads();
    const uint32_t a = blockIdx.x * ch, e = a + ch < n ? a + ch : n;
    for (uint32_t i0 = a; i0 < e; i0 += 256) {     // wave-uniform trip count
        const uint32_t i = i0 + threadIdx.x;
        const bool ok = i < e;
        const uint32_t b = ok ? bin_of(in[i], i, vs) : 0u;
        const uint64_t act = __ballot(ok);
        if (!act) continue;
        const int lead = __ffsll((unsigned long long)act) - 1;
        const uint32_t b0 = (uint32_t)__shfl((int)b, lead, 64);
        if (__ballot(ok && b == b0) == act) {
            if ((int)(threadIdx.x & 63) == lead) atomicAdd(&h[b0], (uint32_t)__popcll(act));
        } else if (ok) {
            atomicAdd(&h[b], 1u);
        }
    }
    __syncthreads();
    // this chunk's place inside each bin: one global atomic per non-empty bin
    // (chunks take their places in any order; a bin's items are independent)
    for (uint32_t i = threadIdx.x; i < nb; i += 256) {
        const uint32_t x = h[i];
        hist[(uint64_t)blockIdx.x * nb + i] = x ? atomicAdd(&colsum[i], x) : 0u;
    }
}

// one workgroup: the bins' totals (k3_bin_hist's atomics), reset for the
// next binning, and their XCD-ordered exclusive scan -> each bin's start;
// seg[x] = start of XCD x's segment.  (Per-(chunk, bin) offsets used to be
// scanned here row by row: a dependent walk over up to 128 rows per bin.)
__global__ void __launch_bounds__(1024) k3_bin_scan(uint32_t* __restrict__ colsum, uint32_t* __restrict__ bstart,
                                                     uint32_t nb, uint32_t* __restrict__ seg)
{
    __shared__ uint32_t scan_sh[1024 / 64 + 1];
    const int tid = threadIdx.x;
    const uint32_t NS = (nb + 7) / 8;               // blocks per XCD segment (upper bound)
    // XCD-ordered sequence j -> block s = (j / NS) + 8 * (j % NS); 4 entries per thread
    uint32_t v[4], sum = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t j = tid * 4 + q;
        const uint32_t s = (j / NS) + 8u * (j % NS);
        v[q] = 0u;
        if (j < 8 * NS && s < nb) {
            v[q] = colsum[s];
            colsum[s] = 0u;
        }
        sum += v[q];
    }
    uint32_t total = 0;
    uint32_t run = block_excl_scan_add<uint32_t>(sum, scan_sh, &total);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t j = tid * 4 + q;
        const uint32_t s = (j / NS) + 8u * (j % NS);
        if (j < 8 * NS && (j % NS) == 0) seg[j / NS] = run;
        if (j < 8 * NS && s < nb) bstart[s] = run;
        run += v[q];
    }
    if (tid == 0) seg[8] = total;
}

__global__ void __launch_bounds__(256) k3_bin_scatter(const uint64_t* __restrict__ in, uint32_t n, uint32_t nb,
                                                       uint32_t ch, const uint32_t* __restrict__ hist,
                                                       const uint32_t* __restrict__ bstart,
                                                       uint64_t* __restrict__ out, uint32_t vs)
{
    __shared__ uint32_t cur[4096];
    for (uint32_t i = threadIdx.x; i < nb; i += 256) cur[i] = bstart[i] + hist[(uint64_t)blockIdx.x * nb + i];
    __syncthreads();
    const uint32_t a = blockIdx.x * ch, e = a + ch < n ? a + ch : n;
    for (uint32_t i0 = a; i0 < e; i0 += 256) {     // wave-uniform trip count
        const uint32_t i = i0 + threadIdx.x;
        const bool ok = i < e;
        const uint64_t it = ok ? in[i] : 0ull;
        const uint32_t b = ok ? bin_of(it, i, vs) : 0u;
        const uint64_t act = __ballot(ok);
        if (!act) continue;
        const int lane = (int)(threadIdx.x & 63), lead = __ffsll((unsigned long long)act) - 1;
        const uint32_t b0 = (uint32_t)__shfl((int)b, lead, 64);
        uint32_t pos;
        if (__ballot(ok && b == b0) == act) {          // one bin: one atomic, items in lane order
            uint32_t base = 0;
            if (lane == lead) base = atomicAdd(&cur[b0], (uint32_t)__popcll(act));
            base = (uint32_t)__shfl((int)base, lead, 64);
            pos = base + (uint32_t)__popcll(act & ((1ull << lane) - 1ull));
        } else {
            pos = ok ? atomicAdd(&cur[b], 1u) : 0u;
        }
        if (ok) out[pos] = it;
    }
}

// ---------------------------------------------------------------------------
// k3_part_l: MSD partition of one large group on its next <= 8 key bits
// (persistent over a binned list; values ping-pong SA <-> V, and in doubling
// mode the K2 <-> K keys with them)
// ---------------------------------------------------------------------------
constexpr int LT = 512;
constexpr int LW = LT / 64;
// round 0 / text rounds: the first pass keeps every element's digit in LDS,
// so the scatter pass re-reads only the (coalesced) rotations, not their
// PSS keys (random 8-byte loads); groups above PL_CAP recompute the keys
constexpr uint32_t PL_CAP = 40960;
#ifndef STARCH_PL_STG
#define STARCH_PL_STG 24576
#endif
constexpr uint32_t PL_STG = STARCH_PL_STG;

#ifdef STARCH_PL_PROF   // timing experiment (dev builds): k3_part_l's phases, shader clocks summed over workgroups
__device__ unsigned long long g_plprof[16];
#define PLT(v) const uint64_t v = __builtin_readcyclecounter()
#define PLA(i, a, b) plp[i] += (b) - (a)
#else
#define PLT(v)
#define PLA(i, a, b)
#endif
template <bool DBL>
__global__ void __launch_bounds__(LT) k3_part_l(Ctx c, const uint64_t* __restrict__ items)
{
#ifdef STARCH_PL_PROF
    uint64_t plp[8] = {};
    PLT(tk0);
#endif
    __shared__ uint32_t wh[LW][256];
    __shared__ uint32_t st[256], cur[256], cntd[256];
    __shared__ uint32_t scan_sh[LW + 1];
    __shared__ uint32_t big[257];
    __shared__ uint32_t qs[8];
    __shared__ uint32_t job_sh;
    __shared__ uint32_t cls_sh[16];
    __shared__ uint8_t dcache[DBL ? 4 : PL_CAP];
    // round 0 / text rounds: the partitioned rotations of a group up to
    // PL_STG are assembled here and stored in one coalesced pass (the scatter
    // into 256 sub-buckets wrote one lone 4-byte word per rotation)
    __shared__ uint32_t stg[DBL ? 1 : PL_STG];
    const int tid = threadIdx.x, wid = tid >> 6;
    const uint32_t x = xcc_id();
    load_qsizes_binned(c, qs);
    for (;;) {
        const uint32_t job = wg_pop(c, qs, &job_sh, x);
        if (job == 0xFFFFFFFFu) break;
        const uint64_t item = items[c.qseg[job >> 28] + (job & 0x0FFFFFFFu)];
        const uint32_t slot = it_slot(item), s = it_start(item), m = it_size(item), shift = it_shift(item),
                       par = it_par(item);
        if (m == 0) continue;                          // taken by the grid-wide path (k3_hg_pick); uniform
        PLT(t0);
#ifdef STARCH_PL_PROF
        plp[6] += m;
        plp[5] += 1;
#endif
        const uint32_t b = c.b0 + slot;
        const uint64_t so = (uint64_t)slot * c.scr.stride;
        const uint64_t base = so + s;
        const KeySrc ks = key_src(c, slot, par);
        const uint32_t* sv = (par ? c.scr.V : c.scr.SA) + base;
        uint32_t* dv = (par ? c.scr.SA : c.scr.V) + base;
        uint64_t* dk = (par ? c.kA : c.kB) + base;              // keys by position (keysrc 1) only
        uint8_t* dl = DBL && ks.l ? (par ? c.lA : c.lB) + base : nullptr;   // round 0: last symbols move too
        uint32_t* SA = c.scr.SA + base;
        uint32_t* RK = c.scr.RK + so;
        const uint32_t db = shift < 8 ? shift : 8;
        const uint32_t sh2 = shift - db;
        const uint64_t dmask = (1ull << db) - 1ull;
        // a top-level L bucket of round 0: the scatter left each rotation's
        // digit (its key bits [SH, SH + 8)) in LL next to it
        const uint8_t* sdig = nullptr;
        if (!DBL && c.sdig && c.rtext == 0 && !c.mode && par == 0 && db == 8) {
            const Geo g = c.L.geo[slot];
            if (shift == g.KB - g.SH) sdig = c.scr.LL + base;
        }
        for (int i = tid; i < LW * 256; i += LT) (&wh[0][0])[i] = 0;
        if (tid == 0) big[256] = 0;
        __syncthreads();
        PLT(t1);
        PLA(0, t0, t1);
#ifndef STARCH_PART_PU
#define STARCH_PART_PU 24   // elements per thread and step, loads batched (cfg2 block sort: 4 -> 16 -> 24 -> 32: 21.3, 20.6, 20.4, 20.7 ms)
#endif
        constexpr int PU = STARCH_PART_PU;             // elements in flight per thread
        // (each pass issues all PU loads of a step before using any: a load
        // chosen per element inside the unrolled loop was waited on one by one)
        for (uint32_t i0 = 0; i0 < m; i0 += PU * LT) {
            uint32_t d[PU];
            if (sdig) {
#pragma unroll
                for (int u = 0; u < PU; ++u) {
                    const uint32_t i = i0 + u * LT + tid;
                    d[u] = sdig[i < m ? i : 0u];
                }
            } else {
                uint32_t vv[PU];
#pragma unroll
                for (int u = 0; u < PU; ++u) {
                    const uint32_t i = i0 + u * LT + tid;
                    vv[u] = ld_nt(sv + (i < m ? i : 0u));
                }
#pragma unroll
                for (int u = 0; u < PU; ++u) {
                    const uint32_t i = i0 + u * LT + tid;
                    d[u] = (uint32_t)((elem_key<DBL>(ks, s + (i < m ? i : 0u), vv[u]) >> sh2) & dmask);
                }
            }
#pragma unroll
            for (int u = 0; u < PU; ++u) {
                const uint32_t i = i0 + u * LT + tid;
                if (!DBL && m <= PL_CAP && i < m) dcache[i] = (uint8_t)d[u];
            }
#pragma unroll
            for (int u = 0; u < PU; ++u)
                if (i0 + u * LT + tid < m) atomicAdd(&wh[wid][d[u]], 1u);
        }
        __syncthreads();
        PLT(t2);
        PLA(1, t1, t2);
        uint32_t tcount = 0;
        if (tid < 256) for (int w = 0; w < LW; ++w) tcount += wh[w][tid];
        const uint32_t pre = block_excl_scan_add<uint32_t>(tid < 256 ? tcount : 0u, scan_sh, (uint32_t*)nullptr);
        if (tid < 256) { st[tid] = pre; cur[tid] = pre; cntd[tid] = tcount; }
        __syncthreads();
        PLT(t3);
        PLA(2, t2, t3);
        const bool staged = !DBL && m <= PL_STG && !(STARCH_PL_STG == 0);
        for (uint32_t i0 = 0; i0 < m; i0 += PU * LT) {
            uint32_t v[PU];
            uint64_t k[PU];
            uint8_t lsy[PU];
#pragma unroll
            for (int u = 0; u < PU; ++u) {
                const uint32_t i = i0 + u * LT + tid;
                v[u] = ld_nt(sv + (i < m ? i : 0u));
            }
            if (!DBL && m <= PL_CAP) {                 // only the digit is used below
#pragma unroll
                for (int u = 0; u < PU; ++u) {
                    const uint32_t i = i0 + u * LT + tid;
                    k[u] = (uint64_t)dcache[i < m ? i : 0u] << sh2;
                }
            } else if (sdig) {
#pragma unroll
                for (int u = 0; u < PU; ++u) {
                    const uint32_t i = i0 + u * LT + tid;
                    k[u] = (uint64_t)sdig[i < m ? i : 0u] << sh2;
                }
            } else {
#pragma unroll
                for (int u = 0; u < PU; ++u) {
                    const uint32_t i = i0 + u * LT + tid;
                    k[u] = elem_key<DBL>(ks, s + (i < m ? i : 0u), v[u]);
                }
            }
#pragma unroll
            for (int u = 0; u < PU; ++u) {
                const uint32_t i = i0 + u * LT + tid;
                lsy[u] = dl ? ks.l[s + (i < m ? i : 0u)] : (uint8_t)0;
            }
#pragma unroll
            for (int u = 0; u < PU; ++u) {
                if (i0 + u * LT + tid < m) {
                    const uint32_t p = atomicAdd(&cur[(uint32_t)((k[u] >> sh2) & dmask)], 1u);
                    if (!DBL && staged) stg[p] = v[u];
                    else st_nt(dv + p, v[u]);
                    if constexpr (DBL) dk[p] = k[u];
                    if (dl) dl[p] = lsy[u];
                }
            }
        }
        __syncthreads();
        if (!DBL && staged) {
            for (uint32_t i = tid; i < m; i += LT) st_nt(dv + i, stg[i]);
            __syncthreads();
        }
        PLT(t4);
        PLA(3, t3, t4);
        uint32_t nruns = 0;
        if (tid < 256) {
            const uint32_t cc = cntd[tid], ss = st[tid];
            if (cc == 1) {
                const uint32_t v = dv[ss];
                if (!par) SA[ss] = v;
                c.scr.LL[base + ss] = dl ? dl[ss] : last_sym(c, slot, v);
                if (c.mode) RK[v] = s + ss;
                if (v == 0) c.blocks[b].orig_ptr = s + ss;
                nruns = 1;
            } else if (size_class(cc) == 6 && sh2 == 0) {
                big[atomicAdd(&big[256], 1u)] = tid;   // all keys equal: one group
                nruns = 1;
            }
        }
        {
            const uint32_t cc = tid < 256 ? cntd[tid] : 0u;
            const bool push = tid < 256 && cc >= 2 && !(size_class(cc) == 6 && sh2 == 0);
            wg_classify(c, cls_sh, push, slot, s + (tid < 256 ? st[tid] : 0u), cc, sh2, par ^ 1u);
        }
        if (tid < 256) {
            const uint32_t r = wave_reduce_add(nruns);
            if (c.mode && (tid & 63) == 0 && r) atomicAdd(&c.L.runs[slot], r);
        }
        __syncthreads();
        PLT(t5);
        PLA(4, t4, t5);
        const uint32_t nbig = big[256];
        for (uint32_t q = 0; q < nbig; ++q) {
            const uint32_t d = big[q];
            const uint32_t ss = st[d], cc = cntd[d];
            for (uint32_t i = tid; i < cc; i += LT) {
                const uint32_t v = dv[ss + i];
                if (!par) SA[ss + i] = v;
                c.scr.LL[base + ss + i] = dl ? dl[ss + i] : last_sym(c, slot, v);
                if (c.mode) RK[v] = s + ss;
                if (v == 0) c.blocks[b].orig_ptr = s + ss + i;
            }
            if (tid == 0) {
                const uint32_t o = atomicAdd(c.L.ctr + C_T0 + c.tsel, 1u);
                c.L.t[c.tsel][o] = mk_item(slot, s + ss, cc, 0, 0);
                atomicAdd(c.L.ctr + C_TS0 + c.tsel, cc);
            }
        }
        __syncthreads();
        PLT(t6);
        PLA(7, t5, t6);
    }
#ifdef STARCH_PL_PROF
    PLT(tk1);
    plp[4] += 0;
    if (tid == 0) {
        for (int q = 0; q < 8; ++q) atomicAdd(&g_plprof[q], (unsigned long long)plp[q]);
        atomicAdd(&g_plprof[8], (unsigned long long)(tk1 - tk0));
    }
#endif
}

// ---------------------------------------------------------------------------
// Huge groups (> HG_MIN rotations): k3_part_l's MSD partition step spread over
// the whole grid.  One k3_part_l workgroup per group left a group of
// hundreds of thousands of tied rotations -- every doubling round of a
// near-periodic block (per-position BED: "0\n" repeated, broken once) -- to
// one CU for the whole round.  Here a group is cut into HG_CH-element chunks:
// per-chunk digit histograms (k3_hg_hist), one workgroup per group scans them
// into per-chunk cursors and classifies the sub-buckets exactly as k3_part_l
// does (k3_hg_scan), every chunk scatters its elements (k3_hg_scatter), and
// sub-buckets that are final (singletons, or all-equal keys with no key bits
// left) are written out by k3_hg_final -- after the scatter, so no chunk's
// source reads race the final SA writes.
// ---------------------------------------------------------------------------
// the grid split over ng groups: several workgroups per group when there are
// fewer groups than workgroups, else one (every workgroup looping over all
// groups cost thousands of empty iterations per workgroup with 4k groups)
struct GridSplit {
    uint32_t per, gstride, q0, slice;
    bool idle;
};
__device__ __forceinline__ GridSplit grid_split(uint32_t ng)
{
    GridSplit s;
    const uint32_t G = gridDim.x;
    s.per = ng >= G ? 1u : G / (ng ? ng : 1u);
    s.gstride = G / s.per;
    s.idle = blockIdx.x >= s.per * s.gstride;
    s.q0 = blockIdx.x / s.per;
    s.slice = blockIdx.x % s.per;
    return s;
}

constexpr uint32_t HG_MIN = HG_MIN_PUSH;
constexpr uint32_t HG_CH = 1024;        // elements per chunk: 4 per thread, every chunk in flight at once
constexpr uint32_t HG_MAXCH = 1u << 22; // chunks per level (the pick's budget: any batch)
constexpr uint32_t HG_MAXN = 8192;      // huge groups per level (two per near-periodic block of a full batch)
constexpr uint32_t HG_FINAL = 1u << 31;
// k3_hg_scan's verdict on a group whose digit window holds no varying key bit
// (hg_vary): HG_SKIP_ALL -- every remaining key bit is equal: the whole group
// is one final tie group, written out from where it is; HG_SKIP_RELABEL -- it
// goes back to the L list with its shift lowered to its highest varying bit.
// Either way no element moves at this level.  (Near-periodic blocks -- a
// per-position BED's "0\n" repeated -- send groups of ~450k rotations whose
// 52-64 key bits are all equal through here: seven 8-bit levels each, per
// round, before this.)
constexpr uint32_t HG_SKIP_ALL = 1, HG_SKIP_RELABEL = 2;
// ... and when more than half the group's keys equal its first element's key
// over every remaining bit -- a doubling round's unresolved rotations, all
// ranked at the same tie group -- the level is a three-way split instead of a
// digit: below / equal / above that key.  The equal part is final at once (a
// tie group for the next round); the other two keep the shift.  One pass per
// round instead of a digit level per 8 key bits, each moving the whole group.
constexpr uint32_t HG_THREE = 3;
// The three-way split in place (par 0, no last-column stream): only the
// elements outside their part's range move (each into a hole of its part,
// through short lists), and the equal part -- most of the group -- stays where
// it is.  Its rank (RK) is any position inside its range (ranks only have to
// order the groups' disjoint ranges), so the previous round's rank is kept
// when it still lies inside: a doubling round of a near-periodic block then
// writes neither SA nor RK for its unresolved rotations.
constexpr uint32_t HG_THREE_IP = 4;
constexpr uint32_t HG_KEEP = 0xFFFFFFFFu;

// L-list items above HG_MIN whose chunks fit go to the huge list; their
// L-list entry gets size 0 (k3_part_l skips it)
__global__ void k3_hg_pick(Ctx c, uint64_t* __restrict__ list, uint32_t n)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t item = list[i];
    const uint32_t m = it_size(item);
    if (m <= HG_MIN) return;
    const uint32_t nch = (m + HG_CH - 1) / HG_CH;
    const uint32_t k = atomicAdd(&c.L.ctr[C_HG], 1u);
    if (k >= HG_MAXN) return;
    const uint32_t base = atomicAdd(&c.L.ctr[C_HGC], nch);
    if (base + nch > HG_MAXCH) {            // over budget: k3_part_l keeps it
        c.L.hg[k] = 0;
        return;
    }
    c.L.hg[k] = item;
    list[i] = mk_item(it_slot(item), it_start(item), 0, it_shift(item), it_par(item));
}

struct HgGroup {
    uint32_t slot, s, m, shift, par, db, sh2, nch;
    uint64_t dmask;
};
__device__ __forceinline__ HgGroup hg_group(uint64_t item)
{
    HgGroup g;
    g.slot = it_slot(item);
    g.s = it_start(item);
    g.m = it_size(item);
    g.shift = it_shift(item);
    g.par = it_par(item);
    g.db = g.shift < 8 ? g.shift : 8;
    g.sh2 = g.shift - g.db;
    g.dmask = (1ull << g.db) - 1ull;
    g.nch = (g.m + HG_CH - 1) / HG_CH;
    return g;
}

// count[d] += 1 for a wave's lanes (one LDS atomic when they share a digit:
// a skewed group sends most elements to one bin); returns the lane's slot
__device__ __forceinline__ uint32_t wave_bin_add(uint32_t* cnt, bool act, uint32_t d)
{
    const uint64_t a = __ballot(act);
    if (!a) return 0;
    const int lead = __ffsll((unsigned long long)a) - 1;
    const uint32_t d0 = (uint32_t)__shfl((int)d, lead, 64);
    const int lane = threadIdx.x & 63;
    if (__ballot(act && d == d0) == a) {
        uint32_t b = 0;
        if (lane == lead) b = atomicAdd(&cnt[d0], (uint32_t)__popcll(a));
        b = (uint32_t)__shfl((int)b, lead, 64);
        return b + (uint32_t)__popcll(a & lanemask_lt());
    }
    return act ? atomicAdd(&cnt[d], 1u) : 0u;
}

// the chunks of every huge group as one flat index space: chunk j of the
// launch -> (group q, chunk in group), from the groups' chunk-count prefix
// (k3_hg_prefix, global: thousands of groups per level)
__device__ __forceinline__ uint32_t hg_count(const Ctx& c) { return min(c.L.ctr[C_HG], HG_MAXN); }
__device__ __forceinline__ uint32_t hg_group_of(const uint32_t* __restrict__ pre, uint32_t nh, uint32_t j)
{
    uint32_t lo = 0, hi = nh - 1;
    while (lo < hi) {                      // last q with pre[q] <= j (empty groups share a start)
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (pre[mid] <= j) lo = mid; else hi = mid - 1;
    }
    return lo;
}

// one workgroup: the huge groups' chunk counts, prefix-summed (0 for a group
// left to k3_part_l)
__global__ void __launch_bounds__(1024) k3_hg_prefix(Ctx c)
{
    __shared__ uint32_t scan_sh[17];
    const uint32_t nh = hg_count(c), tid = threadIdx.x;
    uint32_t run = 0;
    for (uint32_t q0 = 0; q0 < nh; q0 += 1024) {
        const uint32_t q = q0 + tid;
        const uint32_t k = q < nh ? hg_group(c.L.hg[q]).nch : 0u;
        uint32_t tot = 0;
        const uint32_t p = block_excl_scan_add<uint32_t>(k, scan_sh, &tot);
        if (q < nh) c.L.hg_pre[q] = run + p;
        run += tot;
        __syncthreads();
    }
    if (tid == 0) c.L.hg_pre[nh] = run;
}

// per-chunk digit counts, added into the group's 256 bin totals; and the key
// bits that vary inside the group (OR of key ^ the group's first key)
template <bool DBL>
__global__ void __launch_bounds__(256) k3_hg_hist(Ctx c)
{
    __shared__ uint32_t h[256];
    __shared__ uint64_t vx[4];
    __shared__ uint32_t ve[4], vl[4];
    const uint32_t tid = threadIdx.x;
    const uint32_t nh = hg_count(c);
    if (nh == 0) return;
    const uint32_t total = c.L.hg_pre[nh];
    for (uint32_t j = blockIdx.x; j < total; j += gridDim.x) {
        const uint32_t q = hg_group_of(c.L.hg_pre, nh, j), ch = j - c.L.hg_pre[q];
        const HgGroup g = hg_group(c.L.hg[q]);
        const KeySrc ks = key_src(c, g.slot, g.par);
        const uint32_t* sv = (g.par ? c.scr.V : c.scr.SA) + (uint64_t)g.slot * c.scr.stride + g.s;
        h[tid] = 0;
        __syncthreads();
        const uint32_t a = ch * HG_CH, e = min(g.m, a + HG_CH);
        const uint64_t ref = elem_key<DBL>(ks, g.s, sv[0]);
        uint32_t d[HG_CH / 256];
        uint64_t vary = 0;
        uint32_t neq = 0, nlt = 0;
#pragma unroll
        for (uint32_t u = 0; u < HG_CH / 256; ++u) {   // all loads issued first
            const uint32_t i = a + u * 256 + tid, ic = i < e ? i : a;
            const uint64_t k = elem_key<DBL>(ks, g.s + ic, sv[ic]);
            d[u] = (uint32_t)((k >> g.sh2) & g.dmask);
            vary |= k ^ ref;
            neq += (i < e && k == ref) ? 1u : 0u;
            nlt += (i < e && k < ref) ? 1u : 0u;
        }
#pragma unroll
        for (uint32_t u = 0; u < HG_CH / 256; ++u) (void)wave_bin_add(h, a + u * 256 + tid < e, d[u]);
        vary = wave_reduce_or64(vary);
        neq = wave_reduce_add<uint32_t>(neq);
        nlt = wave_reduce_add<uint32_t>(nlt);
        if ((tid & 63) == 0) { vx[tid >> 6] = vary; ve[tid >> 6] = neq; vl[tid >> 6] = nlt; }
        __syncthreads();
        if (h[tid]) atomicAdd(&c.L.hg_info[(uint64_t)q * 512 + 256 + tid], h[tid]);   // bin totals
        if (tid == 0) {
            const uint64_t v = vx[0] | vx[1] | vx[2] | vx[3];
            if (v) atomicOr(reinterpret_cast<unsigned long long*>(&c.L.hg_vary[q]), (unsigned long long)v);
            const uint32_t te = ve[0] + ve[1] + ve[2] + ve[3], tl = vl[0] + vl[1] + vl[2] + vl[3];
            if (te) atomicAdd(&c.L.hg_eqlt[2 * q], te);
            if (tl) atomicAdd(&c.L.hg_eqlt[2 * q + 1], tl);
        }
        __syncthreads();
    }
}

// one workgroup per huge group: bin starts -> the group's global cursors,
// sub-bucket classes (k3_part_l's rules), final-bin flags; or, when the digit
// window holds no varying key bit, one of the two skips (HG_SKIP_*)
__global__ void __launch_bounds__(256) k3_hg_scan(Ctx c)
{
    __shared__ uint32_t scan_sh[5];
    __shared__ uint32_t cls_sh[16];
    const uint32_t q = blockIdx.x, tid = threadIdx.x;
    if (q >= hg_count(c)) return;
    const uint64_t item = c.L.hg[q];
    if (it_size(item) == 0) return;                   // uniform
    const HgGroup g = hg_group(item);
    const uint64_t vary = c.L.hg_vary[q] & (g.shift >= 64 ? ~0ull : ((1ull << g.shift) - 1ull));
    const int hb = vary ? 63 - __clzll((long long)vary) : -1;   // highest unsorted bit that varies
    if (hb < (int)g.sh2) {                            // uniform: no element moves at this level
        if (hb < 0) {                                 // every remaining key bit equal: one final tie group
            if (tid == 0) {
                c.L.hg_flag[q] = HG_SKIP_ALL;
                const uint32_t o = atomicAdd(c.L.ctr + C_T0 + c.tsel, 1u);
                c.L.t[c.tsel][o] = mk_item(g.slot, g.s, g.m, 0, 0);
                atomicAdd(c.L.ctr + C_TS0 + c.tsel, g.m);
                if (c.mode) atomicAdd(&c.L.runs[g.slot], 1u);
            }
            wg_classify(c, cls_sh, false, 0, 0, 0, 0, 0);
        } else {                                      // back to the L list at its highest varying bit
            if (tid == 0) c.L.hg_flag[q] = HG_SKIP_RELABEL;
            wg_classify(c, cls_sh, tid == 0, g.slot, g.s, g.m, (uint32_t)hb + 1u, g.par);
        }
        return;
    }
    uint32_t* info = c.L.hg_info + (uint64_t)q * 512;   // [0,256) start | flags, [256,512) totals -> cursors
    const uint32_t neq = c.L.hg_eqlt[2 * q], nlt = c.L.hg_eqlt[2 * q + 1];
    static_assert(L_MIN < HG_MIN, "three-way parts above L_MIN stay L items");
    if (2 * neq > g.m) {                              // uniform: three-way split around the first key
        const uint32_t ngt = g.m - neq - nlt;
        const uint32_t st3[3] = {0u, nlt, nlt + neq}, n3[3] = {nlt, neq, ngt};
        const KeySrc ks = key_src(c, g.slot, g.par);
        const bool ip = g.par == 0 && ks.l == nullptr;
        if (tid == 0) {
            c.L.hg_flag[q] = ip ? HG_THREE_IP : HG_THREE;
            if (ip) {
                uint32_t rk = g.s + nlt + neq / 2;
                if (c.mode) {                         // keep the previous rank if it lies in the equal part
                    const uint64_t so = (uint64_t)g.slot * c.scr.stride;
                    const uint32_t r0 = c.scr.RK[so + c.scr.SA[so + g.s]];
                    if (r0 >= g.s + nlt && r0 < g.s + nlt + neq) rk = HG_KEEP;
                }
                c.L.hg_rank[q] = rk;
            }
        }
        if (tid < 3) {
            const bool f = tid == 1 || n3[tid] == 1;
            info[tid] = st3[tid] | (f ? HG_FINAL : 0u);
            info[256 + tid] = st3[tid];
        } else {
            info[tid] = g.m;                          // empty bins after the three
            info[256 + tid] = g.m;
        }
        if (tid == 1 && neq >= 2) {                   // the equal part: a final tie group
            const uint32_t o = atomicAdd(c.L.ctr + C_T0 + c.tsel, 1u);
            c.L.t[c.tsel][o] = mk_item(g.slot, g.s + nlt, neq, 0, 0);
            atomicAdd(c.L.ctr + C_TS0 + c.tsel, neq);
        }
        const uint32_t t3 = tid == 2 ? 2u : 0u;      // the two parts that are sorted further
        const bool push = (tid == 0 || tid == 2) && n3[t3] >= 2;
        wg_classify(c, cls_sh, push, g.slot, g.s + st3[t3], n3[t3], g.shift, ip ? g.par : g.par ^ 1u);   // in place: same buffer
        if (tid == 0 && c.mode) atomicAdd(&c.L.runs[g.slot], 1u + (nlt == 1 ? 1u : 0u) + (ngt == 1 ? 1u : 0u));
        return;
    }
    const uint32_t cc = info[256 + tid];
    const uint32_t ss = block_excl_scan_add<uint32_t>(cc, scan_sh, (uint32_t*)nullptr);
    info[256 + tid] = ss;                             // scatter cursor
    const bool alleq = cc >= 2 && size_class(cc) == 6 && g.sh2 == 0;   // one tie group
    const bool fin = cc == 1 || alleq;
    info[tid] = ss | (fin ? HG_FINAL : 0u);
    if (alleq) {
        const uint32_t o = atomicAdd(c.L.ctr + C_T0 + c.tsel, 1u);
        c.L.t[c.tsel][o] = mk_item(g.slot, g.s + ss, cc, 0, 0);
        atomicAdd(c.L.ctr + C_TS0 + c.tsel, cc);
    }
    wg_classify(c, cls_sh, cc >= 2 && !alleq, g.slot, g.s + ss, cc, g.sh2, g.par ^ 1u);
    const uint32_t r = wave_reduce_add<uint32_t>(fin ? 1u : 0u);
    if (c.mode && (tid & 63) == 0 && r) atomicAdd(&c.L.runs[g.slot], r);
}

// In-place three-way lists of a group (parts L = [0, nlt), E, G = [nlt + neq,
// m) of its range): an element outside its part's range is a mover (its
// value -- and, doubling, its key -- goes to its part's list in the
// other-parity buffers, free for this group) and its position a hole of the
// part it sits in.  Lists: movers to L / G / E at offsets 0 / nlt / nlt + ngt
// of dv (and keys of dk; at most nlt / ngt / nlt + ngt of them); holes
// likewise in RK's range (round 0: RK unused)
// or, doubling, in dk after the keys (nlt + ngt < m / 2: everything fits).
__device__ __forceinline__ uint32_t* hg_hole_list(const Ctx& c, const HgGroup& g, uint64_t* dk, uint32_t nlt,
                                                  uint32_t ngt)
{
    if (c.mode) return reinterpret_cast<uint32_t*>(dk + nlt + ngt);
    return c.scr.RK + (uint64_t)g.slot * c.scr.stride + g.s;
}

template <bool DBL>
__device__ __forceinline__ void hg_inplace_lists(const Ctx& c, uint32_t q, const HgGroup& g, const KeySrc& ks,
                                                 const uint32_t* sv, uint32_t* dv, uint64_t* dk, uint32_t a,
                                                 uint32_t e, uint32_t* cnt)
{
    const uint32_t tid = threadIdx.x;
    const uint32_t neq = c.L.hg_eqlt[2 * q], nlt = c.L.hg_eqlt[2 * q + 1], ngt = g.m - neq - nlt;
    const uint32_t lo[3] = {0u, nlt + ngt, nlt};      // list offsets of the parts L, E, G (sizes <= nlt, nlt + ngt, ngt)
    uint32_t* hl = hg_hole_list(c, g, dk, nlt, ngt);
    const uint64_t ref = elem_key<DBL>(ks, g.s, sv[0]);
    constexpr uint32_t U = HG_CH / 256;
    uint32_t v[U], cl[U], rg[U], rm[U], rh[U];
    uint64_t k[U];
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
        const uint32_t i = a + u * 256 + tid, ic = i < e ? i : a;
        v[u] = sv[ic];
        k[u] = elem_key<DBL>(ks, g.s + ic, v[u]);
        cl[u] = k[u] < ref ? 0u : k[u] == ref ? 1u : 2u;
        rg[u] = ic < nlt ? 0u : ic < nlt + neq ? 1u : 2u;
    }
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
        const bool mis = a + u * 256 + tid < e && cl[u] != rg[u];
        rm[u] = wave_bin_add(cnt, mis, cl[u]);
        rh[u] = wave_bin_add(cnt + 3, mis, rg[u]);
    }
    __syncthreads();
    if (tid < 6) {
        const uint32_t x = cnt[tid];
        cnt[8 + tid] = x ? atomicAdd(&c.L.hg_mc[6 * q + tid], x) : 0u;
    }
    __syncthreads();
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
        const uint32_t i = a + u * 256 + tid;
        if (i < e && cl[u] != rg[u]) {
            const uint32_t km = lo[cl[u]] + cnt[8 + cl[u]] + rm[u];
            dv[km] = v[u];
            if constexpr (DBL) if (cl[u] != 1) dk[km] = k[u];
            hl[lo[rg[u]] + cnt[11 + rg[u]] + rh[u]] = i;
        }
    }
    __syncthreads();
}

// in-place three-way groups: every mover into a hole of its part (the k-th
// mover of a part fills its k-th hole); keys move with the values while
// doubling (the parts L and G are sorted further by them)
template <bool DBL>
__global__ void __launch_bounds__(256) k3_hg_move(Ctx c)
{
    const uint32_t nh = hg_count(c);
    const GridSplit gs = grid_split(nh);
    if (gs.idle) return;
    for (uint32_t q = gs.q0; q < nh; q += gs.gstride) {
        if (c.L.hg_flag[q] != HG_THREE_IP) continue;
        const HgGroup g = hg_group(c.L.hg[q]);
        const KeySrc ks = key_src(c, g.slot, g.par);
        const uint64_t base = (uint64_t)g.slot * c.scr.stride + g.s;
        uint32_t* sv = c.scr.SA + base;               // par 0
        const uint32_t* dv = c.scr.V + base;
        uint64_t* dk = c.kB + base;
        uint64_t* sk = c.kA + base;
        const uint32_t neq = c.L.hg_eqlt[2 * q], nlt = c.L.hg_eqlt[2 * q + 1], ngt = g.m - neq - nlt;
        const uint32_t* hl = hg_hole_list(c, g, dk, nlt, ngt);
        const uint32_t n0 = c.L.hg_mc[6 * q], n1 = c.L.hg_mc[6 * q + 1], n2 = c.L.hg_mc[6 * q + 2];
        const uint32_t lo[3] = {0u, nlt + ngt, nlt};   // as in hg_inplace_lists
        (void)ks;
        for (uint32_t x = gs.slice * 256u + threadIdx.x; x < n0 + n1 + n2; x += gs.per * 256u) {
            const uint32_t part = x < n0 ? 0u : x < n0 + n2 ? 2u : 1u;   // L, G, then E
            const uint32_t kk = part == 0 ? x : part == 2 ? x - n0 : x - n0 - n2;
            const uint32_t j = lo[part] + kk;
            const uint32_t pos = hl[j];
            sv[pos] = dv[j];
            if constexpr (DBL) if (part != 1) sk[pos] = dk[j];
        }
    }
}

// every chunk: its elements to their bins (one global reservation per bin
// and chunk, then LDS cursors)
template <bool DBL>
__global__ void __launch_bounds__(256) k3_hg_scatter(Ctx c)
{
    __shared__ uint32_t cnt[256];
    const uint32_t tid = threadIdx.x;
    const uint32_t nh = hg_count(c);
    if (nh == 0) return;
    const uint32_t total = c.L.hg_pre[nh];
    constexpr uint32_t U = HG_CH / 256;
    for (uint32_t j = blockIdx.x; j < total; j += gridDim.x) {
        const uint32_t q = hg_group_of(c.L.hg_pre, nh, j), ch = j - c.L.hg_pre[q];
        const uint32_t flag = c.L.hg_flag[q];
        if (flag && flag != HG_THREE && flag != HG_THREE_IP) continue;   // uniform: skipped at this level
        const HgGroup g = hg_group(c.L.hg[q]);
        const KeySrc ks = key_src(c, g.slot, g.par);
        const uint64_t base = (uint64_t)g.slot * c.scr.stride + g.s;
        const uint32_t* sv = (g.par ? c.scr.V : c.scr.SA) + base;
        uint32_t* dv = (g.par ? c.scr.SA : c.scr.V) + base;
        uint64_t* dk = (g.par ? c.kA : c.kB) + base;
        uint8_t* dl = DBL && ks.l ? (g.par ? c.lA : c.lB) + base : nullptr;
        uint32_t* cur = c.L.hg_info + (uint64_t)q * 512 + 256;
        cnt[tid] = 0;
        __syncthreads();
        const uint32_t a = ch * HG_CH, e = min(g.m, a + HG_CH);
        if (flag == HG_THREE_IP) {                    // uniform
            hg_inplace_lists<DBL>(c, q, g, ks, sv, dv, dk, a, e, cnt);
            continue;
        }
        uint32_t v[U], d[U], r[U];
        uint64_t k[U];
        const uint64_t ref = flag == HG_THREE ? elem_key<DBL>(ks, g.s, sv[0]) : 0ull;
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) {
            const uint32_t i = a + u * 256 + tid, ic = i < e ? i : a;
            v[u] = sv[ic];
            k[u] = elem_key<DBL>(ks, g.s + ic, v[u]);
            d[u] = flag == HG_THREE ? (k[u] < ref ? 0u : k[u] == ref ? 1u : 2u) : (uint32_t)((k[u] >> g.sh2) & g.dmask);
        }
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) r[u] = wave_bin_add(cnt, a + u * 256 + tid < e, d[u]);
        __syncthreads();
        const uint32_t mine = cnt[tid];
        __syncthreads();
        if (mine) cnt[tid] = atomicAdd(&cur[tid], mine);   // this chunk's range of bin tid
        __syncthreads();
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) {
            const uint32_t i = a + u * 256 + tid;
            if (i < e) {
                const uint32_t p = cnt[d[u]] + r[u];
                dv[p] = v[u];
                if constexpr (DBL) dk[p] = k[u];
                if (dl) dl[p] = ks.l[g.s + i];
            }
        }
        __syncthreads();
    }
}

// final sub-buckets of every huge group: SA, last column, RK, origPtr.  The
// grid's workgroups split over the groups (several per group when there are
// fewer groups than workgroups); a group skipped whole (HG_SKIP_ALL) is
// written from where its elements are, as one run headed at its start.
__global__ void __launch_bounds__(256) k3_hg_final(Ctx c)
{
    __shared__ uint32_t fin_pre[257];
    __shared__ uint32_t scan_sh[5];
    const uint32_t tid = threadIdx.x;
    const uint32_t nh = hg_count(c), G = gridDim.x;
    if (nh == 0) return;
    const uint32_t per = nh >= G ? 1u : G / nh;      // workgroups per group
    const uint32_t gstride = G / per;                 // groups in progress at once
    if (blockIdx.x >= per * gstride) return;
    const uint32_t slice = blockIdx.x % per;
    for (uint32_t q = blockIdx.x / per; q < nh; q += gstride) {
        const uint64_t item = c.L.hg[q];
        if (it_size(item) == 0) continue;
        const HgGroup g = hg_group(item);
        const uint32_t flag = c.L.hg_flag[q];
        if (flag == HG_SKIP_RELABEL) continue;
        const uint64_t so = (uint64_t)g.slot * c.scr.stride, base = so + g.s;
        const KeySrc ks = key_src(c, g.slot, g.par);
        if (flag == HG_THREE_IP) {                    // uniform: in SA already (par 0)
            const uint32_t neq = c.L.hg_eqlt[2 * q], nlt = c.L.hg_eqlt[2 * q + 1], ngt = g.m - neq - nlt;
            const uint32_t rk = c.L.hg_rank[q];
            const uint32_t* sa = c.scr.SA + base;
            if (c.mode && rk != HG_KEEP)
                for (uint32_t p = nlt + slice * 256u + tid; p < nlt + neq; p += per * 256u) c.scr.RK[so + sa[p]] = rk;
            if (slice == 0 && tid < 2) {              // a part of one rotation is final
                const bool one = tid == 0 ? nlt == 1 : ngt == 1;
                if (one) {
                    const uint32_t p = tid == 0 ? 0u : g.m - 1u;
                    const uint32_t v = sa[p];
                    c.scr.LL[base + p] = last_sym(c, g.slot, v);
                    if (c.mode) c.scr.RK[so + v] = g.s + p;
                    if (v == 0) c.blocks[c.b0 + g.slot].orig_ptr = g.s + p;
                }
            }
            continue;
        }
        if (flag == HG_SKIP_ALL) {                    // uniform
            const uint32_t* sv = (g.par ? c.scr.V : c.scr.SA) + base;
            // (a tie group: its last column is written once it resolves --
            // every tie is re-sorted later, or its block is periodic and
            // k_fallback_exact rebuilds that block's last column)
            for (uint32_t p = slice * 256u + tid; p < g.m; p += per * 256u) {
                const uint32_t v = sv[p];
                if (g.par) c.scr.SA[base + p] = v;
                if (c.mode) c.scr.RK[so + v] = g.s;
                if (v == 0) c.blocks[c.b0 + g.slot].orig_ptr = g.s + p;
            }
            continue;
        }
        const uint32_t* dv = (g.par ? c.scr.SA : c.scr.V) + base;
        const uint8_t* dl = ks.l ? (g.par ? c.lA : c.lB) + base : nullptr;
        const uint32_t* info = c.L.hg_info + (uint64_t)q * 512;
        // final bins' sizes (bin end = next bin's start; the last ends at m)
        const uint32_t st = info[tid] & ~HG_FINAL;
        const uint32_t en = tid < 255 ? (info[tid + 1] & ~HG_FINAL) : g.m;
        const uint32_t fsz = (info[tid] & HG_FINAL) ? en - st : 0u;
        uint32_t ftot = 0;
        const uint32_t fp = block_excl_scan_add<uint32_t>(fsz, scan_sh, &ftot);
        fin_pre[tid] = fp;
        if (tid == 255) fin_pre[256] = ftot;
        __syncthreads();
        for (uint32_t x = slice * 256u + tid; x < ftot; x += per * 256u) {
            uint32_t lo = 0, hi = 255;                 // the final bin holding flat index x
            while (lo < hi) {
                const uint32_t mid = (lo + hi + 1) >> 1;
                if (fin_pre[mid] <= x) lo = mid; else hi = mid - 1;
            }
            const uint32_t b0 = info[lo] & ~HG_FINAL;
            const uint32_t p = b0 + (x - fin_pre[lo]);
            const uint32_t v = dv[p];
            if (!g.par) c.scr.SA[base + p] = v;
            const uint32_t be = lo < 255 ? (info[lo + 1] & ~HG_FINAL) : g.m;
            if (be - b0 == 1) c.scr.LL[base + p] = dl ? dl[p] : last_sym(c, g.slot, v);   // ties: once resolved
            if (c.mode) c.scr.RK[so + v] = g.s + b0;
            if (v == 0) c.blocks[c.b0 + g.slot].orig_ptr = g.s + p;
        }
        __syncthreads();
    }
}

// Finish a sorted group: SA, RK, origPtr, tie groups, run count.
// Called by every thread of a wave with (j = sorted position in the group,
// v = rotation, valid, hp = head position of j's run, end = j ends its run,
// lsym = last-column symbol of v).
__device__ __forceinline__ void emit_sorted(const Ctx& c, uint32_t slot, uint32_t s, uint32_t j, uint32_t v,
                                            bool valid, uint32_t hp, bool end, uint32_t& runs_acc, uint32_t lsym)
{
    const uint64_t so = (uint64_t)slot * c.scr.stride;
    if (valid) {
        st_nt(c.scr.SA + so + s + j, v);
        st_nt(c.scr.LL + so + s + j, (uint8_t)lsym);
        if (c.mode) c.scr.RK[so + v] = s + hp;
        if (v == 0) c.blocks[c.b0 + slot].orig_ptr = s + j;
    }
    const bool tie = valid && end && j > hp;
    const uint64_t tb = __ballot(tie);
    if (tb) {
        wave_push(c.L.ctr + C_T0 + c.tsel, c.L.t[c.tsel], tie, mk_item(slot, s + hp, j - hp + 1, 0, 0));
        const uint32_t te = wave_reduce_add<uint32_t>(tie ? j - hp + 1 : 0u);
        if ((threadIdx.x & 63) == 0) atomicAdd(c.L.ctr + C_TS0 + c.tsel, te);
    }
    runs_acc += (uint32_t)__popcll(__ballot(valid && end));
}

// The values half of emit_sorted, for the kernels that reserve their tie-list
// slots once per group (tie_reserve) instead of once per wave and row
__device__ __forceinline__ void emit_vals(const Ctx& c, uint32_t slot, uint32_t s, uint32_t j, uint32_t v, bool valid,
                                          uint32_t hp, uint32_t lsym)
{
    if (valid) {
        const uint64_t so = (uint64_t)slot * c.scr.stride;
        st_nt(c.scr.SA + so + s + j, v);
        st_nt(c.scr.LL + so + s + j, (uint8_t)lsym);
        if (c.mode) c.scr.RK[so + v] = s + hp;
        if (v == 0) c.blocks[c.b0 + slot].orig_ptr = s + j;
    }
}

// First tie-list slot for a group's tcnt tie runs (tcnt: this wave's count,
// uniform per wave): one global atomic per group.  The tie-list counter is
// one address shared by every wave of the launch; a returning atomic per wave
// and row serialised there (text with many short repeats -- narrowPeak --
// pushes millions of tie runs per batch).  NW > 1: every wave of the
// workgroup (one group) calls it; tc/tb: NW + 1 words of LDS.
template <int NW>
__device__ __forceinline__ uint32_t tie_reserve(const Ctx& c, uint32_t tcnt, uint32_t* tc, int wid, int lane)
{
    uint32_t* ctr = c.L.ctr + C_T0 + c.tsel;
    if constexpr (NW == 1) {
        uint32_t base = 0;
        if (lane == 0 && tcnt) base = atomicAdd(ctr, tcnt);
        return (uint32_t)__shfl((int)base, 0, 64);
    } else {
        if (lane == 0) tc[wid] = tcnt;
        __syncthreads();
        if (wid == 0 && lane == 0) {
            uint32_t t = 0;
#pragma unroll
            for (int w = 0; w < NW; ++w) t += tc[w];
            tc[NW] = t ? atomicAdd(ctr, t) : 0u;
        }
        __syncthreads();
        uint32_t base = tc[NW];
        for (int w = 0; w < wid; ++w) base += tc[w];
        return base;
    }
}

// ---------------------------------------------------------------------------
// k3_sort_w: groups of <= 64, packed several to a wave.  Each wave takes
// chunks of 64 consecutive items of its XCD's segment (one item per lane,
// one coalesced load); groups are laid out back to back over the 64 lanes as
// far as they fit, so one round of loads (rotations, then keys) serves them
// all -- text-round tie groups are mostly pairs, one group per wave left 60
// lanes idle and paid a full load round trip per pair.  Every element ranks
// itself among its group's members (keys by lane shuffle), then sorted order
// goes through LDS; heads, ends and tie runs are per group.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t shfl64(uint64_t v, uint32_t src)
{
    const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, (int)src, 64);
    const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), (int)src, 64);
    return ((uint64_t)hi << 32) | lo;
}

// arr[slot] += v over the wave's active lanes, one atomic per distinct slot
// (per-group atomics on one block's counter serialise: a block of 450k tied
// pairs spent ~5 ms per doubling round in them).  Wave-uniform call.
__device__ __forceinline__ void wave_add_slot(uint32_t* arr, bool act, uint32_t slot, uint32_t v)
{
    const uint32_t lane = threadIdx.x & 63;
    uint64_t pend = __ballot(act);
    while (pend) {
        const int l = __ffsll((unsigned long long)pend) - 1;
        const uint32_t s0 = (uint32_t)__shfl((int)slot, l, 64);
        const bool mine = act && slot == s0;
        const uint32_t tot = wave_reduce_add<uint32_t>(mine ? v : 0u);
        if (lane == (uint32_t)l && tot) atomicAdd(&arr[s0], tot);
        pend &= ~__ballot(mine);
    }
}

template <bool DBL>
__global__ void __launch_bounds__(256) k3_sort_w(Ctx c, const uint64_t* __restrict__ items)
{
    __shared__ uint64_t skey[4][W_MAX + 1];
    __shared__ uint32_t sval[4][W_MAX];
    const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    // static assignment: workgroup L works segment L mod 8 (the XCD it runs on);
    // its waves take 64-item chunks of that segment in turn
    // (chunks shrink when the segment has fewer than 64 items per wave, so a
    // small batch spreads over all waves instead of queueing on a few)
    const uint32_t xs8 = blockIdx.x & 7u, wseg = (gridDim.x >> 3) * 4u, w_in = (blockIdx.x >> 3) * 4u + wid;
    const uint32_t seg0 = c.qseg[xs8], seg1 = c.qseg[xs8 + 1];
    const uint32_t per_w = (seg1 - seg0 + wseg - 1) / wseg;
    const uint32_t ch = per_w >= 64u ? 64u : (per_w ? per_w : 1u);
    for (uint32_t cb = seg0 + w_in * ch; cb < seg1; cb += wseg * ch) {
        const uint32_t cnt = seg1 - cb < ch ? seg1 - cb : ch;
        const uint64_t myitem = lane < cnt ? items[cb + lane] : 0ull;
        const uint32_t msz = lane < cnt ? it_size(myitem) : 0u;
        for (uint32_t done = 0; done < cnt;) {
            // the groups done.. whose sizes sum to <= 64 (the first always fits)
            const uint32_t sz = (lane >= done && lane < cnt) ? msz : 0u;
            const uint32_t incl = wave_incl_scan_add(sz);
            const bool take = lane >= done && lane < cnt && incl <= 64u;
            const uint32_t ng = (uint32_t)__popcll(__ballot(take));
            const uint32_t off = incl - sz;
            const uint32_t total = (uint32_t)__shfl((int)incl, (int)(done + ng - 1), 64);
            const uint64_t smask = wave_reduce_or64(take ? (1ull << off) : 0ull);
            const bool valid = lane < total;
            const uint64_t upto = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);
            const uint32_t gi = valid ? done + (uint32_t)__popcll(smask & upto) - 1u : done;
            const uint64_t item = shfl64(myitem, gi);
            const uint32_t goff = (uint32_t)__shfl((int)off, (int)gi, 64);   // every lane: gi may be past `total`
            const uint32_t gstart = valid ? goff : 0u;
            const uint32_t slot = it_slot(item), s = it_start(item), m = it_size(item), par = it_par(item);
            const uint32_t j = valid ? lane - gstart : 0u;
            const uint32_t* sv = (par ? c.scr.V : c.scr.SA) + (uint64_t)slot * c.scr.stride + s;
            const KeySrc ks = key_src(c, slot, par);
            const uint32_t v = ld_nt(sv + j);
            uint32_t ls;
            uint64_t k = elem_key<DBL>(c, ks, slot, s + j, v, ls);
            if (!valid) k = ~0ull;
            // rank among the group's members (lanes gstart .. gstart + m - 1):
            // scalar broadcasts when the pass holds one group, lane shuffles otherwise
            uint32_t r = 0;
            if (ng == 1) {
#if STARCH_W_UNROLL
#pragma unroll 4
#endif
                for (uint32_t q = 0; q < total; ++q) {
                    const uint64_t kq = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(k >> 32), (int)q) << 32) |
                                        (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)k, (int)q);
                    r += (kq < k || (kq == k && q < j)) ? 1u : 0u;
                }
            } else {
                const uint32_t maxm = wave_reduce_max(valid ? m : 0u);
#if STARCH_W_UNROLL
#pragma unroll 4
#endif
                for (uint32_t q = 0; q < maxm; ++q) {
                    const bool in = valid && q < m;
                    const uint64_t kq = shfl64(k, in ? gstart + q : lane);
                    r += (in && (kq < k || (kq == k && q < j))) ? 1u : 0u;
                }
            }
            wave_sync_lds3();                            // the previous pass's reads are done
            if (valid) { skey[wid][gstart + r] = k; sval[wid][gstart + r] = v | (ls << 24); }
            wave_sync_lds3();
            const uint64_t key = valid ? skey[wid][lane] : 0;
            const uint32_t val = valid ? sval[wid][lane] : 0;
            const bool head = valid && (j == 0 || skey[wid][lane - 1] != key);
            const bool end = valid && (j + 1 == m || skey[wid][lane + 1] != key);
            const uint32_t hp = wave_incl_scan_max<uint32_t>(head ? lane : 0u) - gstart;   // a group start is a head
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // SA reads done before the writes
            uint32_t runs = 0;
            emit_sorted(c, slot, s, j, val & 0xFFFFFFu, valid, hp, end, runs, val >> 24);
            if (c.mode) {                                // runs per group, by its first lane
                const uint64_t em = __ballot(end);
                const uint64_t gm = (m >= 64 ? ~0ull : ((1ull << m) - 1ull)) << gstart;
                wave_add_slot(c.L.runs, valid && j == 0, slot, (uint32_t)__popcll(em & gm));
            }
            done += ng;
        }
    }
}

// ---------------------------------------------------------------------------
// k3_sort_lds<NW, E>: groups of <= NW*64*E rotations sorted by NW waves
// (NW = 1: four independent wave-private sorts per workgroup, no workgroup
// barrier; NW = 4: one group per workgroup).  Persistent over a binned list.
// Every group's keys share at least their top 12 bits (the bucket digit, the
// partition digits, or unused high bits); dropping them leaves room for the
// group-local index below the key: (key << IDXB) | index is unique and
// ordered like the key, so each exchange moves one u64 per element through
// LDS and ranking is one 64-bit compare per pair.
// Primary path: one MSD digit (the DB bits below the highest varying bit),
// then every element ranks itself inside its sub-bucket by comparison; a
// second digit for sub-buckets above LIMIT.  Otherwise: stable LSD radix over
// the varying 8-bit digits (8 ballots find a lane's digit peers; one lane per
// peer set adds the set's size to the wave's counter with a returning LDS
// atomic).
// ---------------------------------------------------------------------------
// rank of key kj among positions [rs, re) of xk.  Keys are (key << IDXB) |
// group index: unique, so one 64-bit compare orders them (ties of the key
// broken by index)
#ifndef STARCH_RANK_UNROLL
#define STARCH_RANK_UNROLL 4   // keys in flight per step: 4 (cfg2 sort 22.8 -> 21.5-21.9 ms, cfg4 107.6 -> 104.1-104.4); 8 no better; 0 one at a time
#endif
__device__ __forceinline__ uint32_t rank_in(const uint64_t* xk, uint32_t rs, uint32_t re, uint64_t kj)
{
    uint32_t r = 0;
    uint32_t q = rs;
    if constexpr (STARCH_RANK_UNROLL >= 8) {
        for (; q + 8 <= re; q += 8) {
            uint64_t x[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) x[i] = xk[q + i];
#pragma unroll
            for (int i = 0; i < 8; ++i) r += x[i] < kj ? 1u : 0u;
        }
    }
    if constexpr (STARCH_RANK_UNROLL != 0) {
        for (; q + 4 <= re; q += 4) {
            const uint64_t a = xk[q], b = xk[q + 1], c2 = xk[q + 2], d = xk[q + 3];
            r += (a < kj ? 1u : 0u) + (b < kj ? 1u : 0u) + (c2 < kj ? 1u : 0u) + (d < kj ? 1u : 0u);
        }
    }
    for (; q < re; ++q) r += xk[q] < kj ? 1u : 0u;
    return r;
}

template <int NW>
__device__ __forceinline__ void gsync()
{
    if constexpr (NW == 1) wave_sync_lds3();
    else __syncthreads();
}

template <int E>
struct GrpIn {                 // one group's inputs, as loaded
    uint64_t item;
    KeySrc ks;
    uint32_t v[E];
    uint32_t v0;
    uint64_t kx[E];            // keys (PSS rounds: the first raw key word until grp_finish_keys)
    uint32_t ls[E];            // last-column symbols (PSS rounds: the first raw 32-bit window word)
    uint64_t k0;
    uint64_t kb[E];            // PSS rounds: the second raw key word
    uint32_t lb[E];            // ... and the second raw window word of the last-column symbol
    uint64_t k0b;
    bool one;                  // PSS round 0, B in {1,2,4,5,6,8}: kx/kb = ONE 16-B load holding the symbol and the key
};

// loads of a group that does not exist (ok false) go to element 0 of slot 0's
// SA, which always exists; their results are never used
template <int NW, int E>
__device__ __forceinline__ void grp_load_vals(const Ctx& c, GrpIn<E>& x, bool ok, int wid, int lane)
{
    if (!ok) x.item = mk_item(0, 0, 1, 0, 0);
    const uint32_t slot = it_slot(x.item), s = it_start(x.item), m = it_size(x.item), par = it_par(x.item);
    const uint32_t* sv = (par ? c.scr.V : c.scr.SA) + (uint64_t)slot * c.scr.stride + s;
    x.ks = key_src(c, slot, par);
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const uint32_t i = (uint32_t)(wid * 64 * E + e * 64 + lane);
        x.v[e] = ld_nt(sv + (i < m ? i : 0u));
    }
    x.v0 = sv[0];
}

// PSS rounds: the key of rotation r is stream bits [(r + off) * B, + kbits) and its
// last-column symbol bits [(r - 1) * B, + B) (mod n).  grp_load_keys only issues
// the loads (two u64 words for the key, two 32-bit words for the symbol, in the
// stream's MSB-first order: the 32-bit word j of the stream sits at u32 index
// j ^ 1 of the little-endian u64 words); grp_finish_keys combines them one group
// later, so the random PSS reads overlap the current group's sort instead of
// being waited on where they are issued.
__device__ __forceinline__ uint32_t pss_rr(const KeySrc& ks, uint32_t r)
{
    const uint32_t rr = r + ks.off;
    return rr >= ks.n ? rr - ks.n : rr;
}
__device__ __forceinline__ uint32_t pss_pr(const KeySrc& ks, uint32_t r) { return r ? r - 1u : ks.n - 1u; }

#ifndef STARCH_DEFER
#define STARCH_DEFER 1     // deferred key combination: 0 never, 1 one-wave sorts only (measured best), 2 all
#endif
template <int NW, bool DBL>
constexpr bool defer_keys() { return !DBL && (STARCH_DEFER == 2 || (STARCH_DEFER == 1 && NW == 1)); }

template <int NW, int E, bool DBL>
__device__ __forceinline__ void grp_load_keys(const Ctx& c, GrpIn<E>& x, int wid, int lane)
{
    const uint32_t s = it_start(x.item), m = it_size(x.item), slot = it_slot(x.item);
    if constexpr (!defer_keys<NW, DBL>()) {
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const uint32_t i = (uint32_t)(wid * 64 * E + e * 64 + lane);
            x.kx[e] = elem_key<DBL>(c, x.ks, slot, s + (i < m ? i : 0u), x.v[e], x.ls[e]);
        }
        x.k0 = elem_key<DBL>(x.ks, s, x.v0);
    } else {
        const uint64_t* __restrict__ w = x.ks.pss;
        const uint32_t* __restrict__ w32 = reinterpret_cast<const uint32_t*>(w);
        const uint32_t B = x.ks.B;
        // round 0: the last-column symbol's B bits sit right before the key's KB
        // bits, and for these B the B + KB bits after the symbol's bit offset
        // within its word (a multiple of B <= 64 - B ... 63) never pass the
        // next word: one 16-byte load per element instead of four
        x.one = x.ks.off == 0 && (B == 1 || B == 2 || B == 4 || B == 5 || B == 6 || B == 8);
        if (x.one) {
#pragma unroll
            for (int e = 0; e < E; ++e) {
                const uint32_t r = x.v[e];
                const uint64_t q = ((uint64_t)(r ? r - 1u : 0u) * B) >> 6;
                const uint4 kv = *reinterpret_cast<const uint4*>(w + q);
                x.kx[e] = ((uint64_t)kv.y << 32) | kv.x;
                x.kb[e] = ((uint64_t)kv.w << 32) | kv.z;
                if (r == 0) {                      // rotation 0: its symbol is the block's last
                    const uint64_t j = ((uint64_t)(x.ks.n - 1u) * B) >> 5;
                    x.ls[e] = w32[j ^ 1u];
                    x.lb[e] = w32[(j + 1u) ^ 1u];
                }
            }
        } else {
#pragma unroll
            for (int e = 0; e < E; ++e) {
                const uint64_t q = ((uint64_t)pss_rr(x.ks, x.v[e]) * B) >> 6;
                x.kx[e] = w[q];
                x.kb[e] = w[q + 1];
                const uint64_t j = ((uint64_t)pss_pr(x.ks, x.v[e]) * B) >> 5;
                x.ls[e] = w32[j ^ 1u];
                x.lb[e] = w32[(j + 1u) ^ 1u];
            }
        }
        const uint64_t q0 = ((uint64_t)pss_rr(x.ks, x.v0) * x.ks.B) >> 6;
        x.k0 = w[q0];
        x.k0b = w[q0 + 1];
    }
}

template <int NW, int E, bool DBL>
__device__ __forceinline__ void grp_finish_keys(GrpIn<E>& x)
{
    if constexpr (defer_keys<NW, DBL>()) {
        const KeySrc& ks = x.ks;
        if (x.one) {
            const uint32_t B = ks.B;
#pragma unroll
            for (int e = 0; e < E; ++e) {
                const uint32_t r = x.v[e];
                const uint64_t A = x.kx[e], W = x.kb[e];
                if (r) {
                    const uint32_t p0 = (uint32_t)(((uint64_t)(r - 1u) * B) & 63u), pk = p0 + B;
                    x.ls[e] = (uint32_t)(((A << p0) | ((W >> 1) >> (63u - p0))) >> (64u - B));
                    const uint64_t win = pk >= 64u ? (W << (pk - 64u)) : ((A << pk) | ((W >> 1) >> (63u - pk)));
                    x.kx[e] = win >> (64u - ks.kbits);
                } else {
                    x.kx[e] = A >> (64u - ks.kbits);
                    const uint32_t pl = (uint32_t)(((uint64_t)(ks.n - 1u) * B) & 31u);
                    const uint64_t lw = ((uint64_t)x.ls[e] << 32) | x.lb[e];
                    x.ls[e] = (uint32_t)((lw << pl) >> (64u - B));
                }
            }
        } else {
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const uint32_t p = (uint32_t)(((uint64_t)pss_rr(ks, x.v[e]) * ks.B) & 63u);
            const uint64_t v = (x.kx[e] << p) | ((x.kb[e] >> 1) >> (63u - p));
            x.kx[e] = v >> (64u - ks.kbits);
            const uint32_t pl = (uint32_t)(((uint64_t)pss_pr(ks, x.v[e]) * ks.B) & 31u);
            const uint64_t lw = ((uint64_t)x.ls[e] << 32) | x.lb[e];
            x.ls[e] = (uint32_t)((lw << pl) >> (64u - ks.B));
        }
        }
        const uint32_t p0 = (uint32_t)(((uint64_t)pss_rr(ks, x.v0) * ks.B) & 63u);
        const uint64_t v0 = (x.k0 << p0) | ((x.k0b >> 1) >> (63u - p0));
        x.k0 = v0 >> (64u - ks.kbits);
    }
}

// register budget (waves per SIMD) of the sort kernels: keeps a few groups
// resident per CU while their loads are in flight
#ifndef STARCH_WPE_GRP
#define STARCH_WPE_GRP 1
#endif
#ifndef STARCH_WPE_M2
#define STARCH_WPE_M2 3
#endif
#ifndef STARCH_WPE_S
#define STARCH_WPE_S STARCH_WPE_GRP   // the S class (one wave, E = 2)
#endif
#ifndef STARCH_WPE_M1
#define STARCH_WPE_M1 1
#endif
#ifndef STARCH_WPE_M0
#define STARCH_WPE_M0 6   // M0 (257..512): 6 waves per SIMD (cfg2 sort -0.5 ms, cfg4 -3 ms; profiles/r03_v5/sweep_*_m0w6.json)
#endif
constexpr int sort_wpe(int NW, int E)
{
    return NW == 4 && E == 8   ? STARCH_WPE_M2
           : NW == 4 && E == 4 ? STARCH_WPE_M1
           : NW == 4 && E == 2 ? STARCH_WPE_M0
           : (NW == 1 ? (E == 2 ? STARCH_WPE_S : STARCH_WPE_GRP) : 1);
}

// STARCH_SORT_PROF (timing experiment, dev builds only): per-wave shader-clock
// time of the sorts' phases, summed over the launch: k3_sort_grp into
// g_sprof, the workgroup sorts k3_sort_lds<8|16, 4> (M2/M3) and <4, 4> (M1)
// into g_sprof2
#ifdef STARCH_SORT_PROF
__device__ unsigned long long g_sprof[16];
__device__ unsigned long long g_sprof2[16];
#define SPROF(v) const uint64_t v = __builtin_readcyclecounter()
#define SPACC(i, a, b) pacc[i] += (b) - (a)
#else
#define SPROF(v)
#define SPACC(i, a, b)
#endif

template <int NW, int E, bool DBL>
__global__ void __launch_bounds__(NW > 4 ? 64 * NW : 256) __attribute__((amdgpu_waves_per_eu(sort_wpe(NW, E))))
k3_sort_lds(Ctx c, const uint64_t* __restrict__ items,
                                                    const uint32_t* __restrict__ hard_n)
{
    constexpr int IPW = NW >= 4 ? 1 : 4 / NW;      // groups per workgroup
    constexpr int NWV = IPW * NW;                  // waves per workgroup
    constexpr int CAP = NW * 64 * E;
    constexpr int IDXB = CAP <= 256 ? 8 : 12;      // packed local index bits
    constexpr int KEYB = 64 - IDXB;
    constexpr uint64_t KMASK = (1ull << KEYB) - 1ull;
    constexpr int DPT = NW >= 4 ? 1 : 256 / (64 * NW);   // digits per thread in the offset scan (NW > 4: threads 0..255)
    static_assert(CAP <= (1 << IDXB), "index does not fit");
#ifndef STARCH_M2_DB
#define STARCH_M2_DB 11
#endif
    constexpr int DB = CAP <= 128 ? 7 : (CAP <= 256 ? 8 : (CAP <= 1024 ? 10 : (CAP == 2048 ? STARCH_M2_DB : 11)));   // MSD digit bits
    constexpr int NBIN = 1 << DB;
    constexpr int T = NW * 64;
    constexpr int BPT = NBIN / T;                  // bins per thread
#ifndef STARCH_LIM_NUM
#define STARCH_LIM_NUM 256
#endif
#ifndef STARCH_LIM2_NUM
#define STARCH_LIM2_NUM 512
#endif
    constexpr uint32_t LIMIT = STARCH_LIM_NUM / E; // largest sub-bucket ranked by comparison
    __shared__ uint64_t xk_all[IPW][CAP];
    __shared__ uint32_t vb_all[IPW][CAP];          // rotations by group index
    // LDS is what caps residency here: sub-bucket starts as u16 (positions <=
    // CAP), and the scatter cursors share their words with the LSD path's
    // per-wave digit counters (the LSD path runs only after the MSD attempt)
    __shared__ uint16_t bst_all[IPW][NBIN + 2];   // sub-bucket starts
    constexpr int UR = NBIN > 256 * NW ? NBIN : 256 * NW;
    __shared__ uint32_t ur_all[IPW][UR];          // scatter cursors | LSD digit counters
    __shared__ uint32_t sc_all[IPW][NW + 1];
    constexpr int NB2 = NW == 1 ? 256 : 1024;      // second-digit bins
    constexpr uint32_t LIMIT2 = STARCH_LIM2_NUM / E;   // largest second-level sub-bucket ranked by comparison
    __shared__ uint32_t c2_all[IPW][NB2 + 1];
    __shared__ uint32_t sc2_all[IPW][NW + 1];
    __shared__ uint64_t red_all[NWV];
    __shared__ uint32_t wmax_all[NWV];
    __shared__ uint32_t flag_all[NWV];
    __shared__ uint32_t tc_all[NW + 1 > 5 ? NW + 1 : 5];
    uint32_t tacc = 0;                             // tied elements pushed (flushed at exit)
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int g = wave / NW, wid = wave % NW, w0 = g * NW;
    uint64_t* xk = xk_all[g];
    uint32_t* wcnt = ur_all[g] + wid * 256;
    uint32_t* sc = sc_all[g];
    const uint64_t lt = lanemask_lt();
    // binned list: dynamic pops from the XCD's queue (a workgroup per group for
    // NW = 4, a wave per group for NW = 1), so an XCD's groups are worked in
    // list order (neighbouring groups share a block's PSS in its L2).
    // hard_n: an unbinned list of *hard_n groups, grid-strided.
    constexpr uint32_t NONE = 0xFFFFFFFFu;
    __shared__ uint32_t qs[8];
    __shared__ uint32_t job_sh;
    const uint32_t xs = xcc_id();
    if (!hard_n) load_qsizes_binned(c, qs);
    const uint32_t nwk = gridDim.x * (uint32_t)IPW;
    const uint32_t e_end = hard_n ? *hard_n : 0u;
    WaveQueue<1> wq;
    uint32_t it_s = blockIdx.x * (uint32_t)IPW + (uint32_t)g;   // hard_n walk
#ifndef STARCH_LDS_DYN
#define STARCH_LDS_DYN 0
#endif
    const uint32_t xs8 = blockIdx.x & 7u;                        // static: segment L mod 8
    const uint32_t s_end = hard_n ? e_end : c.qseg[xs8 + 1];
    const uint32_t s_nwk = hard_n ? nwk : (gridDim.x >> 3) * (uint32_t)IPW;
    if (!hard_n) it_s = c.qseg[xs8] + (blockIdx.x >> 3) * (uint32_t)IPW + (uint32_t)g;
    auto next_item = [&]() -> uint32_t {
        if (hard_n || !STARCH_LDS_DYN) {
            const uint32_t r = it_s < s_end ? it_s : NONE;
            it_s += s_nwk;
            return r;
        }
        if constexpr (NW == 1) {
            return wq.next(c.qhead, qs, c.qseg, xs);
        } else {
            const uint32_t j = wg_pop(c, qs, &job_sh, xs);
            return j == NONE ? NONE : c.qseg[j >> 28] + (j & 0x0FFFFFFFu);
        }
    };
    // software pipeline (as k3_sort_grp): while a group sorts, the next
    // group's keys are in flight, and the rotations of the one after it
    uint32_t it = next_item();
    uint32_t it1 = it != NONE ? next_item() : NONE;
    GrpIn<E> cur, nxt;
    cur.item = it != NONE ? items[it] : 0ull;
    grp_load_vals<NW, E>(c, cur, it != NONE, wid, lane);
    grp_load_keys<NW, E, DBL>(c, cur, wid, lane);
    nxt.item = it1 != NONE ? items[it1] : 0ull;
    grp_load_vals<NW, E>(c, nxt, it1 != NONE, wid, lane);
#ifdef STARCH_SORT_PROF
    uint64_t pacc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif
    while (it != NONE) {
    SPROF(t0);
    const uint64_t item = cur.item;
    const uint32_t slot = it_slot(item), s = it_start(item), m = it_size(item);
    grp_finish_keys<NW, E, DBL>(cur);
    gsync<NW>();                                   // the previous group's LDS reads are done

    uint64_t k[E];
    uint64_t diff = 0;
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const uint32_t i = (uint32_t)(wid * 64 * E + e * 64 + lane);
        if (i < m) {
            diff |= cur.kx[e] ^ cur.k0;
            k[e] = ((cur.kx[e] & KMASK) << IDXB) | i;
            vb_all[g][i] = cur.v[e] | (cur.ls[e] << 24);
        } else {
            k[e] = ~0ull;                              // pads: max key, last in stable order
        }
    }
    grp_load_keys<NW, E, DBL>(c, nxt, wid, lane);     // next group's keys (its rotations: one group ago)
    diff = wave_reduce_or64(diff);
    if constexpr (NW > 1) {
        if (lane == 0) red_all[wave] = diff;
        __syncthreads();
        diff = 0;
#pragma unroll
        for (int w = 0; w < NW; ++w) diff |= red_all[w0 + w];
    }
    if ((diff >> KEYB) && tid % (64 * NW) == 0) atomicOr(&c.L.ctr[C_ERR], 1u);   // top bits not shared
    SPROF(t1);
    SPACC(0, t0, t1);

    bool moved = false;
    const uint64_t kdiff = diff & KMASK;
    if (kdiff) {
        uint16_t* bst = bst_all[g];
        uint32_t* bcur = ur_all[g];
        const int tg = wid * 64 + lane;
        const int hb = 63 - __clzll((long long)kdiff);
        const int lo = hb + 1 - DB > 0 ? hb + 1 - DB : 0;
        for (int q = tg; q < NBIN; q += T) bcur[q] = 0;
        gsync<NW>();
        uint32_t dg[E];
#pragma unroll
        for (int e = 0; e < E; ++e) {
            dg[e] = (uint32_t)((k[e] >> (lo + IDXB)) & (uint64_t)(NBIN - 1));
            if ((uint32_t)(wid * 64 * E + e * 64 + lane) < m) atomicAdd(&bcur[dg[e]], 1u);
        }
        gsync<NW>();
        uint32_t loc[BPT], sum = 0, mx = 0;
#pragma unroll
        for (int q = 0; q < BPT; ++q) {
            loc[q] = bcur[tg * BPT + q];
            sum += loc[q];
            mx = loc[q] > mx ? loc[q] : mx;
        }
        const uint32_t incl = wave_incl_scan_add(sum);
        uint32_t run = incl - sum;
        mx = wave_reduce_max(mx);
        if constexpr (NW > 1) {
            if (lane == 63) sc[wid] = incl;
            if (lane == 0) wmax_all[wave] = mx;
            __syncthreads();
            for (int w = 0; w < wid; ++w) run += sc[w];
            mx = 0;
            for (int w = 0; w < NW; ++w) mx = wmax_all[w0 + w] > mx ? wmax_all[w0 + w] : mx;
        }
        // rank every element inside its final sub-bucket [rs, re) by comparison
        // (p = its scatter position: the tie-break), then move keys into place
        // rank in digit order: position j holds kj, whose final sub-bucket
        // [rs, re) range_of() recomputes from the key (lanes of a row mostly
        // share a sub-bucket: equal trip counts, broadcast LDS reads); then
        // move keys into place
        auto rank_place = [&](auto&& range_of) {
            uint32_t p[E];
#pragma unroll
            for (int e = 0; e < E; ++e) {
                const uint32_t j = (uint32_t)(wid * 64 * E + e * 64 + lane);
                p[e] = j;                          // pads keep the tail
                if (j < m) {
                    const uint64_t kj = xk[j];
                    uint32_t rs, re;
                    range_of(kj, rs, re);
                    p[e] = rs + rank_in(xk, rs, re, kj);
                    k[e] = kj;
                }
            }
            gsync<NW>();
#pragma unroll
            for (int e = 0; e < E; ++e) xk[p[e]] = k[e];
            gsync<NW>();
#pragma unroll
            for (int e = 0; e < E; ++e) k[e] = xk[wid * 64 * E + e * 64 + lane];
        };
#ifdef STARCH_SORT_PROF
        pacc[1] += __builtin_readcyclecounter() - t1;
#endif
        if (mx <= LIMIT) {                         // uniform per group
#pragma unroll
            for (int q = 0; q < BPT; ++q) { bst[tg * BPT + q] = run; bcur[tg * BPT + q] = run; run += loc[q]; }
            if (tg == T - 1) bst[NBIN] = run;
            gsync<NW>();
#pragma unroll
            for (int e = 0; e < E; ++e)
                if ((uint32_t)(wid * 64 * E + e * 64 + lane) < m) xk[atomicAdd(&bcur[dg[e]], 1u)] = k[e];
            gsync<NW>();
            rank_place([&](uint64_t kj, uint32_t& rs, uint32_t& re) {
                const uint32_t d = (uint32_t)((kj >> (lo + IDXB)) & (uint64_t)(NBIN - 1));
                rs = bst[d];
                re = bst[d + 1];
#ifdef STARCH_SORT_STATS
                atomicAdd(&c.L.ctr[C_STW], re - rs);
#endif
            });
#ifdef STARCH_SORT_STATS
            if (tid % (64 * NW) == 0) atomicAdd(&c.L.ctr[C_STA], 1u);
#endif
            moved = true;
        } else if (lo > 0) {
            // Second MSD digit for the sub-buckets larger than LIMIT: the w2 bits
            // right below the first digit, counted per (big sub-bucket, digit)
            // bin; bins are numbered in key order, so one exclusive scan places
            // them all.  Sub-buckets <= LIMIT keep their first-digit place.
            uint32_t* c2 = c2_all[g];
            uint32_t* sc2 = sc2_all[g];
            uint32_t nbl = 0;
#pragma unroll
            for (int q = 0; q < BPT; ++q) nbl += loc[q] > LIMIT ? 1u : 0u;
            const uint32_t binc = wave_incl_scan_add(nbl);
            uint32_t bb = binc - nbl, nbig = 0;
            if constexpr (NW > 1) {
                if (lane == 63) sc2[wid] = binc;
                __syncthreads();
                for (int w = 0; w < NW; ++w) { if (w < wid) bb += sc2[w]; nbig += sc2[w]; }
            } else {
                nbig = (uint32_t)__builtin_amdgcn_readlane((int)binc, 63);
            }
            uint32_t w2 = 0;
#ifndef STARCH_W2_MAX
#define STARCH_W2_MAX 6
#endif
            while (w2 < STARCH_W2_MAX && (nbig << (w2 + 1)) <= (uint32_t)NB2) ++w2;
            if (w2 > (uint32_t)lo) w2 = (uint32_t)lo;
            const int lo2 = lo - (int)w2;
            const uint32_t nb2 = nbig << w2;
#pragma unroll
            for (int q = 0; q < BPT; ++q) {
                bst[tg * BPT + q] = run;
                bcur[tg * BPT + q] = loc[q] > LIMIT ? (0x80000000u | ((bb++) << w2)) : run;
                run += loc[q];
            }
            if (tg == T - 1) bst[NBIN] = run;
            for (uint32_t q = (uint32_t)tg; q < nb2; q += T) c2[q] = 0;
            gsync<NW>();
            uint32_t b2[E];
#pragma unroll
            for (int e = 0; e < E; ++e) {
                b2[e] = ~0u;
                if ((uint32_t)(wid * 64 * E + e * 64 + lane) < m) {
                    const uint32_t x = bcur[dg[e]];
                    if (x >> 31) {
                        b2[e] = (x & 0x7FFFFFFFu) + (uint32_t)((k[e] >> (lo2 + IDXB)) & ((1ull << w2) - 1ull));
                        atomicAdd(&c2[b2[e]], 1u);
                    }
                }
            }
            gsync<NW>();
            constexpr int BPT2 = (NB2 + T - 1) / T;
            uint32_t l2[BPT2], s2 = 0, m2 = 0;
#pragma unroll
            for (int q = 0; q < BPT2; ++q) {
                const uint32_t ix = (uint32_t)(tg * BPT2 + q);
                l2[q] = ix < nb2 ? c2[ix] : 0u;
                s2 += l2[q];
                m2 = l2[q] > m2 ? l2[q] : m2;
            }
            const uint32_t inc2 = wave_incl_scan_add(s2);
            uint32_t r2 = inc2 - s2;
            m2 = wave_reduce_max(m2);
            if constexpr (NW > 1) {
                __syncthreads();                   // sc2 reads (nbig) done
                if (lane == 63) sc2[wid] = inc2;
                if (lane == 0) wmax_all[wave] = m2;
                __syncthreads();
                for (int w = 0; w < wid; ++w) r2 += sc2[w];
                for (int w = 0; w < NW; ++w) m2 = wmax_all[w0 + w] > m2 ? wmax_all[w0 + w] : m2;
            }
#pragma unroll
            for (int q = 0; q < BPT2; ++q) {
                const uint32_t ix = (uint32_t)(tg * BPT2 + q);
                if (ix < nb2) c2[ix] = r2;
                r2 += l2[q];
            }
            gsync<NW>();
            if (m2 <= LIMIT2) {                    // uniform per group
                // c2 = bin starts among the big sub-buckets' elements; an
                // element's place: its sub-bucket's start + (bin cursor - the
                // start of the sub-bucket's first bin)
                uint32_t sb[E];
#pragma unroll
                for (int e = 0; e < E; ++e) sb[e] = b2[e] != ~0u ? c2[bcur[dg[e]] & 0x7FFFFFFFu] : 0u;
                gsync<NW>();
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    if ((uint32_t)(wid * 64 * E + e * 64 + lane) < m) {
                        const uint32_t p = b2[e] != ~0u ? bst[dg[e]] + atomicAdd(&c2[b2[e]], 1u) - sb[e]
                                                        : atomicAdd(&bcur[dg[e]], 1u);
                        xk[p] = k[e];
                    }
                }
                gsync<NW>();
                // after the scatter c2[b] = end of bin b = start of bin b + 1;
                // big sub-buckets still carry their tag in bcur
                rank_place([&](uint64_t kj, uint32_t& rs, uint32_t& re) {
                    const uint32_t d = (uint32_t)((kj >> (lo + IDXB)) & (uint64_t)(NBIN - 1));
                    const uint32_t x = bcur[d];
                    if (x >> 31) {
                        const uint32_t base = x & 0x7FFFFFFFu;
                        const uint32_t b = base + (uint32_t)((kj >> (lo2 + IDXB)) & ((1ull << w2) - 1ull));
                        const uint32_t s0 = base ? c2[base - 1] : 0u;
                        rs = bst[d] + (b ? c2[b - 1] : 0u) - s0;
                        re = bst[d] + c2[b] - s0;
                    } else {
                        rs = bst[d];
                        re = bst[d + 1];
                    }
                });
                moved = true;
                if (tg == 0) atomicAdd(&c.L.ctr[C_DBG2], 1u);
            }
        } else {
            gsync<NW>();                           // bcur/sc reads done before the LSD passes
        }
    }
    SPROF(t3);
    SPACC(2, t1, t3);
    if (!moved && kdiff && tid % (64 * NW) == 0) atomicAdd(&c.L.ctr[C_DBGL], 1u);
#ifdef STARCH_SORT_STATS
    if (tid % (64 * NW) == 0) { atomicAdd(&c.L.ctr[C_STG], 1u); atomicAdd(&c.L.ctr[C_STE], m); }
#endif
    bool lsd_moved = false;
    for (int dbit = 0; dbit < KEYB && !moved; dbit += 8) {
        if ((kdiff >> dbit & 0xffull) == 0) continue;    // uniform per group
        for (int q = lane; q < 256; q += 64) wcnt[q] = 0;
        wave_sync_lds3();
        uint32_t dg[E], rk[E], ld[E], ret[E];
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const uint32_t d = (uint32_t)((k[e] >> (dbit + IDXB)) & 255u);
            uint64_t peers = ~0ull;
#pragma unroll
            for (int bb = 0; bb < 8; ++bb) {
                const uint64_t bal = __ballot((d >> bb) & 1u);
                peers &= ((d >> bb) & 1u) ? bal : ~bal;
            }
            const uint32_t leader = (uint32_t)__ffsll((unsigned long long)peers) - 1u;
            dg[e] = d;
            ld[e] = leader;
            rk[e] = (uint32_t)__popcll(peers & lt);
            ret[e] = 0;
            if ((uint32_t)lane == leader) ret[e] = atomicAdd(&wcnt[d], (uint32_t)__popcll(peers));
        }
#pragma unroll
        for (int e = 0; e < E; ++e) rk[e] += (uint32_t)__shfl((int)ret[e], (int)ld[e], 64);
        gsync<NW>();
        {   // digit offsets: base(d) + counts of earlier waves, in place
            const int t = wid * 64 + lane;
            const bool has = t * DPT < 256;
            uint32_t loc[DPT], sum = 0;
#pragma unroll
            for (int q = 0; q < DPT; ++q) {
                uint32_t a = 0;
#pragma unroll
                for (int w = 0; w < NW; ++w) a += has ? ur_all[g][w * 256 + t * DPT + q] : 0u;
                loc[q] = a;
                sum += a;
            }
            const uint32_t incl = wave_incl_scan_add(sum);
            uint32_t run = incl - sum;
            if constexpr (NW > 1) {
                if (lane == 63) sc[wid] = incl;
                __syncthreads();
                for (int w = 0; w < wid; ++w) run += sc[w];
            }
#pragma unroll
            for (int q = 0; q < DPT && has; ++q) {
                uint32_t r = run;
#pragma unroll
                for (int w = 0; w < NW; ++w) {
                    const uint32_t xx = ur_all[g][w * 256 + t * DPT + q];
                    ur_all[g][w * 256 + t * DPT + q] = r;
                    r += xx;
                }
                run += loc[q];
            }
        }
        gsync<NW>();
#pragma unroll
        for (int e = 0; e < E; ++e) xk[rk[e] + wcnt[dg[e]]] = k[e];
        gsync<NW>();
#pragma unroll
        for (int e = 0; e < E; ++e) k[e] = xk[wid * 64 * E + e * 64 + lane];
        lsd_moved = true;
#ifdef STARCH_SORT_STATS
        if (tid % (64 * NW) == 0) atomicAdd(&c.L.ctr[C_STLP], 1u);
#endif
    }
    moved |= lsd_moved;
    if (!moved) {
#pragma unroll
        for (int e = 0; e < E; ++e) xk[wid * 64 * E + e * 64 + lane] = k[e];
    }
    gsync<NW>();
    // runs of equal keys in sorted order j = wid*64*E + e*64 + lane
    bool tie_here = false;
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const uint32_t j = (uint32_t)(wid * 64 * E + e * 64 + lane);
        if (j > 0 && j < m && ((xk[j - 1] ^ k[e]) >> IDXB) == 0) tie_here = true;
    }
    bool ties = __ballot(tie_here) != 0;
    if constexpr (NW > 1) {
        if (lane == 0) flag_all[wave] = ties ? 1u : 0u;
        __syncthreads();
        ties = false;
        for (int w = 0; w < NW; ++w) ties |= flag_all[w0 + w] != 0;
    }
    uint32_t hp[E];
    if (!ties) {
#pragma unroll
        for (int e = 0; e < E; ++e) hp[e] = (uint32_t)(wid * 64 * E + e * 64 + lane);
    } else {
        uint32_t carry = 0;
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const uint32_t j = (uint32_t)(wid * 64 * E + e * 64 + lane);
            const bool head = j < m && (j == 0 || ((xk[j - 1] ^ k[e]) >> IDXB) != 0);
            uint32_t xx = wave_incl_scan_max<uint32_t>(head ? j : 0u);
            xx = xx > carry ? xx : carry;
            hp[e] = xx;
            carry = (uint32_t)__builtin_amdgcn_readlane((int)xx, 63);
        }
        if constexpr (NW > 1) {
            if (lane == 0) wmax_all[wave] = carry;
            __syncthreads();
            uint32_t pre = 0;
            for (int w = 0; w < wid; ++w) pre = wmax_all[w0 + w] > pre ? wmax_all[w0 + w] : pre;
#pragma unroll
            for (int e = 0; e < E; ++e) hp[e] = hp[e] > pre ? hp[e] : pre;
        }
    }
    SPROF(t4);
    SPACC(3, t3, t4);
    // the group's rotations and keys were consumed into registers/LDS (their
    // loads complete) before any write of its SA range; the loads in flight
    // now belong to other groups' disjoint ranges
    uint32_t runs = 0, tcnt = 0;
    uint64_t tm[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const uint32_t j = (uint32_t)(wid * 64 * E + e * 64 + lane);
        const bool valid = j < m;
        const uint32_t vb = valid ? vb_all[g][(uint32_t)(k[e] & ((1u << IDXB) - 1u))] : 0u;
        const bool end = valid && (!ties || j + 1 == m || ((xk[j + 1] ^ k[e]) >> IDXB) != 0);
        emit_vals(c, slot, s, j, vb & 0xFFFFFFu, valid, hp[e], vb >> 24);
        const bool tie = end && j > hp[e];
        tm[e] = __ballot(tie);
        tcnt += (uint32_t)__popcll(tm[e]);
        tacc += tie ? j - hp[e] + 1u : 0u;
        runs += (uint32_t)__popcll(__ballot(end));
    }
    if (c.mode && lane == 0 && runs) atomicAdd(&c.L.runs[slot], runs);
    if (ties) {                                    // uniform per group
        uint32_t tb = tie_reserve<NW>(c, tcnt, tc_all, wid, lane);
        uint64_t* tl = c.L.t[c.tsel];
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const uint32_t j = (uint32_t)(wid * 64 * E + e * 64 + lane);
            if ((tm[e] >> lane) & 1ull) tl[tb + (uint32_t)__popcll(tm[e] & lt)] = mk_item(slot, s + hp[e], j - hp[e] + 1u, 0, 0);
            tb += (uint32_t)__popcll(tm[e]);
        }
    }
    SPROF(t5);
    SPACC(4, t4, t5);
    // rotate the pipeline
    const uint32_t it2 = it1 != NONE ? next_item() : NONE;
    cur = nxt;
    nxt.item = it2 != NONE ? items[it2] : 0ull;
    grp_load_vals<NW, E>(c, nxt, it2 != NONE, wid, lane);
    it = it1;
    it1 = it2;
    SPROF(t6);
    SPACC(5, t5, t6);
    SPACC(7, t0, t6);
    }
#ifdef STARCH_SORT_PROF
    if (lane == 0 && E == 4 && NW >= 4 && !DBL)
        for (int q = 0; q < 8; ++q) atomicAdd(&g_sprof2[q + (NW == 4 ? 8 : 0)], (unsigned long long)pacc[q]);
#endif
    tacc = wave_reduce_add<uint32_t>(tacc);
    if (lane == 0 && tacc) atomicAdd(c.L.ctr + C_TS0 + c.tsel, tacc);
}

// ---------------------------------------------------------------------------
// k3_sort_grp<NW, E>: the common case of k3_sort_lds without its LSD path.
// One MSD digit (the DB bits below the highest varying key bit) scatters the
// group in LDS; then every element ranks itself inside its sub-bucket by
// comparison, working in digit order so the lanes of a wave mostly share a
// sub-bucket.  Ranking costs about sum(z^2) comparisons over the sub-bucket
// sizes z: a group whose digit spreads it badly (sum z^2 > HARD_Q * m) is
// left untouched and listed for k3_sort_lds.  While a group is sorted, the
// next group's rotations and keys are already being loaded (software
// pipeline: item two ahead, rotations and keys one ahead).
// ---------------------------------------------------------------------------
#ifndef STARCH_HARD_Q
#define STARCH_HARD_Q 32
#endif
#ifndef STARCH_GRP_EARLY
#define STARCH_GRP_EARLY 1   // the next group's key gathers issued before this group's sort
#endif
constexpr uint32_t HARD_Q = STARCH_HARD_Q;


template <int NW, int E, bool DBL>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(sort_wpe(NW, E))))
k3_sort_grp(Ctx c, const uint64_t* __restrict__ items,
                                                    uint64_t* __restrict__ hard)
{
    constexpr int IPW = 4 / NW;                    // groups per workgroup
    constexpr int CAP = NW * 64 * E;
    constexpr int IDXB = CAP <= 256 ? 8 : 12;      // packed local index bits
    constexpr int KEYB = 64 - IDXB;
    constexpr uint64_t KMASK = (1ull << KEYB) - 1ull;
    static_assert(CAP <= (1 << IDXB), "index does not fit");
    constexpr int DB = CAP <= 128 ? 7 : (CAP <= 256 ? 8 : (CAP <= 1024 ? 10 : 11));   // MSD digit bits
    constexpr int NBIN = 1 << DB;
    constexpr int T = NW * 64;
    constexpr int BPT = NBIN / T;                  // bins per thread
    __shared__ uint64_t xk_all[IPW][CAP];
    __shared__ uint32_t vb_all[IPW][CAP];          // rotations by group index
    __shared__ uint32_t bst_all[IPW][NBIN + 1];    // sub-bucket starts
    __shared__ uint32_t bcur_all[IPW][NBIN];       // scatter cursors
    __shared__ uint32_t sc_all[IPW][NW + 1];
    __shared__ uint64_t red_all[4];
    __shared__ uint32_t wsq_all[4];
    __shared__ uint32_t wmax_all[4];
    __shared__ uint32_t flag_all[4];
    __shared__ uint32_t tc_all[5];
    uint32_t tacc = 0;                             // tied elements pushed (flushed at exit)
    const uint64_t lt = lanemask_lt();
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int g = wave / NW, wid = wave % NW, w0 = g * NW;
    uint64_t* xk = xk_all[g];
    uint32_t* sc = sc_all[g];
    uint32_t* bst = bst_all[g];
    uint32_t* bcur = bcur_all[g];
    const int tg = wid * 64 + lane;
#ifndef STARCH_GRP_CHUNK
#define STARCH_GRP_CHUNK 32   // groups per queue pop (cfg2 block sort: 8 / 16 / 32 / 64 / 128: 25.0, 20.5, 19.7, 20.0, 21.8 ms)
#endif
    // dynamic assignment (NW == 1): each wave pops groups, STARCH_GRP_CHUNK at a time,
    // from its XCD's queue, so the XCD's waves stay on neighbouring groups (one block's
    // PSS in its L2) however uneven the groups' costs; static striding drifted
    // apart by many blocks over a launch (a third of the key loads missed L2)
    static_assert(NW == 1, "k3_sort_grp: one wave per group");
    __shared__ uint32_t qs[8];
    const uint32_t xs = xcc_id();
    load_qsizes_binned(c, qs);
#ifndef STARCH_GRP_CHUNK_S2
#define STARCH_GRP_CHUNK_S2 16   // S2 (E = 4): 8 / 16 / 32 -> ms_bwt 19.17 / 18.91 / 18.97; at 32 the groups in flight
#endif                           // span more blocks per XCD (S2 fetch 6.5 -> 14.5 GB per cfg2 step)
    WaveQueue<E == 4 ? STARCH_GRP_CHUNK_S2 : STARCH_GRP_CHUNK> wq;
    constexpr uint32_t NONE = 0xFFFFFFFFu;
    // software pipeline, three groups deep: while group n sorts, the keys of
    // n + 1 are issued (its rotations arrived an iteration ago) and the
    // rotations of n + 2 are in flight (STARCH_GRP_DEEP=0: two deep, the
    // rotations of n + 1 issued only one iteration before its keys)
#ifndef STARCH_GRP_DEEP
#define STARCH_GRP_DEEP 0   // measured no faster (cfg2 sort 23.2 vs 23.3 ms, profiles/r03_v3/sweep_deep*.json)
#endif
    uint32_t it = wq.next(c.qhead, qs, c.qseg, xs);
    uint32_t it1 = it != NONE ? wq.next(c.qhead, qs, c.qseg, xs) : NONE;
    uint32_t it2 = it1 != NONE ? wq.next(c.qhead, qs, c.qseg, xs) : NONE;
    GrpIn<E> cur, nxt;
    cur.item = it != NONE ? items[it] : 0ull;
    nxt.item = it1 != NONE ? items[it1] : 0ull;
    grp_load_vals<NW, E>(c, cur, it != NONE, wid, lane);
    grp_load_keys<NW, E, DBL>(c, cur, wid, lane);
    grp_load_vals<NW, E>(c, nxt, it1 != NONE, wid, lane);
#if STARCH_GRP_DEEP
    GrpIn<E> vst;                                  // group n + 2: rotations only
    vst.item = it2 != NONE ? items[it2] : 0ull;
    grp_load_vals<NW, E>(c, vst, it2 != NONE, wid, lane);
    uint32_t it3 = it2 != NONE ? wq.next(c.qhead, qs, c.qseg, xs) : NONE;
    uint64_t nitem3 = it3 != NONE ? items[it3] : 0ull;
#else
    uint64_t nitem2 = it2 != NONE ? items[it2] : 0ull;
#endif
#ifdef STARCH_SORT_PROF
    uint64_t pacc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif
    while (it != NONE) {
    SPROF(t0);
    const uint64_t item = cur.item;
    const uint32_t slot = it_slot(item), s = it_start(item), m = it_size(item);
    grp_finish_keys<NW, E, DBL>(cur);
    gsync<NW>();                                   // the previous group's LDS reads are done

    uint64_t k[E];
    uint64_t diff = 0;
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const uint32_t i = (uint32_t)(wid * 64 * E + e * 64 + lane);
        if (i < m) {
            diff |= cur.kx[e] ^ cur.k0;
            k[e] = ((cur.kx[e] & KMASK) << IDXB) | i;
            vb_all[g][i] = cur.v[e] | (cur.ls[e] << 24);
        } else {
            k[e] = ~0ull;                              // pads: max key, last in order
        }
    }
#if STARCH_GRP_EARLY
    // the next group's key gathers go out now, so they are in flight during
    // this group's LDS-only sort phases (issued after the sort, the emit's
    // returning atomics and the queue pops waited for them at once: every
    // vmcnt wait is in issue order)
    grp_load_keys<NW, E, DBL>(c, nxt, wid, lane);
#endif
    diff = wave_reduce_or64(diff);
    if constexpr (NW > 1) {
        if (lane == 0) red_all[wave] = diff;
        __syncthreads();
        diff = 0;
#pragma unroll
        for (int w = 0; w < NW; ++w) diff |= red_all[w0 + w];
    }
    if ((diff >> KEYB) && tg == 0) atomicOr(&c.L.ctr[C_ERR], 1u);   // top bits not shared
    SPROF(t1);
    SPACC(0, t0, t1);

    bool is_hard = false;
    const uint64_t kdiff = diff & KMASK;
    if (kdiff) {
        const int hb = 63 - __clzll((long long)kdiff);
        const int lo = hb + 1 - DB > 0 ? hb + 1 - DB : 0;
        for (int q = tg; q < NBIN; q += T) bcur[q] = 0;
        gsync<NW>();
        uint32_t dg[E];
#pragma unroll
        for (int e = 0; e < E; ++e) {
            dg[e] = (uint32_t)((k[e] >> (lo + IDXB)) & (uint64_t)(NBIN - 1));
            if ((uint32_t)(wid * 64 * E + e * 64 + lane) < m) atomicAdd(&bcur[dg[e]], 1u);
        }
        gsync<NW>();
        uint32_t loc[BPT], sum = 0, sq = 0;
#pragma unroll
        for (int q = 0; q < BPT; ++q) {
            loc[q] = bcur[tg * BPT + q];
            sum += loc[q];
            sq += loc[q] * loc[q];
        }
        const uint32_t incl = wave_incl_scan_add(sum);
        uint32_t run = incl - sum;
        sq = wave_reduce_add(sq);
        if constexpr (NW > 1) {
            if (lane == 63) sc[wid] = incl;
            if (lane == 0) wsq_all[wave] = sq;
            __syncthreads();
            for (int w = 0; w < wid; ++w) run += sc[w];
            sq = 0;
            for (int w = 0; w < NW; ++w) sq += wsq_all[w0 + w];
        }
        is_hard = sq > HARD_Q * m;                 // uniform per group
        SPROF(t2);
        SPACC(1, t1, t2);
#ifdef STARCH_SORT_STATS
        if (tg == 0) { atomicAdd(&c.L.ctr[C_STG], 1u); atomicAdd(&c.L.ctr[C_STE], m); if (is_hard) atomicAdd(&c.L.ctr[C_STH], 1u); }
#endif
        if (!is_hard) {
#pragma unroll
            for (int q = 0; q < BPT; ++q) { bst[tg * BPT + q] = run; bcur[tg * BPT + q] = run; run += loc[q]; }
            if (tg == T - 1) bst[NBIN] = run;
            gsync<NW>();
#pragma unroll
            for (int e = 0; e < E; ++e)
                if ((uint32_t)(wid * 64 * E + e * 64 + lane) < m) xk[atomicAdd(&bcur[dg[e]], 1u)] = k[e];
            gsync<NW>();
            // rank in digit order: position j holds kj; its final place is
            // bs + #{q in its sub-bucket: kq < kj, or kq == kj and q < j}
            uint32_t pos[E];
#pragma unroll
            for (int e = 0; e < E; ++e) {
                const uint32_t j = (uint32_t)(wid * 64 * E + e * 64 + lane);
                pos[e] = j;
                if (j < m) {
                    const uint64_t kj = xk[j];
                    const uint32_t d = (uint32_t)((kj >> (lo + IDXB)) & (uint64_t)(NBIN - 1));
                    const uint32_t bs = bst[d], be = bst[d + 1];
                    pos[e] = bs + rank_in(xk, bs, be, kj);
#ifdef STARCH_SORT_STATS
                    atomicAdd(&c.L.ctr[C_STW], be - bs);
#endif
                    k[e] = kj;
                }
            }
            gsync<NW>();
#pragma unroll
            for (int e = 0; e < E; ++e) xk[pos[e]] = k[e];
        } else {
            gsync<NW>();                           // bcur/sc reads done
            if (tg == 0) hard[atomicAdd(&c.L.ctr[C_H], 1u)] = item;
        }
    } else {
#pragma unroll
        for (int e = 0; e < E; ++e) xk[wid * 64 * E + e * 64 + lane] = k[e];
    }
    SPROF(t3);
    SPACC(2, t1, t3);
#if !STARCH_GRP_EARLY
    // next group's keys (its rotations were loaded one or two groups ago), a new item
    grp_load_keys<NW, E, DBL>(c, nxt, wid, lane);
#endif
    SPROF(t4);
    SPACC(3, t3, t4);
#if STARCH_GRP_DEEP
    const uint32_t it4 = it3 != NONE ? wq.next(c.qhead, qs, c.qseg, xs) : NONE;
    const uint64_t nitem4 = it4 != NONE ? items[it4] : 0ull;
#else
    const uint32_t it3 = it2 != NONE ? wq.next(c.qhead, qs, c.qseg, xs) : NONE;
    const uint64_t nitem3 = it3 != NONE ? items[it3] : 0ull;
#endif
    if (!is_hard) {
    gsync<NW>();
#pragma unroll
    for (int e = 0; e < E; ++e) k[e] = xk[wid * 64 * E + e * 64 + lane];
    // runs of equal keys in sorted order j = wid*64*E + e*64 + lane
    bool tie_here = false;
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const uint32_t j = (uint32_t)(wid * 64 * E + e * 64 + lane);
        if (j > 0 && j < m && ((xk[j - 1] ^ k[e]) >> IDXB) == 0) tie_here = true;
    }
    bool ties = __ballot(tie_here) != 0;
    if constexpr (NW > 1) {
        if (lane == 0) flag_all[wave] = ties ? 1u : 0u;
        __syncthreads();
        ties = false;
        for (int w = 0; w < NW; ++w) ties |= flag_all[w0 + w] != 0;
    }
    uint32_t hp[E];
    if (!ties) {
#pragma unroll
        for (int e = 0; e < E; ++e) hp[e] = (uint32_t)(wid * 64 * E + e * 64 + lane);
    } else {
        uint32_t carry = 0;
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const uint32_t j = (uint32_t)(wid * 64 * E + e * 64 + lane);
            const bool head = j < m && (j == 0 || ((xk[j - 1] ^ k[e]) >> IDXB) != 0);
            uint32_t xx = wave_incl_scan_max<uint32_t>(head ? j : 0u);
            xx = xx > carry ? xx : carry;
            hp[e] = xx;
            carry = (uint32_t)__builtin_amdgcn_readlane((int)xx, 63);
        }
        if constexpr (NW > 1) {
            if (lane == 0) wmax_all[wave] = carry;
            __syncthreads();
            uint32_t pre = 0;
            for (int w = 0; w < wid; ++w) pre = wmax_all[w0 + w] > pre ? wmax_all[w0 + w] : pre;
#pragma unroll
            for (int e = 0; e < E; ++e) hp[e] = hp[e] > pre ? hp[e] : pre;
        }
    }
    SPROF(t5);
    SPACC(4, t4, t5);
    // the group's SA range was read (values consumed above) before any write
    uint32_t runs = 0, tcnt = 0;
    uint64_t tm[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const uint32_t j = (uint32_t)(wid * 64 * E + e * 64 + lane);
        const bool valid = j < m;
        const uint32_t vb = valid ? vb_all[g][(uint32_t)(k[e] & ((1u << IDXB) - 1u))] : 0u;
        const bool end = valid && (!ties || j + 1 == m || ((xk[j + 1] ^ k[e]) >> IDXB) != 0);
        emit_vals(c, slot, s, j, vb & 0xFFFFFFu, valid, hp[e], vb >> 24);
        const bool tie = end && j > hp[e];
        tm[e] = __ballot(tie);
        tcnt += (uint32_t)__popcll(tm[e]);
        tacc += tie ? j - hp[e] + 1u : 0u;
        runs += (uint32_t)__popcll(__ballot(end));
    }
    if (c.mode && lane == 0 && runs) atomicAdd(&c.L.runs[slot], runs);
    if (ties) {                                    // uniform per group
        uint32_t tb = tie_reserve<NW>(c, tcnt, tc_all, wid, lane);
        uint64_t* tl = c.L.t[c.tsel];
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const uint32_t j = (uint32_t)(wid * 64 * E + e * 64 + lane);
            if ((tm[e] >> lane) & 1ull) tl[tb + (uint32_t)__popcll(tm[e] & lt)] = mk_item(slot, s + hp[e], j - hp[e] + 1u, 0, 0);
            tb += (uint32_t)__popcll(tm[e]);
        }
    }
    }
    SPROF(t6);
    SPACC(5, t4, t6);
    // rotate the pipeline
#if STARCH_GRP_DEEP
    cur = nxt;
    nxt.item = vst.item;
    nxt.ks = vst.ks;
#pragma unroll
    for (int e = 0; e < E; ++e) nxt.v[e] = vst.v[e];
    nxt.v0 = vst.v0;
    vst.item = nitem3;
    nitem3 = nitem4;
    grp_load_vals<NW, E>(c, vst, it3 != NONE, wid, lane);
    it = it1;
    it1 = it2;
    it2 = it3;
    it3 = it4;
#else
    cur = nxt;
    nxt.item = nitem2;
    nitem2 = nitem3;
    grp_load_vals<NW, E>(c, nxt, it2 != NONE, wid, lane);
    it = it1;
    it1 = it2;
    it2 = it3;
#endif
    SPROF(t7);
    SPACC(6, t6, t7);
    SPACC(7, t0, t7);
    }
#ifdef STARCH_SORT_PROF
    if (lane == 0)
        for (int q = 0; q < 8; ++q) atomicAdd(&g_sprof[q + (E == 2 ? 0 : 8)], (unsigned long long)pacc[q]);
#endif
    tacc = wave_reduce_add<uint32_t>(tacc);
    if (lane == 0 && tacc) atomicAdd(c.L.ctr + C_TS0 + c.tsel, tacc);
}

// ---------------------------------------------------------------------------
// text rounds: classify the tie groups (keys come from the PSS at an offset)
// ---------------------------------------------------------------------------
constexpr uint32_t CT_IPT = 16;        // tie groups per thread in k3_classify_text

// tie groups -> size-class lists for the next text round (as wg_classify, CT_IPT
// groups per thread: one LDS atomic per thread and class, one global atomic
// per workgroup and class, the groups held in registers between the passes)
__global__ void __launch_bounds__(256) k3_classify_text(Ctx c, const uint64_t* __restrict__ items, uint32_t nitems)
{
    __shared__ uint32_t cls_cnt[8], cls_base[8];
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    if (tid < 8) cls_cnt[tid] = 0;
    __syncthreads();
    const uint64_t i0 = (uint64_t)blockIdx.x * 256u * CT_IPT + tid;
    uint64_t it[CT_IPT];
    uint32_t cnt[8] = {0, 0, 0, 0, 0, 0, 0, 0}, tied = 0;
#pragma unroll
    for (uint32_t k = 0; k < CT_IPT; ++k) {
        const uint64_t i = i0 + (uint64_t)k * 256u;
        it[k] = i < nitems ? items[i] : 0ull;
        if (i < nitems) {
            const uint32_t m = it_size(it[k]);
            ++cnt[size_class(m)];
            tied += m;
        }
    }
    uint32_t off[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) off[q] = cnt[q] ? atomicAdd(&cls_cnt[q], cnt[q]) : 0u;
    __syncthreads();
    if (tid < 8 && cls_cnt[tid]) cls_base[tid] = atomicAdd(class_ctr(c, (int)tid), cls_cnt[tid]);
    __syncthreads();
#pragma unroll
    for (uint32_t k = 0; k < CT_IPT; ++k) {
        const uint64_t i = i0 + (uint64_t)k * 256u;
        if (i < nitems) {
            const uint32_t slot = it_slot(it[k]), m = it_size(it[k]);
            const int cls = size_class(m);
            uint32_t o = 0;
#pragma unroll
            for (int q = 0; q < 8; ++q) if (q == cls) o = off[q]++;
            const Geo g = c.L.geo[slot];
            class_list(c, cls)[cls_base[cls] + o] = mk_item(slot, it_start(it[k]), m, g.Dp * g.B, 0);
            if (cls == 6 && m > HG_MIN_PUSH) atomicMax(&c.L.ctr[C_LM0 + c.lsel], m);
        }
    }
    tied = wave_reduce_add<uint32_t>(tied);
    if (lane == 0 && tied) atomicAdd(&c.L.ctr[C_TIE_ELEMS], tied);
}

// ---------------------------------------------------------------------------
// doubling round: gather keys of tied rotations, classify their groups
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k3_gather(Ctx c, const uint64_t* __restrict__ items, uint32_t nitems,
                                                  uint32_t round, uint32_t rtext)
{
    const int lane = threadIdx.x & 63;
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    bool active = i < nitems;
    uint64_t item = active ? items[i] : 0;
    uint32_t slot = it_slot(item), s = it_start(item), m = it_size(item);
    uint32_t n = 1;
    uint32_t hm = 0;
    if (active) {
        active = c.L.periodic[slot] == 0;
        n = c.blocks[c.b0 + slot].n;
        const Geo g = c.L.geo[slot];
        const uint64_t h = ((uint64_t)g.D + (uint64_t)rtext * g.Dp) << (round - 1);
        if (active && h >= n) {   // sorted on >= n symbols: remaining ties are equal rotations
            c.L.periodic[slot] = 1;
            active = false;
        }
        hm = (uint32_t)(h % n);
    }
    const uint64_t so = (uint64_t)slot * c.scr.stride;
    if (active && m <= 64) {
        for (uint32_t q = s; q < s + m; ++q) {
            uint32_t t = c.scr.SA[so + q] + hm;
            if (t >= n) t -= n;
            c.scr.K2[so + q] = c.scr.RK[so + t];
        }
    }
    // groups above GB_MIN: gathered by the whole grid (k3_gather_big) -- one
    // wave walking a group of 450k tied rotations took most of a round
    bool taken = false;
    {
        const bool huge = active && m > GB_MIN;
        const uint64_t hb = __ballot(huge);
        if (hb) {
            const int lead = __ffsll((unsigned long long)hb) - 1;
            uint32_t b0 = 0;
            if (lane == lead) b0 = atomicAdd(&c.L.ctr[C_GB], (uint32_t)__popcll(hb));
            b0 = (uint32_t)__shfl((int)b0, lead, 64);
            const uint32_t o = b0 + (uint32_t)__popcll(hb & lanemask_lt());
            taken = huge && o < GB_MAXN;
            if (taken) {
                c.L.gb[o] = mk_item(slot, s, m, 0, 0);
                c.L.gb_h[o] = hm;
            }
        }
    }
    uint64_t bigm = __ballot(active && m > 64 && !taken);
    while (bigm) {
        const int l = __ffsll((unsigned long long)bigm) - 1;
        bigm &= bigm - 1;
        const uint32_t ls = __shfl(s, l, 64), lm = __shfl(m, l, 64), lslot = __shfl(slot, l, 64);
        const uint32_t ln = __shfl(n, l, 64), lh = __shfl(hm, l, 64);
        const uint64_t lso = (uint64_t)lslot * c.scr.stride;
        for (uint32_t q = ls + lane; q < ls + lm; q += 64) {
            uint32_t t = c.scr.SA[lso + q] + lh;
            if (t >= ln) t -= ln;
            c.scr.K2[lso + q] = c.scr.RK[lso + t];
        }
    }
    __shared__ uint32_t cls_sh[16];
    wg_classify(c, cls_sh, active, slot, s, m, RBITS, 0);
    wave_add_slot(c.L.gin, active, slot, 1u);
    const uint32_t tied = wave_reduce_add<uint32_t>(active ? m : 0u);
    if (lane == 0 && tied) atomicAdd(&c.L.ctr[C_TIE_ELEMS], tied);
}

__global__ void __launch_bounds__(256) k3_gather_big(Ctx c)
{
    const uint32_t ng = min(c.L.ctr[C_GB], GB_MAXN);
    const GridSplit gs = grid_split(ng);
    if (gs.idle) return;
    const uint32_t step = gs.per * 256u;
    for (uint32_t q = gs.q0; q < ng; q += gs.gstride) {
        const uint64_t item = c.L.gb[q];
        const uint32_t slot = it_slot(item), s = it_start(item), m = it_size(item), hm = c.L.gb_h[q];
        const uint32_t n = c.blocks[c.b0 + slot].n;
        const uint64_t so = (uint64_t)slot * c.scr.stride;
        for (uint32_t i = gs.slice * 256u + threadIdx.x; i < m; i += step) {
            uint32_t t = c.scr.SA[so + s + i] + hm;
            if (t >= n) t -= n;
            c.scr.K2[so + s + i] = c.scr.RK[so + t];
        }
    }
}

// ---- switch to doubling: dense ranks for the blocks that are still tied ----
__global__ void k3_mark_tied(Ctx c, const uint64_t* __restrict__ items, uint32_t nitems)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nitems) c.L.tied[it_slot(items[i])] = 1;
}

__global__ void __launch_bounds__(256) k3_rk_dense(Ctx c)
{
    const uint32_t slot = blockIdx.y;
    if (!c.L.tied[slot]) return;
    const uint32_t n = c.blocks[c.b0 + slot].n;
    const uint64_t so = (uint64_t)slot * c.scr.stride;
    for (uint32_t j = blockIdx.x * 256 + threadIdx.x; j < n; j += gridDim.x * 256) c.scr.RK[so + c.scr.SA[so + j]] = j;
}

__global__ void __launch_bounds__(256) k3_rk_groups(Ctx c, const uint64_t* __restrict__ items, uint32_t nitems)
{
    // one wave per group
    const int lane = threadIdx.x & 63;
    const uint32_t gi = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (gi >= nitems) return;
    const uint64_t item = items[gi];
    const uint32_t slot = it_slot(item), s = it_start(item), m = it_size(item);
    const uint64_t so = (uint64_t)slot * c.scr.stride;
    if (m > GB_MIN) {                     // the whole grid takes it (k3_rk_big) unless the list is full
        uint32_t o = 0;
        if (lane == 0) o = atomicAdd(&c.L.ctr[C_GB], 1u);
        o = (uint32_t)__shfl((int)o, 0, 64);
        if (o < GB_MAXN) {
            if (lane == 0) c.L.gb[o] = item;
            return;
        }
    }
    for (uint32_t q = s + lane; q < s + m; q += 64) c.scr.RK[so + c.scr.SA[so + q]] = s;
}

__global__ void __launch_bounds__(256) k3_rk_big(Ctx c)
{
    const uint32_t ng = min(c.L.ctr[C_GB], GB_MAXN);
    const GridSplit gs = grid_split(ng);
    if (gs.idle) return;
    const uint32_t step = gs.per * 256u;
    for (uint32_t q = gs.q0; q < ng; q += gs.gstride) {
        const uint64_t item = c.L.gb[q];
        const uint32_t slot = it_slot(item), s = it_start(item), m = it_size(item);
        const uint64_t so = (uint64_t)slot * c.scr.stride;
        for (uint32_t i = gs.slice * 256u + threadIdx.x; i < m; i += step) c.scr.RK[so + c.scr.SA[so + s + i]] = s;
    }
}

__global__ void k3_round_end(Ctx c, uint32_t nb)
{
    const uint32_t slot = blockIdx.x * blockDim.x + threadIdx.x;
    if (slot >= nb) return;
    const uint32_t g = c.L.gin[slot];
    if (g) {
        c.L.rounds[slot] += 1;
        if (c.L.runs[slot] == g) c.L.periodic[slot] = 1;   // no group split: equal rotations
    }
    c.L.gin[slot] = 0;
    c.L.runs[slot] = 0;
}

__global__ void k3_finish(Ctx c, uint32_t nb, unsigned long long* stats)
{
    const uint32_t slot = blockIdx.x * blockDim.x + threadIdx.x;
    if (slot >= nb) return;
    const uint32_t p = c.L.periodic[slot];
    c.blocks[c.b0 + slot].flags = p ? 1u : 0u;
    atomicAdd(stats, (unsigned long long)c.L.rounds[slot]);
    if (p) atomicAdd(stats + 1, 1ull);
    if (slot == 0) atomicAdd(stats + 2, (unsigned long long)c.L.ctr[C_TIE_ELEMS]);
}

// Periodic blocks up front: a cyclic block has equal rotations iff its minimal
// period divides n and is < n, iff block[i] == block[i + n/q] (i < n - n/q)
// for a prime q of n.  Flagged blocks take no doubling round (k3_gather drops
// their groups); the flag is the one the rounds would reach.  One workgroup per
// block, 4 KiB steps, so a non-periodic block stops after its first step.
__global__ void __launch_bounds__(256) k3_period(Ctx c)
{
    __shared__ uint32_t q_sh[16];
    __shared__ uint32_t nq_sh;
    __shared__ uint32_t dv[32];                    // divisors d <= sqrt(n) < 1024, as bits
    const uint32_t slot = blockIdx.x, b = c.b0 + slot;
    const uint32_t n = c.blocks[b].n;
    if (n < 2) return;
    // prime factors of n: the workgroup marks every divisor <= sqrt(n) (a few
    // trial divisions per thread: there is no integer divide, and one thread
    // walking all ~950 candidates took ~70 us), then one thread divides out the
    // marked ones in increasing order (composites no longer divide by then)
    if (threadIdx.x < 32) dv[threadIdx.x] = 0;
    __syncthreads();
    for (uint32_t d = 2 + threadIdx.x; d * d <= n; d += 256)
        if (n % d == 0) atomicOr(&dv[d >> 5], 1u << (d & 31));
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t m = n, k = 0;
        for (uint32_t w = 0; w < 32; ++w)
            for (uint32_t bits = dv[w]; bits; bits &= bits - 1) {
                const uint32_t d = 32 * w + (uint32_t)__builtin_ctz(bits);
                if (m % d == 0) {
                    q_sh[k++] = d;
                    while (m % d == 0) m /= d;
                }
            }
        if (m > 1) q_sh[k++] = m;
        nq_sh = k;
    }
    __syncthreads();
    const uint8_t* blk = c.blkbytes + (uint64_t)b * c.stride;
    const uint32_t nq = nq_sh;
    for (uint32_t j = 0; j < nq; ++j) {
        const uint32_t p = n / q_sh[j], e = n - p;
        int bad = 0;
        for (uint32_t a = 0; a < e && !bad; a += 4096) {
            const uint32_t z = a + 4096 < e ? a + 4096 : e;
            int mis = 0;
            for (uint32_t i = a + threadIdx.x; i < z; i += 256) mis |= blk[i] != blk[i + p];
            bad = __syncthreads_or(mis);
        }
        if (!bad) {
            if (threadIdx.x == 0) c.L.periodic[slot] = 1;
            return;
        }
    }
}

// round 0 (STARCH_KGATHER): every rotation's key window and last-column
// symbol next to its SA entry, in SA order (KM0 / LS0), 4 per thread with
// every gather issued before any is used
__global__ void __launch_bounds__(256) k3_keys(Ctx c)
{
    const uint32_t slot = blockIdx.y;
    const uint32_t n = c.blocks[c.b0 + slot].n;
    const uint64_t so = (uint64_t)slot * c.scr.stride;
    const KeySrc ks = key_src(c, slot, 0);
    const uint32_t* SA = c.scr.SA + so;
    uint64_t* KM = c.kA + so;
    uint8_t* LS = c.lA + so;
    constexpr uint32_t U = 4;
    for (uint32_t i0 = blockIdx.x * 256u * U; i0 < n; i0 += gridDim.x * 256u * U) {
        uint32_t v[U], ls[U];
        uint64_t k[U];
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) {
            const uint32_t i = i0 + u * 256u + threadIdx.x;
            v[u] = SA[i < n ? i : 0u];
        }
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) k[u] = ks.key_pss(v[u], ls[u]);
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) {
            const uint32_t i = i0 + u * 256u + threadIdx.x;
            if (i < n) {
                KM[i] = k[u];
                LS[i] = (uint8_t)ls[u];
            }
        }
    }
}

}  // namespace

// zero the counters whose bits are set (one launch instead of a memset each)
__global__ void k3_zero(uint32_t* __restrict__ ctr, uint64_t mask)
{
    const uint32_t i = threadIdx.x;
    if (i < 64 && ((mask >> i) & 1ull)) ctr[i] = 0;
}

// Host orchestration.  A handful of host round trips per batch (list sizes).
// STARCH_KGATHER=1: round-0 keys gathered into a position-ordered array by
// their own pass after the top-level scatter (k3_keys: SA read and key
// writes coalesced, the PSS gathers at the L2's random-read rate), so the
// sorts read keys by position; STARCH_KMAT=1: the scatter writes them
bool bwt_kgather()
{
    static const bool on = [] { const char* e = getenv("STARCH_KGATHER"); return e && !strcmp(e, "1"); }();
    return on;
}

bool bwt_kmat()
{
    static const bool on = [] { const char* e = getenv("STARCH_KMAT"); return e && !strcmp(e, "1"); }();
    return on || bwt_kgather();
}

bool launch_bwt3(BlockDesc* blocks, uint32_t b0, uint32_t nb, const uint8_t* blkbytes, uint64_t stride,
                 const BwtScratch& scr, DevBuf& meta, uint32_t* hctr, unsigned long long* stats, hipStream_t st,
                 bool wide)
{
    if (nb == 0) return false;
    if (nb > 4095) throw StarchError(-2, "bwt3: batch too large");
    // the tile histograms live in K after the PSS: [MAXT + 1][bins] words (small
    // blocks, -1 .. -2, have room for the 4096-bin binary digit only)
    if (wide && pss_words(scr.stride) * 2 + (uint64_t)(MAXT + 1) * PNB_WIDE > 2 * scr.stride) wide = false;
    if (pss_words(scr.stride) * 2 + (uint64_t)(MAXT + 1) * PNB > 2 * scr.stride)
        throw StarchError(-2, "bwt3: block stride too small");
    const uint64_t N = (uint64_t)nb * scr.stride;
    const uint64_t cap_s = N / (W_MAX + 1) + 64, cap_s2 = N / (S1_MAX + 1) + 64, cap_m0 = N / (S_MAX + 1) + 64,
                   cap_m1 = N / (M0_MAX + 1) + 64,
                   cap_m2 = N / (M1_MAX + 1) + 64,
                   cap_m3 = N / (M2_MAX + 1) + 64, cap_l = N / ((L_MIN < M3_MAX ? L_MIN : M3_MAX) + 1) + 64;
    const uint64_t nwg_bin = BIN_MAXWG;
    const uint64_t nb_bins = nb < 64 ? 8ull * nb : nb;     // bins of k3_bin_* (see bin_of)
    constexpr uint32_t QSETS = 64, QSET = 8 * XQ_STRIDE + 32;   // queue heads (a line each) + segments per launch
    const uint64_t hg_words = 2ull * HG_MAXN + (uint64_t)HG_MAXN * 512 + 3ull * GB_MAXN + 64 + (HG_MAXN + 1) +
                              2ull * HG_MAXN + HG_MAXN + 2ull * HG_MAXN + 6ull * HG_MAXN + HG_MAXN + 8;
    const uint64_t words = 2 * C_N + 14ull * nb + QSETS * QSET + (nwg_bin + 2) * nb_bins +
                           2 * (cap_s + cap_s2 + cap_m0 + cap_m1 + cap_m2 + cap_m3 + 2 * cap_l) + 64 + hg_words;
    uint32_t* mw = meta.as<uint32_t>(words);
    Ctx c;
    c.blocks = blocks;
    c.b0 = b0;
    c.blkbytes = blkbytes;
    c.stride = stride;
    c.scr = scr;
    c.nb = nb;
    c.L.ctr = mw;
    c.L.gin = mw + 2 * C_N;
    c.L.runs = c.L.gin + nb;
    c.L.periodic = c.L.runs + nb;
    c.L.rounds = c.L.periodic + nb;
    c.L.tied = c.L.rounds + nb;
    c.L.geo = reinterpret_cast<Geo*>(c.L.tied + nb);            // 8 words per slot
    uint32_t* qpool = reinterpret_cast<uint32_t*>(c.L.geo + nb);
    uint32_t* bincol = qpool + QSETS * QSET;       // per-bin running totals (zeroed below, reset by k3_bin_scan)
    uint32_t* binst = bincol + nb_bins;            // per-bin starts
    uint32_t* binh = binst + nb_bins;
    uintptr_t p = reinterpret_cast<uintptr_t>(binh + nwg_bin * nb_bins);
    p = (p + 7) & ~(uintptr_t)7;
    c.L.s = reinterpret_cast<uint64_t*>(p);
    c.L.s2 = c.L.s + cap_s;
    c.L.m0 = c.L.s2 + cap_s2;
    c.L.m1 = c.L.m0 + cap_m0;
    c.L.m2 = c.L.m1 + cap_m1;
    c.L.m3 = c.L.m2 + cap_m2;
    c.L.l[0] = c.L.m3 + cap_m3;
    c.L.l[1] = c.L.l[0] + cap_l;
    {   // huge-group path (k3_hg_*, k3_gather_big): after the class lists
        uintptr_t q = reinterpret_cast<uintptr_t>(c.L.l[1] + cap_l);
        q = (q + 7) & ~(uintptr_t)7;
        c.L.hg = reinterpret_cast<uint64_t*>(q);
        c.L.gb = c.L.hg + HG_MAXN;
        c.L.gb_h = reinterpret_cast<uint32_t*>(c.L.gb + GB_MAXN);
        c.L.hg_info = c.L.gb_h + GB_MAXN;
        uintptr_t r = reinterpret_cast<uintptr_t>(c.L.hg_info + (uint64_t)HG_MAXN * 512);
        r = (r + 7) & ~(uintptr_t)7;
        c.L.hg_vary = reinterpret_cast<uint64_t*>(r);
        c.L.hg_flag = reinterpret_cast<uint32_t*>(c.L.hg_vary + HG_MAXN);
        c.L.hg_pre = c.L.hg_flag + HG_MAXN;
        c.L.hg_eqlt = c.L.hg_pre + HG_MAXN + 1;
        c.L.hg_mc = c.L.hg_eqlt + 2 * HG_MAXN;
        c.L.hg_rank = c.L.hg_mc + 6 * HG_MAXN;
        if (reinterpret_cast<uintptr_t>(c.L.hg_rank + HG_MAXN) > reinterpret_cast<uintptr_t>(mw + words))
            throw StarchError(-10, "bwt3: meta layout");
    }
    c.L.w = reinterpret_cast<uint64_t*>(scr.U);
    c.L.t[0] = reinterpret_cast<uint64_t*>(scr.U2);
    c.L.t[1] = reinterpret_cast<uint64_t*>(scr.V2);
    c.lsel = 0;
    c.tsel = 0;
    c.mode = 0;
    c.keysrc = 0;
    c.kA = scr.K2;
    c.kB = scr.K;
    c.lA = c.lB = nullptr;
    c.rtext = 0;
    c.qhead = nullptr;
    c.qseg = nullptr;
    c.nbins = wide ? PNB_WIDE : PNB;
    c.sdig = 0;
    HIP_CHECK(hipMemsetAsync(mw, 0, (2 * C_N + 14ull * nb + QSETS * QSET + nb_bins) * sizeof(uint32_t), st));
    static const bool period_off = [] { const char* e = getenv("STARCH_PERIOD_CHECK"); return e && !strcmp(e, "0"); }();
    if (!period_off) hipLaunchKernelGGL(k3_period, dim3(nb), dim3(256), 0, st, c);

    static_assert(C_N <= 64, "k3_zero masks");
    auto zero = [&](uint64_t mask) { hipLaunchKernelGGL(k3_zero, dim3(1), dim3(64), 0, st, c.L.ctr, mask); };
    auto bit = [](uint32_t i) { return 1ull << i; };
    uint32_t qnext = 0;
    auto next_q = [&](uint32_t*& head, uint32_t*& seg) {
        if (qnext == QSETS) {
            HIP_CHECK(hipMemsetAsync(qpool, 0, QSETS * QSET * sizeof(uint32_t), st));
            qnext = 0;
        }
        head = qpool + qnext * QSET;
        seg = head + 8 * XQ_STRIDE;
        ++qnext;
    };
    auto read_ctr = [&]() {
        HIP_CHECK(hipMemcpyAsync(hctr, c.L.ctr, C_N * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
        HIP_CHECK(hipStreamSynchronize(st));
#ifndef STARCH_EXP_NOGATHER
        if (hctr[C_ERR]) throw StarchError(-11, "bwt3: group keys do not share 12 top bits");
#endif
    };
    int dev = 0;
    HIP_CHECK(hipGetDevice(&dev));
    static int ncu = 0;
    if (!ncu) {
        hipDeviceProp_t prop;
        HIP_CHECK(hipGetDeviceProperties(&prop, dev));
        ncu = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
    }
    // bin a list (n items, device) into `out`; sets c.qseg/c.qhead for the next launch
    auto bin = [&](const uint64_t* list, uint32_t n, uint64_t* out) {
        uint32_t* head;
        uint32_t* seg;
        next_q(head, seg);
        uint32_t nwg = (n + BIN_CH - 1) / BIN_CH;
        if (nwg > BIN_MAXWG) nwg = BIN_MAXWG;
        const uint32_t ch = ((n + nwg - 1) / nwg + 63) & ~63u;   // whole waves of items
        const uint32_t vs = nb_bins > nb ? 3u : 0u, nbv = nb << vs;
        hipLaunchKernelGGL(k3_bin_hist, dim3(nwg), dim3(256), 0, st, list, n, nbv, ch, binh, bincol, vs);
        hipLaunchKernelGGL(k3_bin_scan, dim3(1), dim3(1024), 0, st, bincol, binst, nbv, seg);
        hipLaunchKernelGGL(k3_bin_scatter, dim3(nwg), dim3(256), 0, st, list, n, nbv, ch, binh, binst, out, vs);
        HIP_CHECK(hipGetLastError());
        c.qhead = head;
        c.qseg = seg;
    };
    // partition large groups level by level, then run the leaf sorts.  Binned
    // copies go to K2 (free outside doubling) or, while doubling, to the tie
    // list the gather has just consumed (capacity N/2 items either way).
    auto sort_groups = [&]() {
        uint64_t* bout = c.keysrc ? c.L.t[c.tsel ^ 1u] : reinterpret_cast<uint64_t*>(scr.K2);
        uint32_t lsel = 0;
        for (int level = 0;; ++level) {
            read_ctr();
            const uint32_t nl = hctr[C_L0 + lsel];
            if (nl == 0) break;
            if (level > 64) throw StarchError(-10, "bwt3: partition did not converge");
            const bool huge = hctr[C_LM0 + lsel] > HG_MIN;
            static const bool ldbg = getenv("STARCH_BWT_DEBUG") != nullptr;
            if (ldbg) {   // the L list of this level: sizes and shifts
                std::vector<uint64_t> it(nl);
                HIP_CHECK(hipMemcpyAsync(it.data(), c.L.l[lsel], nl * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
                HIP_CHECK(hipStreamSynchronize(st));
                uint64_t tot = 0, big = 0, nbig = 0, mx = 0;
                uint32_t sh[128] = {};
                for (uint64_t v : it) {
                    const uint64_t m = (v >> 12) & 0xFFFFFu;
                    tot += m;
                    mx = m > mx ? m : mx;
                    if (m > HG_MIN) { big += m; ++nbig; }
                    ++sh[v & 127u];
                }
                fprintf(stderr, "[bwt3] rtext %u mode %u level %d: L items %u elems %llu max %llu | >HG_MIN %llu items %llu elems | shifts",
                        c.rtext, c.mode, level, nl, (unsigned long long)tot, (unsigned long long)mx,
                        (unsigned long long)nbig, (unsigned long long)big);
                for (int q = 0; q < 128; ++q)
                    if (sh[q]) fprintf(stderr, " %d:%u", q, sh[q]);
                fprintf(stderr, "\n");
            }
            if (huge) {   // groups above HG_MIN: partitioned by the whole grid
                zero(bit(C_HG) | bit(C_HGC));
                const uint64_t nhm = std::min<uint64_t>(nl, HG_MAXN);   // huge groups: at most this many
                HIP_CHECK(hipMemsetAsync(c.L.hg_info, 0, nhm * 512 * sizeof(uint32_t), st));
                HIP_CHECK(hipMemsetAsync(c.L.hg_vary, 0, nhm * sizeof(uint64_t), st));
                HIP_CHECK(hipMemsetAsync(c.L.hg_flag, 0, nhm * sizeof(uint32_t), st));
                HIP_CHECK(hipMemsetAsync(c.L.hg_eqlt, 0, 2 * nhm * sizeof(uint32_t), st));
                HIP_CHECK(hipMemsetAsync(c.L.hg_mc, 0, 6 * nhm * sizeof(uint32_t), st));
                hipLaunchKernelGGL(k3_hg_pick, dim3((nl + 255) / 256), dim3(256), 0, st, c, c.L.l[lsel], nl);
                hipLaunchKernelGGL(k3_hg_prefix, dim3(1), dim3(1024), 0, st, c);
            }
            bin(c.L.l[lsel], nl, bout);
            c.lsel = lsel ^ 1u;
            zero(bit(C_L0 + (lsel ^ 1u)) | bit(C_LM0 + (lsel ^ 1u)));
            if (huge) {
                const dim3 gh(ncu * 4);
                if (c.keysrc) hipLaunchKernelGGL(k3_hg_hist<true>, gh, dim3(256), 0, st, c);
                else hipLaunchKernelGGL(k3_hg_hist<false>, gh, dim3(256), 0, st, c);
                hipLaunchKernelGGL(k3_hg_scan, dim3((uint32_t)std::min<uint64_t>(nl, HG_MAXN)), dim3(256), 0, st, c);
                if (c.keysrc) hipLaunchKernelGGL(k3_hg_scatter<true>, gh, dim3(256), 0, st, c);
                else hipLaunchKernelGGL(k3_hg_scatter<false>, gh, dim3(256), 0, st, c);
                if (c.keysrc) hipLaunchKernelGGL(k3_hg_move<true>, gh, dim3(256), 0, st, c);
                else hipLaunchKernelGGL(k3_hg_move<false>, gh, dim3(256), 0, st, c);
                hipLaunchKernelGGL(k3_hg_final, gh, dim3(256), 0, st, c);
                HIP_CHECK(hipGetLastError());
            }
#ifndef STARCH_PL_WG
#define STARCH_PL_WG 2   // k3_part_l workgroups per CU
#endif
            if (c.keysrc) hipLaunchKernelGGL(k3_part_l<true>, dim3(ncu * STARCH_PL_WG), dim3(LT), 0, st, c, bout);
            else hipLaunchKernelGGL(k3_part_l<false>, dim3(ncu * STARCH_PL_WG), dim3(LT), 0, st, c, bout);
            HIP_CHECK(hipGetLastError());
#ifdef STARCH_PL_PROF
            {
                unsigned long long h[16];
                HIP_CHECK(hipStreamSynchronize(st));
                HIP_CHECK(hipMemcpyFromSymbol(h, HIP_SYMBOL(g_plprof), sizeof(h)));
                static const unsigned long long z[16] = {};
                HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_plprof), z, sizeof(z)));
                const char* nm[9] = {"zero", "pass1", "scan", "pass2", "final+classify", "groups", "elems", "big", "kernel(all wg)"};
                fprintf(stderr, "[plprof] level %d sdig %u:", level, c.sdig);
                for (int q = 0; q < 9; ++q) fprintf(stderr, " %s %llu", nm[q], h[q]);
                fprintf(stderr, "\n");
            }
#endif
            c.sdig = 0;                  // (deeper levels: the sub-buckets' digits are gathered)
            zero(bit(C_L0 + lsel) | bit(C_LM0 + lsel));
            lsel ^= 1u;
        }
        c.lsel = 0;
        const uint32_t n0 = hctr[C_M0];
        const uint32_t nw = hctr[C_W], ns = hctr[C_S], ns2 = hctr[C_S2], n1 = hctr[C_M1], n2 = hctr[C_M2],
                       n3 = hctr[C_M3];
        static const bool dbg = getenv("STARCH_BWT_DEBUG") != nullptr;
        if (dbg)
            fprintf(stderr, "[bwt3] rtext %u mode %u: W %u S %u S2 %u M0 %u M1 %u M2 %u M3 %u | level-2 %u lsd %u (so far)\n",
                    c.rtext, c.mode, nw, ns, ns2, n0, n1, n2, n3, hctr[C_DBG2], hctr[C_DBGL]);
        // every launch reads its own binned copy; stream order lets them share one buffer
        // grids: a multiple of 8 (static per-XCD segments), about one resident wave of workgroups
        auto g8 = [](uint32_t x) { return dim3((x + 7) / 8 * 8); };
        // static assignment needs every workgroup resident at once: one wave of
        // workgroups, sized by the kernel's occupancy
        auto resident = [&](const void* f, int threads = 256, const char* env = nullptr) {
            int per_cu = 0;
            HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, f, threads, 0));
            // experiments: fewer workgroups per CU (never more than can be resident:
            // the static assignment would wait on workgroups that never start)
            const char* e = env ? getenv(env) : nullptr;
            if (e && atoi(e) > 0 && atoi(e) < per_cu) per_cu = atoi(e);
            if (getenv("STARCH_BWT_DEBUG")) fprintf(stderr, "[bwt3] resident %s: %d per CU\n", env ? env : "-", per_cu);
            return g8((uint32_t)ncu * (uint32_t)(per_cu > 0 ? per_cu : 1));
        };
        // M classes: k3_sort_lds (MSD digit(s) + compare, LSD fallback); S: k3_sort_grp,
        // then the groups it listed as hard (k3_sort_lds) from the class list it consumed.
        // Doubling rounds (keys in K/K2) run their own instantiations.
        const uint32_t* hard_n = c.L.ctr + C_H;
        auto clear_h = [&]() { zero(bit(C_H)); };
        auto sstat = [&](const char* name) {
#ifdef STARCH_SORT_STATS
            HIP_CHECK(hipMemcpyAsync(hctr, c.L.ctr, C_N * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
            HIP_CHECK(hipStreamSynchronize(st));
            fprintf(stderr, "[sort] r%u m%u %-8s groups %u elems %u pathA %u rankwork %u lsdpasses %u hard %u lvl2 %u lsdg %u\n",
                    c.rtext, c.mode, name, hctr[C_STG], hctr[C_STE], hctr[C_STA], hctr[C_STW], hctr[C_STLP], hctr[C_STH],
                    hctr[C_DBG2], hctr[C_DBGL]);
            HIP_CHECK(hipMemsetAsync(c.L.ctr + C_DBG2, 0, 2 * sizeof(uint32_t), st));
            HIP_CHECK(hipMemsetAsync(c.L.ctr + C_STG, 0, 6 * sizeof(uint32_t), st));
#else
            (void)name;
#endif
        };
        auto leaf = [&](auto dbl) {
            constexpr bool D = decltype(dbl)::value;
            // M2 / M3: 8 / 16 waves of 4 rotations per lane (the 4-wave, 8 / 16
            // per lane forms held 168 / 294 VGPRs: 3 / 1 waves per SIMD)
#ifndef STARCH_M_WIDE
#define STARCH_M_WIDE 1
#endif
            constexpr int M2W = STARCH_M_WIDE ? 8 : 4, M2E = STARCH_M_WIDE ? 4 : 8;
            constexpr int M3W = STARCH_M_WIDE ? 16 : 4, M3E = STARCH_M_WIDE ? 4 : 16;
            static const dim3 gm3 = resident(reinterpret_cast<const void*>(&k3_sort_lds<M3W, M3E, D>), 64 * M3W, "STARCH_RES_M3");
            static const dim3 gm2 = resident(reinterpret_cast<const void*>(&k3_sort_lds<M2W, M2E, D>), 64 * M2W, "STARCH_RES_M2");
            static const dim3 gm1 = resident(reinterpret_cast<const void*>(&k3_sort_lds<4, 4, D>), 256, "STARCH_RES_M1");
            static const dim3 gm0 = resident(reinterpret_cast<const void*>(&k3_sort_lds<4, 2, D>), 256, "STARCH_RES_M0");
            static const dim3 gs = resident(reinterpret_cast<const void*>(&k3_sort_grp<1, 2, D>), 256, "STARCH_RES_S");
            static const dim3 gs2 = resident(reinterpret_cast<const void*>(&k3_sort_grp<1, 4, D>), 256, "STARCH_RES_S2");
            static const dim3 gw = resident(reinterpret_cast<const void*>(&k3_sort_w<D>), 256, "STARCH_RES_W");
            if (n3) {
                bin(c.L.m3, n3, bout);
                hipLaunchKernelGGL((k3_sort_lds<M3W, M3E, D>), gm3, dim3(64 * M3W), 0, st, c, bout, nullptr);
                sstat("M3");
            }
            if (n2) {
                bin(c.L.m2, n2, bout);
                hipLaunchKernelGGL((k3_sort_lds<M2W, M2E, D>), gm2, dim3(64 * M2W), 0, st, c, bout, nullptr);
                sstat("M2");
            }
            if (n0) {
                bin(c.L.m0, n0, bout);
#ifdef STARCH_M0_1W
                static const dim3 gm0w = resident(reinterpret_cast<const void*>(&k3_sort_grp<1, 8, D>));
                clear_h();
                hipLaunchKernelGGL((k3_sort_grp<1, 8, D>), gm0w, dim3(256), 0, st, c, bout, c.L.m0);
                hipLaunchKernelGGL((k3_sort_lds<1, 8, D>), dim3(ncu / 2), dim3(256), 0, st, c, c.L.m0, hard_n);
#else
                hipLaunchKernelGGL((k3_sort_lds<4, 2, D>), gm0, dim3(256), 0, st, c, bout, nullptr);
#endif
                sstat("M0");
            }
            if (n1) {
                bin(c.L.m1, n1, bout);
                hipLaunchKernelGGL((k3_sort_lds<4, 4, D>), gm1, dim3(256), 0, st, c, bout, nullptr);
                sstat("M1");
            }
            if (ns) {
                bin(c.L.s, ns, bout);
                clear_h();
                hipLaunchKernelGGL((k3_sort_grp<1, 2, D>), gs, dim3(256), 0, st, c, bout, c.L.s);
                sstat("S");
                hipLaunchKernelGGL((k3_sort_lds<1, 2, D>), dim3(ncu / 2), dim3(256), 0, st, c, c.L.s, hard_n);
                sstat("S-hard");
            }
            if (ns2) {
                bin(c.L.s2, ns2, bout);
#ifdef STARCH_S2_LDS   // experiment: S2 groups by four waves of one rotation per lane
                static const dim3 gs2l = resident(reinterpret_cast<const void*>(&k3_sort_lds<4, 1, D>));
                hipLaunchKernelGGL((k3_sort_lds<4, 1, D>), gs2l, dim3(256), 0, st, c, bout, nullptr);
                sstat("S2");
#else
                clear_h();
                hipLaunchKernelGGL((k3_sort_grp<1, 4, D>), gs2, dim3(256), 0, st, c, bout, c.L.s2);
                sstat("S2");
                hipLaunchKernelGGL((k3_sort_lds<1, 4, D>), dim3(ncu / 2), dim3(256), 0, st, c, c.L.s2, hard_n);
                sstat("S2-hard");
#endif
            }
            if (nw) {
                bin(c.L.w, nw, bout);
                hipLaunchKernelGGL(k3_sort_w<D>, gw, dim3(256), 0, st, c, bout);
                sstat("W");
            }
        };
        if (c.keysrc) leaf(std::true_type{});
        else leaf(std::false_type{});
        HIP_CHECK(hipGetLastError());
        zero((0x3Full << C_W) | bit(C_M0));
    };

    // ---- round 0: packed prefix keys gathered from the PSS by every sort, as
    // the text rounds do (bwt_kmat(): materialised next to SA by the scatter) ----
    static const bool direct = [] { const char* e = getenv("STARCH_SCATTER"); return e && !strcmp(e, "direct"); }();
    const bool kgather = bwt_kgather() && scr.KM0 && !direct;
    if (bwt_kmat() && scr.KM0 && !direct) {   // (the direct scatter writes SA only)
        c.keysrc = 1;
        c.kA = scr.KM0;
        c.kB = scr.KM1;
        c.lA = scr.LS0;
        c.lB = scr.LS1;
    }
    {
        const uint32_t maxw = (uint32_t)pss_words(scr.stride);
        hipLaunchKernelGGL(k3_pss, dim3((maxw + 255) / 256, nb), dim3(256), 0, st, c);
        if (wide) {
            hipLaunchKernelGGL(k3_hist<PNB_WIDE>, dim3(MAXT, nb), dim3(PT), 0, st, c);
            hipLaunchKernelGGL(k3_scan<PNB_WIDE>, dim3(nb), dim3(ST), 0, st, c);
        } else {
            hipLaunchKernelGGL(k3_hist<PNB>, dim3(MAXT, nb), dim3(PT), 0, st, c);
            hipLaunchKernelGGL(k3_scan<PNB>, dim3(nb), dim3(ST), 0, st, c);
        }
        uint32_t* head;
        uint32_t* seg;
        next_q(head, seg);
        c.qhead = head;
        c.qseg = nullptr;
        // about one block in flight per XCD: one 1024-thread workgroup per CU,
        // a block's MAXT tiles spread over its XCD's CUs
        const dim3 gsc((ncu + 7) / 8 * 8);
        // (k3_scatter_lds leaves the L buckets' first partition digits in LL;
        // STARCH_SDIG=0: k3_part_l gathers them instead)
        static const bool sdig_off = [] { const char* e = getenv("STARCH_SDIG"); return e && !strcmp(e, "0"); }();
        c.sdig = direct || sdig_off ? 0u : 1u;
        if (direct && wide) hipLaunchKernelGGL(k3_scatter<PNB_WIDE>, gsc, dim3(SCT), 0, st, c);
        else if (direct) hipLaunchKernelGGL(k3_scatter<PNB>, gsc, dim3(SCT), 0, st, c);
        else if (wide && c.lA && !kgather) hipLaunchKernelGGL((k3_scatter_lds<PNB_WIDE, true>), gsc, dim3(SCT), 0, st, c);
        else if (wide) hipLaunchKernelGGL((k3_scatter_lds<PNB_WIDE, false>), gsc, dim3(SCT), 0, st, c);
        else if (c.lA && !kgather) hipLaunchKernelGGL((k3_scatter_lds<PNB, true>), gsc, dim3(SCT), 0, st, c);
        else hipLaunchKernelGGL((k3_scatter_lds<PNB, false>), gsc, dim3(SCT), 0, st, c);
        if (kgather) {   // keys by position after the scatter (its PSS reads are the key source: keysrc 0 here)
            Ctx ck = c;
            ck.keysrc = 0;
            hipLaunchKernelGGL(k3_keys, dim3(((uint32_t)(scr.stride / 1024) + 7) / 8 * 8 / 2 + 1, nb), dim3(256), 0, st, ck);
        }
        HIP_CHECK(hipGetLastError());
    }
    sort_groups();
    c.sdig = 0;
    c.keysrc = 0;                    // text rounds read the PSS at an offset
    c.kA = scr.K2;
    c.kB = scr.K;
    c.lA = c.lB = nullptr;
    // ---- text rounds: extend the tied rotations' keys from the PSS ----
    uint32_t rtext = 0;
    uint64_t prev_tied = ~0ull;
    bool done = false;
    for (;;) {
        read_ctr();
        const uint32_t nt = hctr[C_T0 + c.tsel];
        const uint64_t tied = hctr[C_TS0 + c.tsel];
        if (nt == 0) { done = true; break; }
        if (rtext == TEXT_ROUNDS || (rtext > 0 && 2 * tied > prev_tied)) break;   // long repeats: double
        prev_tied = tied;
        ++rtext;
        c.rtext = rtext;
        const uint32_t cur = c.tsel;
        c.tsel ^= 1u;
        zero(bit(C_T0 + c.tsel) | bit(C_TS0 + c.tsel));
        hipLaunchKernelGGL(k3_classify_text, dim3((nt + 256 * CT_IPT - 1) / (256 * CT_IPT)), dim3(256), 0, st, c,
                           c.L.t[cur], nt);
        HIP_CHECK(hipGetLastError());
        zero(bit(C_T0 + cur));
        sort_groups();
    }
    // ---- prefix doubling on the blocks still tied ----
    if (!done) {
        const uint32_t nt = hctr[C_T0 + c.tsel];
        const uint64_t* T = c.L.t[c.tsel];
        hipLaunchKernelGGL(k3_mark_tied, dim3((nt + 255) / 256), dim3(256), 0, st, c, T, nt);
        hipLaunchKernelGGL(k3_rk_dense, dim3(64, nb), dim3(256), 0, st, c);
        zero(bit(C_GB));
        hipLaunchKernelGGL(k3_rk_groups, dim3((nt + 3) / 4), dim3(256), 0, st, c, T, nt);
        hipLaunchKernelGGL(k3_rk_big, dim3(ncu * 4), dim3(256), 0, st, c);
        HIP_CHECK(hipGetLastError());
        c.mode = 1;
        c.keysrc = 1;
        for (uint32_t round = 1;; ++round) {
            if (round > 1) read_ctr();
            const uint32_t n2 = hctr[C_T0 + c.tsel];
            if (n2 == 0) break;
            if (round > 40) throw StarchError(-10, "bwt3: doubling did not converge");
            const uint32_t cur = c.tsel;
            c.tsel ^= 1u;
            zero(bit(C_T0 + c.tsel) | bit(C_TS0 + c.tsel) | bit(C_GB));
            hipLaunchKernelGGL(k3_gather, dim3((n2 + 255) / 256), dim3(256), 0, st, c, c.L.t[cur], n2, round, rtext);
            hipLaunchKernelGGL(k3_gather_big, dim3(ncu * 4), dim3(256), 0, st, c);
            HIP_CHECK(hipGetLastError());
            zero(bit(C_T0 + cur));
            sort_groups();
            hipLaunchKernelGGL(k3_round_end, dim3((nb + 255) / 256), dim3(256), 0, st, c, nb);
        }
    }
    hipLaunchKernelGGL(k3_finish, dim3((nb + 255) / 256), dim3(256), 0, st, c, nb, stats);
    HIP_CHECK(hipGetLastError());
#ifdef STARCH_SORT_PROF
    {
        unsigned long long h[16];
        HIP_CHECK(hipStreamSynchronize(st));
        HIP_CHECK(hipMemcpyFromSymbol(h, HIP_SYMBOL(g_sprof), sizeof(h)));
        static const unsigned long long zero[16] = {};
        HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_sprof), zero, sizeof(zero)));
        const char* nm[8] = {"keys-wait+finish", "digit+hist+scan", "digit..place", "next-keys-issue", "ties+heads",
                             "tail(ties..emit)", "rotate+next-vals", "total"};
        for (int e = 0; e < 2; ++e)
            for (int q = 0; q < 8; ++q)
                fprintf(stderr, "[sprof] E=%d %-18s %14llu (%.1f%%)\n", e ? 4 : 2, nm[q], h[8 * e + q],
                        100.0 * (double)h[8 * e + q] / (double)(h[8 * e + 7] ? h[8 * e + 7] : 1));
        unsigned long long h2[16];
        HIP_CHECK(hipMemcpyFromSymbol(h2, HIP_SYMBOL(g_sprof2), sizeof(h2)));
        HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_sprof2), zero, sizeof(zero)));
        const char* nm2[8] = {"finish-keys+diff", "digit count+scan", "scatter+rank", "ties+heads", "emit",
                              "rotate+next-vals", "-", "total"};
        for (int e = 0; e < 2; ++e)
            for (int q = 0; q < 8; ++q)
                fprintf(stderr, "[sprof2] %s %-18s %14llu (%.1f%%)\n", e ? "M1" : "M2/M3", nm2[q], h2[8 * e + q],
                        100.0 * (double)h2[8 * e + q] / (double)(h2[8 * e + 7] ? h2[8 * e + 7] : 1));
    }
#endif
    return !done;   // prefix doubling ran: some block may be periodic (flags bit 0)
}

}  // namespace bz
