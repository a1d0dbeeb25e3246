// starch_amd/csrc/bz2_bwt3.hip -- block sort v3 (the default): a batch-wide
// segmented sort of every rotation of every block, then prefix doubling on
// the rotations whose packed prefix keys tie.
//
// Contract (same as k_bwt, bz2_bwt.hip): SA = the exact sorted order of the
// cyclic rotations of every non-periodic block (BZ2_blockSort's ptr[],
// bz:blocksort.c:1031-1089; unique because all rotations differ), origPtr =
// rank of rotation 0; periodic blocks are flagged (flags bit0) for
// k_fallback_exact, which reproduces fallbackSort's tie order.
//
// Why this shape: a 900 KB transformed-BED block almost never needs more than
// its packed D-symbol prefix (D = 64 / ceil(log2 nInUse) symbols in a u64 key;
// 16 for BED3 text): measured on cfg2 blocks, ~5 tied pairs per 900k
// rotations; cfg4 (narrowPeak) ~0.8 %.  So the work is a segmented sort of
// (block, 64-bit key) pairs, done for ALL blocks of a batch at once so every
// CU is busy, instead of one workgroup walking one block:
//
//   k3_hist     per 32k-rotation tile: keys rolled from the block text in
//               LDS, 4096-bucket histogram of the top 12 key bits
//   k3_scan     per block: bucket starts, per-tile cursors (deterministic
//               offsets, no global atomics), bucket -> size class lists
//   k3_scatter  per tile: keys again, (key, rotation) scattered to buckets
//   k3_part_l   buckets > 4096: MSD partition on the next 8 bits, repeated
//   k3_sort_w   buckets <= 64: one wave, rank by comparison
//   k3_sort_lds buckets <= 256: one wave; <= 1024/2048/4096: one workgroup;
//               keys in registers, stable LSD radix with an LDS exchange,
//               only over the key bits that vary inside the bucket
//   -- every sort writes SA and lists the groups of equal keys --
//   k3_gather_text  text rounds: a tied group is re-sorted by the NEXT D'
//               symbols of each rotation, packed straight from the block text
//               (D' = 52/B so 12 key bits stay free); enough for BED text,
//               where ties are rare and short
//   k3_rk_*     blocks still tied after the text rounds (long repeats,
//               periodic blocks): dense RK = head position of every
//               rotation's group, then prefix doubling --
//   k3_gather   doubling round r: key(q) = RK[(SA[q] + h0*2^(r-1)) mod n] for
//               the tied rotations only; the same part/sort kernels re-sort
//               the groups and update RK.  A round in which no group of a
//               block splits proves the block periodic.
//
// Scratch (BwtScratch, per batch slot, stride S elements): K2/SA = keys and
// rotations in bucket order; K/V = ping-pong for the MSD partition (and the
// per-tile cursors before that); RK ranks; U = wave-class list; U2/V2 = the
// tie-group lists of consecutive rounds (u64 items).
#include "bz2_int.hpp"
#include "bz2_bwt.hpp"

#include <string.h>

#include <algorithm>
#include <vector>

namespace bz {
namespace {

constexpr int PT = 256;                 // partition threads
constexpr int PE = 32;                  // rotations per thread per sub-tile
constexpr int PSUB = PT * PE;           // 8192-rotation sub-tile
constexpr int PSUBS = 4;
constexpr int PTILE = PSUB * PSUBS;     // 32768-rotation tile (one workgroup)
constexpr int PDIG = 12;
constexpr int PNB = 1 << PDIG;          // 4096 top-level buckets per block
constexpr int MAXT = (900064 + PTILE - 1) / PTILE;   // tiles per block (bs <= 9)
// size classes: W rank-by-compare (one wave), S wave-private LDS radix,
// M1..M3 workgroup LDS radix, L MSD partition
constexpr uint32_t W_MAX = 64, S_MAX = 256, M1_MAX = 1024, M2_MAX = 2048, M3_MAX = 4096;
constexpr uint32_t RBITS = 20;          // rank bits (n <= 899,985 < 2^20)

// counters (u32) in the meta buffer
enum { C_W = 0, C_S, C_M1, C_M2, C_M3, C_L0, C_L1, C_T0, C_T1, C_TIE_ELEMS, C_ERR, C_TS0, C_TS1, C_N = 16 };
constexpr uint32_t TEXT_ROUNDS = 4;     // max text-extension rounds before doubling

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

struct Lists {
    uint32_t* ctr;          // C_N counters
    uint64_t* w;            // m <= 64
    uint64_t* s;            // m <= 256
    uint64_t* m1;           // m <= 1024
    uint64_t* m2;           // m <= 2048
    uint64_t* m3;           // m <= 4096
    uint64_t* l[2];         // m > 4096 (MSD partition), ping-pong by level
    uint64_t* t[2];         // tie groups, ping-pong by round
    uint32_t* sD;           // per slot: D (symbols per key)
    uint32_t* sDp;          // per slot: D' (symbols per text-round key, 12 top bits free)
    uint32_t* tied;         // per slot: still tied when doubling starts
    uint8_t* sym;           // per slot: 256-byte symbol map
    uint32_t* gin;          // per slot: groups entering this round
    uint32_t* runs;         // per slot: runs produced this round
    uint32_t* periodic;     // per slot
    uint32_t* rounds;       // per slot: doubling rounds with work
};

struct Ctx {
    BlockDesc* blocks;
    uint32_t b0;
    const uint8_t* blkbytes;
    uint64_t stride;        // block byte stride
    BwtScratch scr;
    Lists L;
    uint32_t lsel;          // L list that part/classify pushes into
    uint32_t tsel;          // tie list the sorts push into
    uint32_t mode;          // 0: SA only (round 0, text rounds); 1: doubling (RK, runs)
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

// push a group [s, s+m) of slot with key bits [0, shift) still unsorted to its size class
__device__ __forceinline__ void wave_classify(const Ctx& c, bool pred, uint32_t slot, uint32_t s, uint32_t m,
                                              uint32_t shift, uint32_t par)
{
    const uint64_t it = mk_item(slot, s, m, shift, par);
    wave_push(c.L.ctr + C_W, c.L.w, pred && m <= W_MAX, it);
    wave_push(c.L.ctr + C_S, c.L.s, pred && m > W_MAX && m <= S_MAX, it);
    wave_push(c.L.ctr + C_M1, c.L.m1, pred && m > S_MAX && m <= M1_MAX, it);
    wave_push(c.L.ctr + C_M2, c.L.m2, pred && m > M1_MAX && m <= M2_MAX, it);
    wave_push(c.L.ctr + C_M3, c.L.m3, pred && m > M2_MAX && m <= M3_MAX, it);
    wave_push(c.L.ctr + C_L0 + c.lsel, c.L.l[c.lsel], pred && m > M3_MAX, it);
}

// symbol map of a block (rank among used byte values), 256 threads or more
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

struct KeyGeo {
    int B, D, KB;
    uint64_t mask;
};
__device__ __forceinline__ KeyGeo key_geo(uint32_t nin)
{
    KeyGeo g;
    g.B = nin > 1 ? bits_for3(nin - 1) : 1;
    g.D = 64 / g.B;
    g.KB = g.D * g.B;
    g.mask = g.KB == 64 ? ~0ull : ((1ull << g.KB) - 1ull);
    return g;
}

// Load the symbols of rotations [r0, r0 + cnt + D - 1) (cyclic) into tb.
__device__ __forceinline__ void load_text(const uint8_t* blk, uint32_t n, uint32_t r0, uint32_t cnt, int D,
                                          const uint8_t* sym, uint8_t* tb)
{
    const int tid = threadIdx.x;
    const uint32_t len = cnt + (uint32_t)D - 1u;
    if ((uint64_t)r0 + PSUB + 64 <= n) {
        const uint32_t* w = reinterpret_cast<const uint32_t*>(blk + r0);
        uint32_t* o = reinterpret_cast<uint32_t*>(tb);
        for (uint32_t i = tid; i < (PSUB + 64) / 4; i += PT) {
            uint32_t x = w[i];
            o[i] = (uint32_t)sym[x & 255u] | ((uint32_t)sym[(x >> 8) & 255u] << 8) |
                   ((uint32_t)sym[(x >> 16) & 255u] << 16) | ((uint32_t)sym[x >> 24] << 24);
        }
    } else {
        for (uint32_t i = tid; i < len; i += PT) {
            uint32_t p = r0 + i;
            if (p >= n) p %= n;
            tb[i] = sym[blk[p]];
        }
    }
}

struct PartSmem {
    uint32_t cnt[PNB];       // histogram / cursors
    uint32_t tot[PNB];       // block totals (scatter: singleton test)
    uint8_t tb[PSUB + 64 + 16];
    uint8_t sym[256];
};

// ---------------------------------------------------------------------------
// k3_hist: per-tile bucket histogram -> thist[slot][tile][4096] (in K)
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(PT) k3_hist(Ctx c)
{
    __shared__ PartSmem sm;
    const int tid = threadIdx.x;
    const uint32_t slot = blockIdx.y, b = c.b0 + slot, tile = blockIdx.x;
    const uint32_t n = c.blocks[b].n;
    const uint32_t t0 = tile * PTILE;
    if (t0 >= n) return;
    uint32_t nin;
    load_sym(c.blocks[b], sm.sym, &nin);
    const KeyGeo g = key_geo(nin);
    const uint8_t* blk = c.blkbytes + (uint64_t)b * c.stride;
    for (int i = tid; i < PNB; i += PT) sm.cnt[i] = 0;
    for (uint32_t sub = 0; sub < PSUBS; ++sub) {
        const uint32_t r0 = t0 + sub * PSUB;
        if (r0 >= n) break;
        const uint32_t cnt = min((uint32_t)PSUB, n - r0);
        __syncthreads();
        load_text(blk, n, r0, cnt, g.D, sm.sym, sm.tb);
        __syncthreads();
        const uint32_t o = tid * PE;
        if (o < cnt) {
            uint64_t key = 0;
            for (int k = 0; k < g.D; ++k) key = (key << g.B) | sm.tb[o + k];
            const uint32_t e = min((uint32_t)PE, cnt - o);
            for (uint32_t k = 0; k < e; ++k) {
                atomicAdd(&sm.cnt[(uint32_t)(key >> (g.KB - PDIG))], 1u);
                key = ((key << g.B) | sm.tb[o + k + g.D]) & g.mask;
            }
        }
    }
    __syncthreads();
    uint32_t* th = reinterpret_cast<uint32_t*>(c.scr.K + (uint64_t)slot * c.scr.stride) + (uint64_t)tile * PNB;
    for (int i = tid; i < PNB; i += PT) th[i] = sm.cnt[i];
}

// ---------------------------------------------------------------------------
// k3_scan: per block -- totals, bucket starts, per-tile cursors, class lists
// ---------------------------------------------------------------------------
constexpr int ST = 1024;              // k3_scan threads: 4 buckets each

__global__ void __launch_bounds__(ST) k3_scan(Ctx c)
{
    __shared__ uint32_t scan_sh[ST / 64 + 1];
    __shared__ uint8_t sym[256];
    const int tid = threadIdx.x;
    const uint32_t slot = blockIdx.x, b = c.b0 + slot;
    const uint32_t n = c.blocks[b].n;
    uint32_t nin;
    load_sym(c.blocks[b], sym, &nin);
    const KeyGeo g = key_geo(nin);
    if (tid == 0) {
        c.blocks[b].n_in_use = nin;
        c.L.sD[slot] = (uint32_t)g.D;
        c.L.sDp[slot] = (uint32_t)((64 - PDIG) / g.B);
    }
    if (tid < 256) c.L.sym[(uint64_t)slot * 256 + tid] = sym[tid];
    const uint32_t ntile = (n + PTILE - 1) / PTILE;
    uint4* th = reinterpret_cast<uint4*>(c.scr.K + (uint64_t)slot * c.scr.stride);   // [tile][PNB/4]
    uint4* tot = th + (uint64_t)MAXT * (PNB / 4);
    uint4 a = make_uint4(0, 0, 0, 0);
    for (uint32_t k = 0; k < ntile; ++k) {
        const uint4 x = th[(uint64_t)k * (PNB / 4) + tid];
        a.x += x.x; a.y += x.y; a.z += x.z; a.w += x.w;
    }
    tot[tid] = a;
    const uint32_t sum = a.x + a.y + a.z + a.w;
    const uint32_t pre = block_excl_scan_add<uint32_t>(sum, scan_sh, (uint32_t*)nullptr);
    uint4 run = make_uint4(pre, pre + a.x, pre + a.x + a.y, pre + a.x + a.y + a.z);
    for (uint32_t k = 0; k < ntile; ++k) {
        uint4& x = th[(uint64_t)k * (PNB / 4) + tid];
        const uint4 v = x;
        x = run;
        run.x += v.x; run.y += v.y; run.z += v.z; run.w += v.w;
    }
    const uint32_t shift = (uint32_t)(g.KB - PDIG);
    const uint32_t cnt4[4] = {a.x, a.y, a.z, a.w};
    uint32_t st = pre;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        wave_classify(c, cnt4[q] >= 2, slot, st, cnt4[q], shift, 0);
        st += cnt4[q];
    }
}

// ---------------------------------------------------------------------------
// k3_scatter: (key, rotation) -> bucket order in (K2, SA); singletons final
// ---------------------------------------------------------------------------
// Workgroup L of a 1-D grid -> (slot, tile) with slot = L mod 8 inside each
// group of 8 slots: workgroups are dealt round-robin over the 8 XCDs, so all
// tiles of a block run on one XCD and its scattered writes meet in one L2
// (placement is a speed matter only, MI355X_MICROARCH.md "Workgroup dispatch").
__device__ __forceinline__ bool xcd_slot_tile(uint32_t L, uint32_t ntile, uint32_t nb, uint32_t& slot,
                                              uint32_t& tile)
{
    const uint32_t grp = L / (8u * ntile), r = L % (8u * ntile);
    slot = grp * 8u + (r & 7u);
    tile = r >> 3;
    return slot < nb;
}

__global__ void __launch_bounds__(PT) k3_scatter(Ctx c, uint32_t nb)
{
    __shared__ PartSmem sm;
    const int tid = threadIdx.x;
    uint32_t slot, tile;
    if (!xcd_slot_tile(blockIdx.x, MAXT, nb, slot, tile)) return;
    const uint32_t b = c.b0 + slot;
    const uint32_t n = c.blocks[b].n;
    const uint32_t t0 = tile * PTILE;
    if (t0 >= n) return;
    uint32_t nin;
    load_sym(c.blocks[b], sm.sym, &nin);
    const KeyGeo g = key_geo(nin);
    const uint8_t* blk = c.blkbytes + (uint64_t)b * c.stride;
    const uint64_t so = (uint64_t)slot * c.scr.stride;
    const uint32_t* th = reinterpret_cast<const uint32_t*>(c.scr.K + so) + (uint64_t)tile * PNB;
    const uint32_t* tot = reinterpret_cast<const uint32_t*>(c.scr.K + so) + (uint64_t)MAXT * PNB;
    for (int i = tid; i < PNB; i += PT) { sm.cnt[i] = th[i]; sm.tot[i] = tot[i]; }
    uint64_t* K2 = c.scr.K2 + so;
    uint32_t* SA = c.scr.SA + so;
    for (uint32_t sub = 0; sub < PSUBS; ++sub) {
        const uint32_t r0 = t0 + sub * PSUB;
        if (r0 >= n) break;
        const uint32_t cnt = min((uint32_t)PSUB, n - r0);
        __syncthreads();
        load_text(blk, n, r0, cnt, g.D, sm.sym, sm.tb);
        __syncthreads();
        const uint32_t o = tid * PE;
        if (o < cnt) {
            uint64_t key = 0;
            for (int k = 0; k < g.D; ++k) key = (key << g.B) | sm.tb[o + k];
            const uint32_t e = min((uint32_t)PE, cnt - o);
            for (uint32_t k = 0; k < e; ++k) {
                const uint32_t bk = (uint32_t)(key >> (g.KB - PDIG));
                const uint32_t p = atomicAdd(&sm.cnt[bk], 1u);
                const uint32_t r = r0 + o + k;
                K2[p] = key;
                SA[p] = r;
                if (r == 0 && sm.tot[bk] == 1u) c.blocks[b].orig_ptr = p;
                key = ((key << g.B) | sm.tb[o + k + g.D]) & g.mask;
            }
        }
    }
}

// ---------------------------------------------------------------------------
// k3_part_l: MSD partition of one large group on its next <= 8 key bits
// ---------------------------------------------------------------------------
constexpr int LT = 512;
constexpr int LW = LT / 64;

__global__ void __launch_bounds__(LT) k3_part_l(Ctx c, const uint64_t* __restrict__ items)
{
    __shared__ uint32_t wh[LW][256];
    __shared__ uint32_t st[256], cur[256], cntd[256];
    __shared__ uint32_t scan_sh[LW + 1];
    __shared__ uint32_t big[257];
    const int tid = threadIdx.x, wid = tid >> 6;
    const uint64_t item = items[blockIdx.x];
    const uint32_t slot = it_slot(item), s = it_start(item), m = it_size(item), shift = it_shift(item),
                   par = it_par(item);
    const uint32_t b = c.b0 + slot;
    const uint64_t base = (uint64_t)slot * c.scr.stride + s;
    const uint64_t* sk = (par ? c.scr.K : c.scr.K2) + base;
    const uint32_t* sv = (par ? c.scr.V : c.scr.SA) + base;
    uint64_t* dk = (par ? c.scr.K2 : c.scr.K) + base;
    uint32_t* dv = (par ? c.scr.SA : c.scr.V) + base;
    uint32_t* SA = c.scr.SA + base;
    uint32_t* RK = c.scr.RK + (uint64_t)slot * c.scr.stride;
    const uint32_t n = c.blocks[b].n;
    const uint8_t* blk = c.blkbytes + (uint64_t)b * c.stride;
    const uint32_t db = shift < 8 ? shift : 8;
    const uint32_t sh2 = shift - db;
    const uint64_t dmask = (1ull << db) - 1ull;
    for (int i = tid; i < LW * 256; i += LT) (&wh[0][0])[i] = 0;
    if (tid == 0) big[256] = 0;
    __syncthreads();
    for (uint32_t i = tid; i < m; i += LT) atomicAdd(&wh[wid][(uint32_t)((sk[i] >> sh2) & dmask)], 1u);
    __syncthreads();
    uint32_t tcount = 0;
    if (tid < 256) for (int w = 0; w < LW; ++w) tcount += wh[w][tid];
    const uint32_t pre = block_excl_scan_add<uint32_t>(tid < 256 ? tcount : 0u, scan_sh, (uint32_t*)nullptr);
    if (tid < 256) { st[tid] = pre; cur[tid] = pre; cntd[tid] = tcount; }
    __syncthreads();
    for (uint32_t i = tid; i < m; i += LT) {
        const uint64_t k = sk[i];
        const uint32_t p = atomicAdd(&cur[(uint32_t)((k >> sh2) & dmask)], 1u);
        dk[p] = k;
        dv[p] = sv[i];
    }
    __syncthreads();
    uint32_t nruns = 0;
    if (tid < 256) {
        const uint32_t cc = cntd[tid], ss = st[tid];
        if (cc == 1) {
            const uint32_t v = dv[ss];
            if (!par) SA[ss] = v;
            if (c.mode) RK[v] = s + ss;
            if (v == 0) c.blocks[b].orig_ptr = s + ss;
            nruns = 1;
        } else if (cc > M3_MAX && sh2 == 0) {
            big[atomicAdd(&big[256], 1u)] = tid;   // all keys equal: one group
            nruns = 1;
        }
    }
    if (tid < 256) {
        const uint32_t cc = cntd[tid];
        const bool push = cc >= 2 && !(cc > M3_MAX && sh2 == 0);
        wave_classify(c, push, slot, s + st[tid], cc, sh2, par ^ 1u);
    }
    if (tid < 256) {
        const uint32_t r = wave_reduce_add(nruns);
        if (c.mode && (tid & 63) == 0 && r) atomicAdd(&c.L.runs[slot], r);
    }
    __syncthreads();
    const uint32_t nbig = big[256];
    for (uint32_t q = 0; q < nbig; ++q) {
        const uint32_t d = big[q];
        const uint32_t ss = st[d], cc = cntd[d];
        for (uint32_t i = tid; i < cc; i += LT) {
            const uint32_t v = dv[ss + i];
            if (!par) SA[ss + i] = v;
            if (c.mode) RK[v] = s + ss;
            if (v == 0) c.blocks[b].orig_ptr = s + ss + i;
        }
        if (tid == 0) {
            const uint32_t o = atomicAdd(c.L.ctr + C_T0 + c.tsel, 1u);
            c.L.t[c.tsel][o] = mk_item(slot, s + ss, cc, 0, 0);
            atomicAdd(c.L.ctr + C_TS0 + c.tsel, cc);
        }
    }
}

// Finish a sorted group: SA, RK, origPtr, tie groups, run count.
// Called by every thread of a wave with (j = sorted position in the group,
// key, val, valid, hp = head position of j's run, end = j ends its run).
__device__ __forceinline__ void emit_sorted(const Ctx& c, uint32_t slot, uint32_t s, uint32_t j, uint32_t v,
                                            uint32_t llb, bool valid, uint32_t hp, bool end, uint32_t& runs_acc)
{
    const uint64_t so = (uint64_t)slot * c.scr.stride;
    if (valid) {
        c.scr.SA[so + s + j] = v;
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

// ---------------------------------------------------------------------------
// k3_sort_w: groups of <= 64, one wave each
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k3_sort_w(Ctx c, const uint64_t* __restrict__ items, uint32_t nitems)
{
    __shared__ uint64_t skey[4][W_MAX + 1];
    __shared__ uint32_t sval[4][W_MAX];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint32_t idx = blockIdx.x * 4 + wid;
    if (idx >= nitems) return;                     // whole wave; no workgroup barrier below
    const uint64_t item = items[idx];
    const uint32_t slot = it_slot(item), s = it_start(item), m = it_size(item), par = it_par(item);
    const uint64_t base = (uint64_t)slot * c.scr.stride + s;
    const uint64_t* sk = (par ? c.scr.K : c.scr.K2) + base;
    const uint32_t* sv = (par ? c.scr.V : c.scr.SA) + base;
    const bool valid = (uint32_t)lane < m;
    const uint64_t k = valid ? sk[lane] : ~0ull;
    const uint32_t v = valid ? sv[lane] : 0u;
    const uint32_t vl = v;
    uint32_t r = 0;
    for (uint32_t j = 0; j < m; ++j) {
        const uint64_t kj = __shfl(k, (int)j, 64);
        r += (kj < k || (kj == k && (int)j < lane)) ? 1u : 0u;
    }
    if (valid) { skey[wid][r] = k; sval[wid][r] = vl; }
    wave_sync_lds3();
    const uint64_t key = valid ? skey[wid][lane] : 0;
    const uint32_t val = valid ? sval[wid][lane] : 0;
    const bool head = valid && (lane == 0 || skey[wid][lane - 1] != key);
    const bool end = valid && ((uint32_t)lane + 1 == m || skey[wid][lane + 1] != key);
    const uint32_t hp = wave_incl_scan_max<uint32_t>(head ? (uint32_t)lane : 0u);
    uint32_t runs = 0;
    emit_sorted(c, slot, s, (uint32_t)lane, val, 0u, valid, hp, end, runs);
    if (c.mode && lane == 0) atomicAdd(&c.L.runs[slot], runs);
}

// ---------------------------------------------------------------------------
// k3_sort_lds<NW, E>: groups of <= NW*64*E rotations sorted by NW waves
// (NW = 1: four independent wave-private sorts per workgroup, no workgroup
// barrier; NW = 4: one group per workgroup).  Stable LSD radix on 8-bit
// digits over only the key bits that vary inside the group.  The group-local
// index rides in the key's constant top bits (every group's keys share at
// least 12 top bits: the bucket digit, the partition digits, or the unused
// bits of a < 2^20 rank), so each pass exchanges one u64 per element through
// LDS.  Ranking: 8 ballots give each lane its peers with the same digit; one
// lane per peer set adds the set's size to the wave's digit counter with a
// returning LDS atomic (all E atomics in flight, in program order).
// ---------------------------------------------------------------------------
template <int NW>
__device__ __forceinline__ void gsync()
{
    if constexpr (NW == 1) wave_sync_lds3();
    else __syncthreads();
}

template <int NW, int E>
__global__ void __launch_bounds__(256) k3_sort_lds(Ctx c, const uint64_t* __restrict__ items, uint32_t nitems)
{
    constexpr int IPW = 4 / NW;                    // groups per workgroup
    constexpr int CAP = NW * 64 * E;
    constexpr int IDXB = CAP <= 256 ? 8 : 12;      // packed local index bits
    constexpr int KEYB = 64 - IDXB;
    constexpr uint64_t KMASK = (1ull << KEYB) - 1ull;
    constexpr int DPT = 256 / (64 * NW);           // digits per thread in the offset scan
    static_assert(CAP <= (1 << IDXB), "index does not fit");
    constexpr int DB = CAP <= 256 ? 8 : (CAP <= 1024 ? 10 : 11);   // MSD digit bits
    constexpr int NBIN = 1 << DB;
    constexpr int T = NW * 64;
    constexpr int BPT = NBIN / T;                  // bins per thread
    constexpr uint32_t LIMIT = 256 / E;            // largest sub-bucket ranked by comparison
    __shared__ uint64_t xk_all[IPW][CAP];
    __shared__ uint32_t vb_all[IPW][CAP];          // rotations by group index
    __shared__ uint32_t bst_all[IPW][NBIN + 1];   // sub-bucket starts
    __shared__ uint32_t bcur_all[IPW][NBIN];      // scatter cursors
    __shared__ uint32_t cnt_all[4][256];
    __shared__ uint32_t sc_all[IPW][NW + 1];
    __shared__ uint64_t red_all[4];
    __shared__ uint32_t wmax_all[4];
    __shared__ uint32_t flag_all[4];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int g = wave / NW, wid = wave % NW, w0 = g * NW;
    const uint32_t gi = blockIdx.x * IPW + g;
    if (gi >= nitems) return;                      // NW = 1: per wave; NW = 4: IPW = 1, whole workgroup
    uint64_t* xk = xk_all[g];
    uint32_t* wcnt = cnt_all[wave];
    uint32_t* sc = sc_all[g];
    const uint64_t item = items[gi];
    const uint32_t slot = it_slot(item), s = it_start(item), m = it_size(item), par = it_par(item);
    const uint64_t base = (uint64_t)slot * c.scr.stride + s;
    const uint64_t* sk = (par ? c.scr.K : c.scr.K2) + base;
    const uint32_t* sv = (par ? c.scr.V : c.scr.SA) + base;
    const uint64_t lt = lanemask_lt();

    uint64_t k[E];
    const uint64_t k0 = sk[0];
    uint64_t diff = 0;
    {
        uint32_t vv[E];
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const uint32_t i = (uint32_t)(wid * 64 * E + e * 64 + lane);
            vv[e] = i < m ? sv[i] : 0u;
        }
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const uint32_t i = (uint32_t)(wid * 64 * E + e * 64 + lane);
            if (i < m) {
                const uint64_t x = sk[i];
                diff |= x ^ k0;
                k[e] = (x & KMASK) | ((uint64_t)i << KEYB);
                vb_all[g][i] = vv[e];
            } else {
                k[e] = ~0ull;                          // pads: max key, last in stable order
            }
        }
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) diff |= __shfl_xor(diff, d, 64);
    if constexpr (NW > 1) {
        if (lane == 0) red_all[wave] = diff;
        __syncthreads();
        diff = 0;
#pragma unroll
        for (int w = 0; w < NW; ++w) diff |= red_all[w0 + w];
    }
    if ((diff >> KEYB) && tid % (64 * NW) == 0) atomicOr(&c.L.ctr[C_ERR], 1u);   // top bits not shared

    bool moved = false;
    const uint64_t kdiff = diff & KMASK;
    if (kdiff) {
        // ---- one MSD digit (the DB bits below the highest varying bit), then every
        // element ranks itself inside its sub-bucket by direct comparison ----
        uint32_t* bst = bst_all[g];
        uint32_t* bcur = bcur_all[g];
        const int tg = wid * 64 + lane;
        const int hb = 63 - __clzll((long long)kdiff);
        const int lo = hb + 1 - DB > 0 ? hb + 1 - DB : 0;
        for (int q = tg; q < NBIN; q += T) bcur[q] = 0;
        gsync<NW>();
        uint32_t dg[E];
#pragma unroll
        for (int e = 0; e < E; ++e) {
            dg[e] = (uint32_t)(((k[e] & KMASK) >> lo) & (uint64_t)(NBIN - 1));
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
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) { const uint32_t o = __shfl_xor(mx, d, 64); mx = o > mx ? o : mx; }
        if constexpr (NW > 1) {
            if (lane == 63) sc[wid] = incl;
            if (lane == 0) wmax_all[wave] = mx;
            __syncthreads();
            for (int w = 0; w < wid; ++w) run += sc[w];
            mx = 0;
            for (int w = 0; w < NW; ++w) mx = wmax_all[w0 + w] > mx ? wmax_all[w0 + w] : mx;
        }
        if (mx <= LIMIT) {                         // uniform per group
#pragma unroll
            for (int q = 0; q < BPT; ++q) { bst[tg * BPT + q] = run; bcur[tg * BPT + q] = run; run += loc[q]; }
            if (tg == T - 1) bst[NBIN] = run;
            gsync<NW>();
            uint32_t p[E];
#pragma unroll
            for (int e = 0; e < E; ++e) {
                p[e] = 0;
                if ((uint32_t)(wid * 64 * E + e * 64 + lane) < m) { p[e] = atomicAdd(&bcur[dg[e]], 1u); xk[p[e]] = k[e]; }
            }
            gsync<NW>();
#pragma unroll
            for (int e = 0; e < E; ++e) {
                const uint32_t i = (uint32_t)(wid * 64 * E + e * 64 + lane);
                if (i < m) {
                    const uint32_t bs = bst[dg[e]], be = bst[dg[e] + 1];
                    const uint64_t km = k[e] & KMASK;
                    uint32_t r = 0;
                    for (uint32_t q = bs; q < be; ++q) {
                        const uint64_t kq = xk[q] & KMASK;
                        r += (kq < km || (kq == km && q < p[e])) ? 1u : 0u;
                    }
                    p[e] = bs + r;
                } else {
                    p[e] = i;                      // pads keep the tail
                }
            }
            gsync<NW>();
#pragma unroll
            for (int e = 0; e < E; ++e) xk[p[e]] = k[e];
            gsync<NW>();
#pragma unroll
            for (int e = 0; e < E; ++e) k[e] = xk[wid * 64 * E + e * 64 + lane];
            moved = true;
        } else {
            gsync<NW>();                           // bcur/sc reads done before the LSD passes
        }
    }
    bool lsd_moved = false;
    for (int dbit = 0; dbit < KEYB && !moved; dbit += 8) {
        if ((kdiff >> dbit & 0xffull) == 0) continue;    // uniform per group
        for (int q = lane; q < 256; q += 64) wcnt[q] = 0;
        wave_sync_lds3();
        uint32_t dg[E], rk[E], ld[E], ret[E];
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const uint32_t d = (uint32_t)(((k[e] & KMASK) >> dbit) & 255u);
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
            uint32_t loc[DPT], sum = 0;
#pragma unroll
            for (int q = 0; q < DPT; ++q) {
                uint32_t a = 0;
#pragma unroll
                for (int w = 0; w < NW; ++w) a += cnt_all[w0 + w][t * DPT + q];
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
            for (int q = 0; q < DPT; ++q) {
                uint32_t r = run;
#pragma unroll
                for (int w = 0; w < NW; ++w) {
                    const uint32_t x = cnt_all[w0 + w][t * DPT + q];
                    cnt_all[w0 + w][t * DPT + q] = r;
                    r += x;
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
        if (j > 0 && j < m && ((xk[j - 1] ^ k[e]) & KMASK) == 0) tie_here = true;
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
            const bool head = j < m && (j == 0 || ((xk[j - 1] ^ k[e]) & KMASK) != 0);
            uint32_t x = wave_incl_scan_max<uint32_t>(head ? j : 0u);
            x = x > carry ? x : carry;
            hp[e] = x;
            carry = __shfl(x, 63, 64);
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
    // values were loaded (and their last-column bytes gathered) before the sort;
    // every global read of the group's SA range happened before any write
    uint32_t runs = 0;
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const uint32_t j = (uint32_t)(wid * 64 * E + e * 64 + lane);
        const bool valid = j < m;
        const uint32_t vb = valid ? vb_all[g][(uint32_t)(k[e] >> KEYB)] : 0u;
        const bool end = valid && (!ties || j + 1 == m || ((xk[j + 1] ^ k[e]) & KMASK) != 0);
        emit_sorted(c, slot, s, j, vb, 0u, valid, hp[e], end, runs);
    }
    if (c.mode && lane == 0 && runs) atomicAdd(&c.L.runs[slot], runs);
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
        const uint64_t h = ((uint64_t)c.L.sD[slot] + (uint64_t)rtext * c.L.sDp[slot]) << (round - 1);
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
    uint64_t bigm = __ballot(active && m > 64);
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
    wave_classify(c, active, slot, s, m, RBITS, 0);
    if (active) atomicAdd(&c.L.gin[slot], 1u);
    const uint32_t tied = wave_reduce_add<uint32_t>(active ? m : 0u);
    if (lane == 0 && tied) atomicAdd(&c.L.ctr[C_TIE_ELEMS], tied);
}

// text round r >= 1: key(q) = D' symbols of rotation SA[q] starting D + (r-1)*D'
// symbols in (the group already agrees on everything before that)
__device__ __forceinline__ uint64_t text_key(const uint8_t* blk, const uint8_t* sym, uint32_t n, uint32_t pos,
                                             uint32_t Dp, uint32_t B)
{
    uint64_t key = 0;
    for (uint32_t k = 0; k < Dp; ++k) {
        key = (key << B) | sym[blk[pos]];
        if (++pos == n) pos = 0;
    }
    return key;
}

__global__ void __launch_bounds__(256) k3_gather_text(Ctx c, const uint64_t* __restrict__ items, uint32_t nitems,
                                                       uint32_t r)
{
    const int lane = threadIdx.x & 63;
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    const bool active = i < nitems;
    const uint64_t item = active ? items[i] : 0;
    const uint32_t slot = it_slot(item), s = it_start(item), m = it_size(item);
    const uint32_t b = c.b0 + slot;
    const uint32_t n = c.blocks[b].n;
    const uint32_t D = c.L.sD[slot], Dp = c.L.sDp[slot];
    uint32_t B = 8;
    for (uint32_t q = 1; q <= 8; ++q)
        if (64 / q == D) { B = q; break; }       // D = 64 / B is distinct for B = 1..8
    const uint32_t off = (uint32_t)(((uint64_t)D + (uint64_t)(r - 1) * Dp) % n);
    const uint8_t* blk = c.blkbytes + (uint64_t)b * c.stride;
    const uint8_t* sym = c.L.sym + (uint64_t)slot * 256;
    const uint64_t so = (uint64_t)slot * c.scr.stride;
    if (active && m <= 64) {
        for (uint32_t q = s; q < s + m; ++q) {
            uint32_t pos = c.scr.SA[so + q] + off;
            if (pos >= n) pos -= n;
            c.scr.K2[so + q] = text_key(blk, sym, n, pos, Dp, B);
        }
    }
    uint64_t bigm = __ballot(active && m > 64);
    while (bigm) {
        const int l = __ffsll((unsigned long long)bigm) - 1;
        bigm &= bigm - 1;
        const uint32_t ls = __shfl(s, l, 64), lm = __shfl(m, l, 64), lslot = __shfl(slot, l, 64);
        const uint32_t ln = __shfl(n, l, 64), loff = __shfl(off, l, 64), lDp = __shfl(Dp, l, 64),
                       lB = __shfl(B, l, 64);
        const uint8_t* lblk = c.blkbytes + (uint64_t)(c.b0 + lslot) * c.stride;
        const uint8_t* lsym = c.L.sym + (uint64_t)lslot * 256;
        const uint64_t lso = (uint64_t)lslot * c.scr.stride;
        for (uint32_t q = ls + lane; q < ls + lm; q += 64) {
            uint32_t pos = c.scr.SA[lso + q] + loff;
            if (pos >= ln) pos -= ln;
            c.scr.K2[lso + q] = text_key(lblk, lsym, ln, pos, lDp, lB);
        }
    }
    wave_classify(c, active, slot, s, m, Dp * B, 0);
    const uint32_t tied = wave_reduce_add<uint32_t>(active ? m : 0u);
    if (lane == 0 && tied) atomicAdd(&c.L.ctr[C_TIE_ELEMS], tied);
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
    for (uint32_t q = s + lane; q < s + m; q += 64) c.scr.RK[so + c.scr.SA[so + q]] = s;
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

}  // namespace

// Host orchestration.  A handful of host round trips per batch (list sizes).
void launch_bwt3(BlockDesc* blocks, uint32_t b0, uint32_t nb, const uint8_t* blkbytes, uint64_t stride,
                 const BwtScratch& scr, DevBuf& meta, uint32_t* hctr, unsigned long long* stats, hipStream_t st)
{
    if (nb == 0) return;
    if (nb > 4095) throw StarchError(-2, "bwt3: batch too large");
    if (2 * scr.stride < (uint64_t)(MAXT + 1) * PNB) throw StarchError(-2, "bwt3: block stride too small");
    const uint64_t N = (uint64_t)nb * scr.stride;
    const uint64_t cap_s = N / (W_MAX + 1) + 64, cap_m1 = N / (S_MAX + 1) + 64, cap_m2 = N / (M1_MAX + 1) + 64,
                   cap_m3 = N / (M2_MAX + 1) + 64, cap_l = N / (M3_MAX + 1) + 64;
    const uint64_t words = C_N * 2 + 7ull * nb + 64ull * nb + 2 * (cap_s + cap_m1 + cap_m2 + cap_m3 + 2 * cap_l) + 64;
    uint32_t* mw = meta.as<uint32_t>(words);
    Ctx c;
    c.blocks = blocks;
    c.b0 = b0;
    c.blkbytes = blkbytes;
    c.stride = stride;
    c.scr = scr;
    c.L.ctr = mw;
    c.L.sD = mw + 2 * C_N;
    c.L.gin = c.L.sD + nb;
    c.L.runs = c.L.gin + nb;
    c.L.periodic = c.L.runs + nb;
    c.L.rounds = c.L.periodic + nb;
    c.L.sDp = c.L.rounds + nb;
    c.L.tied = c.L.sDp + nb;
    c.L.sym = reinterpret_cast<uint8_t*>(c.L.tied + nb);
    uintptr_t p = reinterpret_cast<uintptr_t>(c.L.sym + 256ull * nb);
    p = (p + 7) & ~(uintptr_t)7;
    c.L.s = reinterpret_cast<uint64_t*>(p);
    c.L.m1 = c.L.s + cap_s;
    c.L.m2 = c.L.m1 + cap_m1;
    c.L.m3 = c.L.m2 + cap_m2;
    c.L.l[0] = c.L.m3 + cap_m3;
    c.L.l[1] = c.L.l[0] + cap_l;
    c.L.w = reinterpret_cast<uint64_t*>(scr.U);
    c.L.t[0] = reinterpret_cast<uint64_t*>(scr.U2);
    c.L.t[1] = reinterpret_cast<uint64_t*>(scr.V2);
    c.lsel = 0;
    c.tsel = 0;
    c.mode = 0;
    HIP_CHECK(hipMemsetAsync(mw, 0, (2 * C_N + 7ull * nb) * sizeof(uint32_t), st));

    auto read_ctr = [&]() {
        HIP_CHECK(hipMemcpyAsync(hctr, c.L.ctr, C_N * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
        HIP_CHECK(hipStreamSynchronize(st));
        if (hctr[C_ERR]) throw StarchError(-11, "bwt3: group keys do not share 12 top bits");
    };
    // partition large groups level by level, then run the leaf sorts
    auto sort_groups = [&]() {
        uint32_t lsel = 0;
        for (int level = 0;; ++level) {
            read_ctr();
            const uint32_t nl = hctr[C_L0 + lsel];
            if (nl == 0) break;
            if (level > 64) throw StarchError(-10, "bwt3: partition did not converge");
            c.lsel = lsel ^ 1u;
            HIP_CHECK(hipMemsetAsync(c.L.ctr + C_L0 + (lsel ^ 1u), 0, sizeof(uint32_t), st));
            hipLaunchKernelGGL(k3_part_l, dim3(nl), dim3(LT), 0, st, c, c.L.l[lsel]);
            HIP_CHECK(hipGetLastError());
            HIP_CHECK(hipMemsetAsync(c.L.ctr + C_L0 + lsel, 0, sizeof(uint32_t), st));
            lsel ^= 1u;
        }
        c.lsel = 0;
        const uint32_t nw = hctr[C_W], ns = hctr[C_S], n1 = hctr[C_M1], n2 = hctr[C_M2], n3 = hctr[C_M3];
        // largest groups first so the long workgroups start early
        if (n3) hipLaunchKernelGGL((k3_sort_lds<4, 16>), dim3(n3), dim3(256), 0, st, c, c.L.m3, n3);
        if (n2) hipLaunchKernelGGL((k3_sort_lds<4, 8>), dim3(n2), dim3(256), 0, st, c, c.L.m2, n2);
        if (n1) hipLaunchKernelGGL((k3_sort_lds<4, 4>), dim3(n1), dim3(256), 0, st, c, c.L.m1, n1);
        if (ns) hipLaunchKernelGGL((k3_sort_lds<1, 4>), dim3((ns + 3) / 4), dim3(256), 0, st, c, c.L.s, ns);
        if (nw) hipLaunchKernelGGL(k3_sort_w, dim3((nw + 3) / 4), dim3(256), 0, st, c, c.L.w, nw);
        HIP_CHECK(hipGetLastError());
        HIP_CHECK(hipMemsetAsync(c.L.ctr + C_W, 0, 5 * sizeof(uint32_t), st));
    };

    // ---- round 0: packed prefix keys ----
    hipLaunchKernelGGL(k3_hist, dim3(MAXT, nb), dim3(PT), 0, st, c);
    hipLaunchKernelGGL(k3_scan, dim3(nb), dim3(ST), 0, st, c);
    hipLaunchKernelGGL(k3_scatter, dim3(MAXT * ((nb + 7) / 8 * 8)), dim3(PT), 0, st, c, nb);
    HIP_CHECK(hipGetLastError());
    sort_groups();
    // ---- text rounds: extend the tied rotations' keys from the block text ----
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
        const uint32_t cur = c.tsel;
        c.tsel ^= 1u;
        HIP_CHECK(hipMemsetAsync(c.L.ctr + C_T0 + c.tsel, 0, sizeof(uint32_t), st));
        HIP_CHECK(hipMemsetAsync(c.L.ctr + C_TS0 + c.tsel, 0, sizeof(uint32_t), st));
        hipLaunchKernelGGL(k3_gather_text, dim3((nt + 255) / 256), dim3(256), 0, st, c, c.L.t[cur], nt, rtext);
        HIP_CHECK(hipGetLastError());
        HIP_CHECK(hipMemsetAsync(c.L.ctr + C_T0 + cur, 0, sizeof(uint32_t), st));
        sort_groups();
    }
    // ---- prefix doubling on the blocks still tied ----
    if (!done) {
        const uint32_t nt = hctr[C_T0 + c.tsel];
        const uint64_t* T = c.L.t[c.tsel];
        hipLaunchKernelGGL(k3_mark_tied, dim3((nt + 255) / 256), dim3(256), 0, st, c, T, nt);
        hipLaunchKernelGGL(k3_rk_dense, dim3(64, nb), dim3(256), 0, st, c);
        hipLaunchKernelGGL(k3_rk_groups, dim3((nt + 3) / 4), dim3(256), 0, st, c, T, nt);
        HIP_CHECK(hipGetLastError());
        c.mode = 1;
        for (uint32_t round = 1;; ++round) {
            if (round > 1) read_ctr();
            const uint32_t n2 = hctr[C_T0 + c.tsel];
            if (n2 == 0) break;
            if (round > 40) throw StarchError(-10, "bwt3: doubling did not converge");
            const uint32_t cur = c.tsel;
            c.tsel ^= 1u;
            HIP_CHECK(hipMemsetAsync(c.L.ctr + C_T0 + c.tsel, 0, sizeof(uint32_t), st));
            HIP_CHECK(hipMemsetAsync(c.L.ctr + C_TS0 + c.tsel, 0, sizeof(uint32_t), st));
            hipLaunchKernelGGL(k3_gather, dim3((n2 + 255) / 256), dim3(256), 0, st, c, c.L.t[cur], n2, round, rtext);
            HIP_CHECK(hipGetLastError());
            HIP_CHECK(hipMemsetAsync(c.L.ctr + C_T0 + cur, 0, sizeof(uint32_t), st));
            sort_groups();
            hipLaunchKernelGGL(k3_round_end, dim3((nb + 255) / 256), dim3(256), 0, st, c, nb);
        }
    }
    hipLaunchKernelGGL(k3_finish, dim3((nb + 255) / 256), dim3(256), 0, st, c, nb, stats);
    HIP_CHECK(hipGetLastError());
}

}  // namespace bz
