// starch_amd/csrc/bz2_bwt2.hip -- block sort v2: MSD bucket partition + LDS
// sorts of small groups (the default; bz2_bwt.hip's all-LSD k_bwt remains as
// the reference implementation selectable with STARCH_BWT=lsd).
//
// Same contract as k_bwt (exact cyclic-rotation order for non-periodic
// blocks; periodic blocks flagged for k_fallback_exact), different cost:
//   1. key pass   : each lane rolls the packed D-symbol prefix key over a
//                   contiguous strip (1 text byte per rotation);
//   2. partition  : top 12 key bits -> LDS histogram -> LDS-atomic scatter
//                   (one global pass; order inside a bucket is irrelevant);
//   3. group sort : every bucket is sorted by its full 64-bit key by ONE lane
//                   (<= 16 elements, insertion sort), ONE wave (<= 64, rank
//                   by shuffles; <= WCAP, bitonic in the wave's LDS slice) or
//                   the whole workgroup (larger: stable LSD radix in HBM);
//   4. ranks      : group heads, rank = head position, groups of equal keys;
//   5. doubling   : per round, keys RK[(SA+h) mod n] are gathered for every
//                   unresolved position, then each unresolved group is
//                   re-sorted by the same lane/wave/workgroup ladder and split.
// A round that splits nothing proves the remaining groups are equal rotations
// (periodic block).  No workgroup-wide barrier is needed inside a ladder
// step: lanes/waves own disjoint groups.
#include "bz2_int.hpp"
#include "bz2_bwt.hpp"

namespace bz {

constexpr int B2T = 512;                 // threads per workgroup (8 waves)
constexpr int B2W = B2T / 64;
constexpr int WCAP = 512;                // elements a wave sorts in its LDS slice
constexpr int TCAP = 16;                 // elements a single lane sorts
constexpr int DIG = 12;                  // MSD partition bits
constexpr int NBK = 1 << DIG;
constexpr int LCAP = 1024;               // large-group list capacity (LDS)

struct Bwt2Smem {
    union {
        struct {
            uint32_t cnt[NBK];
            uint32_t cur[NBK];
        } part;
        struct {
            uint64_t key[B2W][WCAP];
            uint32_t val[B2W][WCAP];
        } wave;
        struct {
            uint32_t hist[256];
            uint32_t base[256];
            uint32_t wcnt[B2W][256];
            uint32_t flag;
        } rad;
    } u;
    uint32_t stk[LCAP][3];                // MSD refinement stack: (start, size, remaining bits)
    uint32_t rh[256], rs[256], rc[256];   // refinement histogram, sub-bucket starts, cursors
    uint32_t scan[B2W + 1];
    uint32_t ctr[8];
    uint8_t sym[256];
};

__device__ __forceinline__ void wave_sync_lds()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// --------------------------------------------------------------------------
// group sorts; (K, V) hold the group at [s, s+m), sorted ascending by K
// --------------------------------------------------------------------------
__device__ void wave_rank_sort(uint64_t* K, uint32_t* V, uint32_t s, uint32_t m)   // m <= 64, whole wave
{
    const int lane = threadIdx.x & 63;
    uint64_t k = ~0ull;
    uint32_t v = 0;
    if ((uint32_t)lane < m) { k = K[s + lane]; v = V[s + lane]; }
    uint32_t r = 0;
    for (uint32_t j = 0; j < m; ++j) {
        uint64_t kj = __shfl(k, (int)j, 64);
        r += (kj < k || (kj == k && (int)j < lane)) ? 1u : 0u;
    }
    wave_sync_lds();
    if ((uint32_t)lane < m) { K[s + r] = k; V[s + r] = v; }
}

__device__ void wave_bitonic_sort(uint64_t* K, uint32_t* V, uint32_t s, uint32_t m, uint64_t* lk, uint32_t* lv)
{
    const int lane = threadIdx.x & 63;
    uint32_t P = 64;
    while (P < m) P <<= 1;
    for (uint32_t i = lane; i < P; i += 64) {
        lk[i] = (i < m) ? K[s + i] : ~0ull;
        lv[i] = (i < m) ? V[s + i] : 0xffffffffu;
    }
    wave_sync_lds();
    for (uint32_t k = 2; k <= P; k <<= 1) {
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t i = lane; i < P; i += 64) {
                uint32_t p = i ^ j;
                if (p > i) {
                    uint64_t a = lk[i], b = lk[p];
                    uint32_t va = lv[i], vb = lv[p];
                    bool up = (i & k) == 0;
                    bool gt = (a > b) || (a == b && va > vb);   // pads (val ~0) stay last
                    if (gt == up) {
                        lk[i] = b; lk[p] = a;
                        uint32_t t = lv[i]; lv[i] = lv[p]; lv[p] = t;
                    }
                }
            }
            wave_sync_lds();
        }
    }
    for (uint32_t i = lane; i < m; i += 64) { K[s + i] = lk[i]; V[s + i] = lv[i]; }
}

__device__ void lane_insertion_sort(uint64_t* K, uint32_t* V, uint32_t s, uint32_t m)   // m <= TCAP, one lane
{
    for (uint32_t i = 1; i < m; ++i) {
        uint64_t k = K[s + i];
        uint32_t v = V[s + i];
        uint32_t j = i;
        while (j > 0 && K[s + j - 1] > k) { K[s + j] = K[s + j - 1]; V[s + j] = V[s + j - 1]; --j; }
        K[s + j] = k;
        V[s + j] = v;
    }
}

// stable LSD radix of one large group by the low `bits` bits, whole workgroup;
// result written back to (K, V) at [s, s+m) using (K2, V2) as scratch
__device__ void wg_radix_group(uint64_t* K, uint32_t* V, uint64_t* K2, uint32_t* V2, uint32_t s, uint32_t m, int bits,
                               Bwt2Smem& sm)
{
    const int tid = threadIdx.x, wid = tid >> 6;
    uint64_t* ks = K + s;
    uint32_t* vs = V + s;
    uint64_t* kd = K2 + s;
    uint32_t* vd = V2 + s;
    for (int sh = 0; sh < bits; sh += 8) {
        for (int i = tid; i < 256; i += B2T) sm.u.rad.hist[i] = 0;
        for (int i = tid; i < B2W * 256; i += B2T) (&sm.u.rad.wcnt[0][0])[i] = 0;
        __syncthreads();
        for (uint32_t i = tid; i < m; i += B2T) atomicAdd(&sm.u.rad.hist[(ks[i] >> sh) & 255u], 1u);
        __syncthreads();
        if (tid < 64) {
            uint32_t a0 = sm.u.rad.hist[4 * tid], a1 = sm.u.rad.hist[4 * tid + 1], a2 = sm.u.rad.hist[4 * tid + 2],
                     a3 = sm.u.rad.hist[4 * tid + 3];
            uint32_t sum = a0 + a1 + a2 + a3;
            uint32_t inc = wave_incl_scan_add(sum);
            uint32_t e = inc - sum;
            sm.u.rad.base[4 * tid] = e;
            sm.u.rad.base[4 * tid + 1] = e + a0;
            sm.u.rad.base[4 * tid + 2] = e + a0 + a1;
            sm.u.rad.base[4 * tid + 3] = e + a0 + a1 + a2;
            uint64_t any = __ballot(a0 == m || a1 == m || a2 == m || a3 == m);
            if (tid == 0) sm.u.rad.flag = any ? 1u : 0u;
        }
        __syncthreads();
        if (sm.u.rad.flag) continue;          // one digit value: pass is the identity
        for (uint32_t t0 = 0; t0 < m; t0 += B2T) {
            const uint32_t i = t0 + tid;
            const bool valid = i < m;
            uint64_t k = 0;
            uint32_t v = 0, d = 0;
            if (valid) { k = ks[i]; v = vs[i]; d = (uint32_t)(k >> sh) & 255u; }
            uint64_t mask = __ballot(valid);
#pragma unroll
            for (int bb = 0; bb < 8; ++bb) {
                uint64_t bal = __ballot((d >> bb) & 1u);
                mask &= ((d >> bb) & 1u) ? bal : ~bal;
            }
            const int lane = tid & 63;
            const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
            const uint32_t rank = __popcll(mask & lt);
            if (valid && rank == 0) sm.u.rad.wcnt[wid][d] = __popcll(mask);
            __syncthreads();
            if (tid < 256) {
                uint32_t run = sm.u.rad.base[tid];
                for (int w = 0; w < B2W; ++w) { uint32_t c = sm.u.rad.wcnt[w][tid]; sm.u.rad.wcnt[w][tid] = run; run += c; }
                sm.u.rad.base[tid] = run;
            }
            __syncthreads();
            if (valid) { uint32_t dst = sm.u.rad.wcnt[wid][d] + rank; kd[dst] = k; vd[dst] = v; }
            __syncthreads();
            for (int j = tid; j < B2W * 256; j += B2T) (&sm.u.rad.wcnt[0][0])[j] = 0;
            __syncthreads();
        }
        uint64_t* tk = ks; ks = kd; kd = tk;
        uint32_t* tv = vs; vs = vd; vd = tv;
    }
    if (ks != K + s) {
        for (uint32_t i = tid; i < m; i += B2T) { K[s + i] = ks[i]; V[s + i] = vs[i]; }
    }
    __syncthreads();
}

// Sort one sub-bucket ladder step: lanes for <= TCAP, waves for <= WCAP.
__device__ __forceinline__ void sort_small(uint64_t* K, uint32_t* V, uint32_t s, uint32_t m, Bwt2Smem& sm, int wid)
{
    if (m <= 64) wave_rank_sort(K, V, s, m);
    else wave_bitonic_sort(K, V, s, m, sm.u.wave.key[wid], sm.u.wave.val[wid]);
    wave_sync_lds();
}

__device__ void push_large(Bwt2Smem& sm, uint32_t s, uint32_t m, uint32_t bits)
{
    uint32_t slot = atomicAdd(&sm.ctr[4], 1u);
    if (slot < (uint32_t)LCAP) { sm.stk[slot][0] = s; sm.stk[slot][1] = m; sm.stk[slot][2] = bits; }
    else atomicAdd(&sm.ctr[5], 1u);          // overflow: handled by the LSD fallback
}

// MSD refinement of one large group on its next (up to) 8 key bits, in place
// via (K2, V2); sub-buckets are sorted at once (lanes / waves) or pushed.
__device__ void msd_refine(uint64_t* K, uint32_t* V, uint64_t* K2, uint32_t* V2, uint32_t s, uint32_t m,
                           uint32_t bits, Bwt2Smem& sm)
{
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const uint32_t db = bits < 8 ? bits : 8;
    const uint32_t sh = bits - db;
    const uint64_t dm = (1ull << db) - 1ull;
    if (tid < 256) sm.rh[tid] = 0;
    __syncthreads();
    for (uint32_t i = tid; i < m; i += B2T) atomicAdd(&sm.rh[(uint32_t)((K[s + i] >> sh) & dm)], 1u);
    __syncthreads();
    if (tid < 64) {
        uint32_t a0 = sm.rh[4 * tid], a1 = sm.rh[4 * tid + 1], a2 = sm.rh[4 * tid + 2], a3 = sm.rh[4 * tid + 3];
        uint32_t sum = a0 + a1 + a2 + a3;
        uint32_t e = wave_incl_scan_add(sum) - sum;
        sm.rs[4 * tid] = e; sm.rs[4 * tid + 1] = e + a0; sm.rs[4 * tid + 2] = e + a0 + a1;
        sm.rs[4 * tid + 3] = e + a0 + a1 + a2;
    }
    __syncthreads();
    if (tid < 256) sm.rc[tid] = sm.rs[tid];
    __syncthreads();
    for (uint32_t i = tid; i < m; i += B2T) {
        uint64_t k = K[s + i];
        uint32_t pos = atomicAdd(&sm.rc[(uint32_t)((k >> sh) & dm)], 1u);
        K2[s + pos] = k;
        V2[s + pos] = V[s + i];
    }
    __syncthreads();
    for (uint32_t i = tid; i < m; i += B2T) { K[s + i] = K2[s + i]; V[s + i] = V2[s + i]; }
    __syncthreads();
    // sub-buckets
    if (tid < 256) {
        uint32_t c = sm.rh[tid];
        if (c >= 2 && c <= (uint32_t)TCAP) lane_insertion_sort(K, V, s + sm.rs[tid], c);
        else if (c > (uint32_t)WCAP && sh > 0) push_large(sm, s + sm.rs[tid], c, sh);
    }
    for (int d0 = wid * 64; d0 < 256; d0 += B2W * 64) {
        uint32_t c = sm.rh[d0 + lane];
        uint64_t want = __ballot(c > (uint32_t)TCAP && c <= (uint32_t)WCAP);
        while (want) {
            int l = __ffsll((unsigned long long)want) - 1;
            want &= want - 1;
            sort_small(K, V, s + sm.rs[d0 + l], sm.rh[d0 + l], sm, wid);
        }
    }
    __syncthreads();
}

// Sort every listed group [s, s+m) of (K, V) by its low `bits` key bits:
// lanes take groups of <= TCAP elements, waves groups of <= WCAP, and larger
// groups are refined MSD-first 8 bits at a time by the whole workgroup.
// groups: pairs (start, size) in global memory; returns after a barrier.
__device__ void sort_groups(uint64_t* K, uint32_t* V, uint64_t* K2, uint32_t* V2, const uint32_t* groups, uint32_t ng,
                            int bits, Bwt2Smem& sm)
{
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    for (uint32_t g = tid; g < ng; g += B2T) {
        uint32_t m = groups[2 * g + 1];
        if (m <= (uint32_t)TCAP) lane_insertion_sort(K, V, groups[2 * g], m);
    }
    if (tid == 0) { sm.ctr[4] = 0; sm.ctr[5] = 0; }
    __syncthreads();
    for (uint32_t base = (uint32_t)wid * 64; base < ng; base += B2W * 64) {
        uint32_t g = base + lane;
        uint32_t m = (g < ng) ? groups[2 * g + 1] : 0u;
        uint64_t want = __ballot(m > (uint32_t)TCAP && m <= (uint32_t)WCAP);
        if (m > (uint32_t)WCAP) push_large(sm, groups[2 * g], m, (uint32_t)bits);
        while (want) {
            int l = __ffsll((unsigned long long)want) - 1;
            want &= want - 1;
            sort_small(K, V, groups[2 * (base + l)], groups[2 * (base + l) + 1], sm, wid);
        }
    }
    __syncthreads();
    // depth-first MSD refinement of large groups (LIFO stack in LDS)
    for (;;) {
        __syncthreads();
        uint32_t top = sm.ctr[4] < (uint32_t)LCAP ? sm.ctr[4] : (uint32_t)LCAP;
        if (top == 0) break;
        uint32_t s = sm.stk[top - 1][0], m = sm.stk[top - 1][1], rb = sm.stk[top - 1][2];
        __syncthreads();
        if (tid == 0) sm.ctr[4] = top - 1;
        __syncthreads();
        msd_refine(K, V, K2, V2, s, m, rb, sm);
    }
    if (sm.ctr[5]) {
        // stack overflow (pathological): finish every still-large group with stable LSD
        // radix; sorting an already sorted range is harmless
        __syncthreads();
        for (uint32_t g = 0; g < ng; ++g) {
            uint32_t m = groups[2 * g + 1];
            if (m > (uint32_t)WCAP) wg_radix_group(K, V, K2, V2, groups[2 * g], m, bits, sm);
        }
    }
    __syncthreads();
}

__device__ __forceinline__ int bits_for2(uint32_t x) { return x ? 32 - __clz(x) : 0; }

// Build heads / ranks / the list of unresolved groups from keys K[0..n) sorted
// inside every listed group.  `first` = true: all positions [0,n) (round 0).
// Returns (#groups kept, #groups seen) through sm.ctr[1..2].
__device__ void rank_pass(const uint64_t* K, const uint32_t* V, uint32_t* SA, uint32_t* RK, const uint32_t* groups,
                          uint32_t ng, uint32_t n, uint32_t* out_groups, Bwt2Smem& sm)
{
    // one lane per listed group: split it by key, write SA and RK, list sub-groups
    const int tid = threadIdx.x;
    for (uint32_t g = tid; g < ng; g += B2T) {
        const uint32_t s = groups[2 * g], m = groups[2 * g + 1];
        if (m > 256) continue;                       // big groups: cooperative pass below
        uint32_t head = s;
        uint64_t hk = K[s];
        uint32_t nsub = 0;
        for (uint32_t j = s; j <= s + m; ++j) {
            bool end = (j == s + m);
            uint64_t k = end ? 0 : K[j];
            if (end || k != hk) {
                uint32_t sz = j - head;
                for (uint32_t q = head; q < j; ++q) { uint32_t sa = V[q]; SA[q] = sa; RK[sa] = head; }
                if (sz >= 2) {
                    uint32_t o = atomicAdd(&sm.ctr[1], 1u);
                    out_groups[2 * o] = head;
                    out_groups[2 * o + 1] = sz;
                }
                ++nsub;
                if (!end) { head = j; hk = k; }
            }
        }
        atomicAdd(&sm.ctr[2], nsub);
    }
    __syncthreads();
    // big groups: workgroup scan per group
    for (uint32_t g = 0; g < ng; ++g) {
        const uint32_t s = groups[2 * g], m = groups[2 * g + 1];
        if (m <= 256) continue;
        if (threadIdx.x == 0) sm.ctr[3] = s;   // running head
        __syncthreads();
        for (uint32_t t0 = 0; t0 < m; t0 += B2T) {
            const uint32_t j = s + t0 + tid;
            const bool valid = j < s + m;
            const uint64_t k = valid ? K[j] : 0;
            const bool h = valid && (j == s || K[j - 1] != k);
            const bool last = valid && (j + 1 == s + m || K[j + 1] != k);
            uint32_t hp = block_incl_scan_max<uint32_t>(h ? j : 0u, sm.scan);
            uint32_t cm = sm.ctr[3];
            hp = hp > cm ? hp : cm;
            if (valid) { uint32_t sa = V[j]; SA[j] = sa; RK[sa] = hp; }
            if (last) {
                uint32_t sz = j - hp + 1;
                if (sz >= 2) {
                    uint32_t o = atomicAdd(&sm.ctr[1], 1u);
                    out_groups[2 * o] = hp;
                    out_groups[2 * o + 1] = sz;
                }
                atomicAdd(&sm.ctr[2], 1u);
            }
            __syncthreads();
            if (tid == B2T - 1) sm.ctr[3] = hp;
            __syncthreads();
        }
    }
    __syncthreads();
}

__global__ void __launch_bounds__(B2T) k_bwt2(BlockDesc* __restrict__ blocks, uint32_t b0,
                                               const uint8_t* __restrict__ blkbytes, uint64_t stride, BwtScratch scr,
                                               unsigned long long* __restrict__ stats)
{
    __shared__ Bwt2Smem sm;
    const int tid = threadIdx.x;
    const uint32_t b = b0 + blockIdx.x;
    const uint32_t n = blocks[b].n;
    const uint8_t* blk = blkbytes + (uint64_t)b * stride;
    const uint64_t so = (uint64_t)blockIdx.x * scr.stride;
    uint64_t* K = scr.K + so;       // keys by position (round 0) / gathered ranks (doubling)
    uint64_t* K2 = scr.K2 + so;     // keys in bucket order
    uint32_t* V = scr.V + so;       // radix scratch values
    uint32_t* V2 = scr.V2 + so;     // values (rotation index) in bucket order
    uint32_t* SA = scr.SA + so;
    uint32_t* RK = scr.RK + so;
    uint32_t* G = scr.U + so;       // group list (pairs), capacity n/2 pairs
    uint32_t* G2 = scr.U2 + so;

    if (tid < 256) {
        uint32_t c = tid, below = 0;
        for (uint32_t j = 0; j < (c >> 5); ++j) below += __popc(blocks[b].in_use[j]);
        below += __popc(blocks[b].in_use[c >> 5] & ((1u << (c & 31)) - 1u));
        sm.sym[c] = (uint8_t)below;
    }
    if (tid == 0) {
        uint32_t nu = 0;
        for (int j = 0; j < 8; ++j) nu += __popc(blocks[b].in_use[j]);
        sm.ctr[7] = nu;
    }
    __syncthreads();
    const uint32_t n_in_use = sm.ctr[7];
    const int B = n_in_use > 1 ? bits_for2(n_in_use - 1) : 1;
    const int D = 64 / B;
    const int KB = D * B;
    if (n <= 1) {
        if (tid == 0) { blocks[b].orig_ptr = 0; SA[0] = 0; blocks[b].flags = 0; blocks[b].n_in_use = n_in_use; }
        return;
    }
    // ---- 1. keys: rolling D-symbol window over a contiguous strip per lane ----
    {
        const uint32_t strip = (n + B2T - 1) / B2T;
        const uint32_t a = tid * strip;
        uint32_t e = a + strip;
        if (e > n) e = n;
        if (a < e) {
            const uint64_t mask = (KB == 64) ? ~0ull : ((1ull << KB) - 1ull);
            uint64_t key = 0;
            uint32_t j = a;
            for (int k = 0; k < D; ++k) { key = (key << B) | sm.sym[blk[j]]; if (++j == n) j = 0; }
            for (uint32_t i = a; i < e; ++i) {
                K[i] = key;
                key = ((key << B) | sm.sym[blk[j]]) & mask;
                if (++j == n) j = 0;
            }
        }
    }
    // ---- 2. MSD partition on the top DIG bits ----
    const int dig = KB < DIG ? KB : DIG;
    const int dsh = KB - dig;
    for (int i = tid; i < NBK; i += B2T) sm.u.part.cnt[i] = 0;
    __syncthreads();
    for (uint32_t i = tid; i < n; i += B2T) atomicAdd(&sm.u.part.cnt[(uint32_t)(K[i] >> dsh)], 1u);
    __syncthreads();
    {
        // exclusive scan of NBK counts (8 per thread)
        uint32_t loc[NBK / B2T];
        uint32_t s = 0;
#pragma unroll
        for (int q = 0; q < NBK / B2T; ++q) { loc[q] = sm.u.part.cnt[tid * (NBK / B2T) + q]; s += loc[q]; }
        uint32_t pre = block_excl_scan_add<uint32_t>(s, sm.scan, (uint32_t*)nullptr);
#pragma unroll
        for (int q = 0; q < NBK / B2T; ++q) { sm.u.part.cur[tid * (NBK / B2T) + q] = pre; pre += loc[q]; }
    }
    __syncthreads();
    // bucket list (start, size) of buckets with >= 2 entries -> G; singletons need no sort
    if (tid == 0) sm.ctr[0] = 0;
    __syncthreads();
    for (int d = tid; d < NBK; d += B2T) {
        uint32_t c = sm.u.part.cnt[d];
        if (c >= 2) {
            uint32_t o = atomicAdd(&sm.ctr[0], 1u);
            G[2 * o] = sm.u.part.cur[d];
            G[2 * o + 1] = c;
        }
    }
    __syncthreads();
    for (uint32_t i = tid; i < n; i += B2T) {
        const uint64_t k = K[i];
        const uint32_t pos = atomicAdd(&sm.u.part.cur[(uint32_t)(k >> dsh)], 1u);
        K2[pos] = k;
        V2[pos] = i;
    }
    __syncthreads();
    const uint32_t nbuckets = sm.ctr[0];
    // ---- 3. sort buckets by full key ----
    sort_groups(K2, V2, K, V, G, nbuckets, KB, sm);
    // ---- 4. ranks + unresolved groups (all positions: singleton buckets too) ----
    // singletons and sorted buckets: a position-parallel pass covers everything
    if (tid == 0) { sm.ctr[1] = 0; sm.ctr[2] = 0; sm.ctr[3] = 0; }
    __syncthreads();
    for (uint32_t t0 = 0; t0 < n; t0 += B2T) {
        const uint32_t j = t0 + tid;
        const bool valid = j < n;
        const uint64_t k = valid ? K2[j] : 0;
        const bool h = valid && (j == 0 || K2[j - 1] != k);
        const bool last = valid && (j + 1 == n || K2[j + 1] != k);
        uint32_t hp = block_incl_scan_max<uint32_t>(h ? j : 0u, sm.scan);
        uint32_t cm = sm.ctr[3];
        hp = hp > cm ? hp : cm;
        if (valid) { uint32_t sa = V2[j]; SA[j] = sa; RK[sa] = hp; }
        if (last && j - hp + 1 >= 2) {
            uint32_t o = atomicAdd(&sm.ctr[1], 1u);
            G2[2 * o] = hp;
            G2[2 * o + 1] = j - hp + 1;
        }
        __syncthreads();
        if (tid == B2T - 1) sm.ctr[3] = hp;
        __syncthreads();
    }
    uint32_t ng = sm.ctr[1];
    __syncthreads();
    // ---- 5. doubling on unresolved groups ----
    const int rbits = bits_for2(n - 1);
    uint64_t h = (uint64_t)D;
    uint32_t rounds = 0;
    bool periodic = false;
    uint32_t* Gc = G2;   // current groups
    uint32_t* Gn = G;    // next groups
    while (ng > 0) {
        ++rounds;
        // gather keys for every unresolved position: lanes over groups' elements
        for (uint32_t g = tid; g < ng; g += B2T) {
            const uint32_t s = Gc[2 * g], m = Gc[2 * g + 1];
            if (m > 64) continue;
            for (uint32_t j = s; j < s + m; ++j) {
                uint32_t sa = SA[j];
                K2[j] = RK[(uint32_t)(((uint64_t)sa + h) % n)];
                V2[j] = sa;
            }
        }
        {
            const int lane = tid & 63, wid = tid >> 6;
            for (uint32_t g = wid; g < ng; g += B2W) {
                const uint32_t s = Gc[2 * g], m = Gc[2 * g + 1];
                if (m <= 64) continue;
                for (uint32_t j = s + lane; j < s + m; j += 64) {
                    uint32_t sa = SA[j];
                    K2[j] = RK[(uint32_t)(((uint64_t)sa + h) % n)];
                    V2[j] = sa;
                }
            }
        }
        __syncthreads();
        sort_groups(K2, V2, K, V, Gc, ng, rbits, sm);
        if (tid == 0) { sm.ctr[1] = 0; sm.ctr[2] = 0; }
        __syncthreads();
        rank_pass(K2, V2, SA, RK, Gc, ng, n, Gn, sm);
        const uint32_t kept = sm.ctr[1], seen = sm.ctr[2];
        __syncthreads();
        if (seen == ng) { periodic = true; break; }     // no group split: equal rotations
        uint32_t* t = Gc; Gc = Gn; Gn = t;
        ng = kept;
        h *= 2;
        if (h >= 2ull * n + (uint64_t)D) { periodic = ng > 0; break; }
    }
    __syncthreads();
    for (uint32_t j = tid; j < n; j += B2T)
        if (SA[j] == 0) blocks[b].orig_ptr = j;
    if (tid == 0) {
        blocks[b].flags = periodic ? 1u : 0u;
        blocks[b].n_in_use = n_in_use;
        atomicAdd(stats, (unsigned long long)rounds);
        if (periodic) atomicAdd(stats + 1, 1ull);
    }
}

void launch_bwt2(BlockDesc* blocks, uint32_t b0, uint32_t nb, const uint8_t* blkbytes, uint64_t stride,
                 const BwtScratch& scr, unsigned long long* stats, hipStream_t st)
{
    hipLaunchKernelGGL(k_bwt2, dim3(nb), dim3(B2T), 0, st, blocks, b0, blkbytes, stride, scr, stats);
    HIP_CHECK(hipGetLastError());
}

}  // namespace bz
