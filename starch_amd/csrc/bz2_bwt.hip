// starch_amd/csrc/bz2_bwt.hip -- Burrows-Wheeler block sort on MI355X.
//
// Replaces BZ2_blockSort (bz:blocksort.c:1031-1089).  For a non-periodic
// block every rotation is distinct, so the sorted order -- and hence origPtr
// and the last column -- is unique: any exact cyclic-rotation sort reproduces
// bzip2's bytes.  We sort with prefix doubling, one 1024-thread
// workgroup per block, all state in HBM:
//   round 0: key = first D symbols of the rotation, packed with
//            B = ceil(log2(nInUse)) bits each (D = 64/B: 16 symbols for the
//            <=16-symbol alphabets of BED3 transforms), stable LSD radix sort
//            (8-bit digits, histogram + wave-ballot ranking in LDS);
//   round r: only rotations in unresolved groups are re-sorted by
//            (group head, rank of rotation + h), h = D*2^(r-1).
// A round that splits no group proves the remaining groups are true ties, i.e.
// the block is periodic.  For those blocks bzip2's origPtr is
// fallbackSort's tie order, so k_fallback_exact re-runs a restatement of
// fallbackSort (bz:blocksort.c:30-329) for that block only, with the
// all-equal-key buckets (whose 3-way partition is the identity) skipped.
#include <string.h>
#include "bz2_int.hpp"
#include "bz2_bwt.hpp"

namespace bz {

constexpr int BT = 1024;          // threads per block-sort workgroup
constexpr int NWV = BT / 64;      // waves

struct RadixSmem {
    uint32_t hist[256];
    uint32_t base[256];
    uint32_t wcnt[NWV][256];
    uint32_t scan[NWV + 1];
    uint32_t flag;
};

__device__ __forceinline__ uint64_t lanemask_lt()
{
    const int lane = threadIdx.x & 63;
    return lane ? (~0ull >> (64 - lane)) : 0ull;
}

// One stable LSD pass by digit (key >> shift) & 255 over [0, m).
// Returns false (and writes nothing) when every key has the same digit.
template <class V>
__device__ bool radix_pass(const uint64_t* Ks, const V* Vs, uint64_t* Kd, V* Vd, uint32_t m, int shift,
                           RadixSmem& sm)
{
    const int tid = threadIdx.x, wid = tid >> 6;
    for (int i = tid; i < 256; i += BT) sm.hist[i] = 0;
    for (int i = tid; i < NWV * 256; i += BT) (&sm.wcnt[0][0])[i] = 0;
    __syncthreads();
    for (uint32_t i = tid; i < m; i += BT) atomicAdd(&sm.hist[(Ks[i] >> shift) & 255u], 1u);
    __syncthreads();
    if (tid < 64) {   // exclusive scan of 256 bins, 4 per lane
        uint32_t a0 = sm.hist[4 * tid], a1 = sm.hist[4 * tid + 1], a2 = sm.hist[4 * tid + 2],
                 a3 = sm.hist[4 * tid + 3];
        uint32_t s = a0 + a1 + a2 + a3;
        uint32_t inc = wave_incl_scan_add(s);
        uint32_t e = inc - s;
        sm.base[4 * tid] = e;
        sm.base[4 * tid + 1] = e + a0;
        sm.base[4 * tid + 2] = e + a0 + a1;
        sm.base[4 * tid + 3] = e + a0 + a1 + a2;
        bool single = (a0 == m) || (a1 == m) || (a2 == m) || (a3 == m);
        uint64_t any = __ballot(single);
        if (tid == 0) sm.flag = any ? 1u : 0u;
    }
    __syncthreads();
    if (sm.flag) return false;
    for (uint32_t t0 = 0; t0 < m; t0 += BT) {
        const uint32_t i = t0 + tid;
        const bool valid = i < m;
        uint64_t k = 0;
        V v = V(0);
        uint32_t d = 0;
        if (valid) { k = Ks[i]; v = Vs[i]; d = (uint32_t)(k >> shift) & 255u; }
        uint64_t mask = __ballot(valid);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            uint64_t bal = __ballot((d >> b) & 1u);
            mask &= ((d >> b) & 1u) ? bal : ~bal;
        }
        const uint32_t rank = __popcll(mask & lanemask_lt());
        if (valid && rank == 0) sm.wcnt[wid][d] = __popcll(mask);
        __syncthreads();
        if (tid < 256) {
            uint32_t run = sm.base[tid];
#pragma unroll
            for (int w = 0; w < NWV; ++w) { uint32_t c = sm.wcnt[w][tid]; sm.wcnt[w][tid] = run; run += c; }
            sm.base[tid] = run;
        }
        __syncthreads();
        if (valid) {
            uint32_t dst = sm.wcnt[wid][d] + rank;
            Kd[dst] = k;
            Vd[dst] = v;
        }
        __syncthreads();
        for (int j = tid; j < NWV * 256; j += BT) (&sm.wcnt[0][0])[j] = 0;
        __syncthreads();
    }
    return true;
}

// Sort (K,V)[0,m) by the low `bits` bits; result may end in either buffer.
template <class V>
__device__ void radix_sort(uint64_t*& K, V*& Vv, uint64_t*& K2, V*& V2, uint32_t m, int bits, RadixSmem& sm)
{
    for (int sh = 0; sh < bits; sh += 8) {
        if (radix_pass<V>(K, Vv, K2, V2, m, sh, sm)) {
            uint64_t* tk = K; K = K2; K2 = tk;
            V* tv = Vv; Vv = V2; V2 = tv;
        }
    }
}

__device__ __forceinline__ int bits_for(uint32_t x) { return x ? 32 - __clz(x) : 0; }

__global__ void __launch_bounds__(BT) k_bwt(BlockDesc* __restrict__ blocks, uint32_t b0,
                                             const uint8_t* __restrict__ blkbytes, uint64_t stride,
                                             BwtScratch scr, unsigned long long* __restrict__ stats)
{
    __shared__ RadixSmem sm;
    __shared__ uint8_t sym[256];
    __shared__ uint32_t carry[4];
    const int tid = threadIdx.x;
    const uint32_t b = b0 + blockIdx.x;
    const uint32_t n = blocks[b].n;
    const uint8_t* blk = blkbytes + (uint64_t)b * stride;
    const uint64_t so = (uint64_t)blockIdx.x * scr.stride;
    uint64_t* K = scr.K + so;
    uint64_t* K2 = scr.K2 + so;
    uint32_t* Vv = scr.V + so;
    uint32_t* V2 = scr.V2 + so;
    uint32_t* SA = scr.SA + so;
    uint32_t* RK = scr.RK + so;
    uint32_t* U = scr.U + so;
    uint32_t* U2 = scr.U2 + so;

    // alphabet -> dense order-preserving symbols
    if (tid < 256) {
        uint32_t c = tid;
        uint32_t w = blocks[b].in_use[c >> 5];
        uint32_t below = 0;
        for (uint32_t j = 0; j < (c >> 5); ++j) below += __popc(blocks[b].in_use[j]);
        below += __popc(w & ((1u << (c & 31)) - 1u));
        sym[c] = (uint8_t)below;
    }
    if (tid == 0) {
        uint32_t nu = 0;
        for (int j = 0; j < 8; ++j) nu += __popc(blocks[b].in_use[j]);
        carry[0] = nu;
    }
    __syncthreads();
    const uint32_t n_in_use = carry[0];
    const int B = n_in_use > 1 ? bits_for(n_in_use - 1) : 1;
    const int D = 64 / B;
    __syncthreads();

    if (n <= 1) {
        if (tid == 0) { blocks[b].orig_ptr = 0; SA[0] = 0; blocks[b].flags = 0; blocks[b].n_in_use = n_in_use; }
        return;
    }
    // ---- round 0: sort by D-symbol packed prefix ----
    for (uint32_t i = tid; i < n; i += BT) {
        uint64_t key = 0;
        uint32_t j = i;
        for (int k = 0; k < D; ++k) {
            key = (key << B) | sym[blk[j]];
            if (++j == n) j = 0;
        }
        K[i] = key;
        Vv[i] = i;
    }
    __syncthreads();
    radix_sort<uint32_t>(K, Vv, K2, V2, n, D * B, sm);
    // heads, ranks, unresolved list
    if (tid == 0) { carry[0] = 0; carry[1] = 0; carry[2] = 0; }
    __syncthreads();
    for (uint32_t t0 = 0; t0 < n; t0 += BT) {
        const uint32_t j = t0 + tid;
        const bool valid = j < n;
        uint64_t kj = valid ? K[j] : 0;
        bool head = valid && (j == 0 || K[j - 1] != kj);
        bool nexth = !valid || (j + 1 >= n) || K[j + 1] != kj;
        uint32_t hp = block_incl_scan_max<uint32_t>(head ? j : 0u, sm.scan);
        uint32_t cm = carry[0];
        hp = hp > cm ? hp : cm;
        uint32_t sa = valid ? Vv[j] : 0;
        if (valid) { SA[j] = sa; RK[sa] = hp; }
        bool unres = valid && !(head && nexth);
        uint32_t tot, gtot;
        uint32_t pre = block_excl_scan_add<uint32_t>(unres ? 1u : 0u, sm.scan, &tot);
        if (unres) U[carry[1] + pre] = j;
        (void)block_excl_scan_add<uint32_t>((unres && head) ? 1u : 0u, sm.scan, &gtot);
        if (tid == BT - 1) { carry[0] = hp; carry[1] += tot; carry[2] += gtot; }
        __syncthreads();
    }
    uint32_t m = carry[1];
    uint32_t groups = carry[2];
    const int rbits = bits_for(n - 1);
    uint64_t h = (uint64_t)D;
    uint32_t rounds = 0;
    bool periodic = false;
    while (m > 0) {
        ++rounds;
        for (uint32_t k = tid; k < m; k += BT) {
            uint32_t j = U[k];
            uint32_t sa = SA[j];
            uint32_t nx = (uint32_t)(((uint64_t)sa + h) % n);
            K[k] = ((uint64_t)RK[sa] << rbits) | RK[nx];
            Vv[k] = sa;
        }
        __syncthreads();
        radix_sort<uint32_t>(K, Vv, K2, V2, m, 2 * rbits, sm);
        if (tid == 0) { carry[0] = 0; carry[1] = 0; carry[2] = 0; }
        __syncthreads();
        for (uint32_t t0 = 0; t0 < m; t0 += BT) {
            const uint32_t k = t0 + tid;
            const bool valid = k < m;
            uint64_t key = valid ? K[k] : 0;
            bool nh = valid && (k == 0 || K[k - 1] != key);
            bool nexth = !valid || (k + 1 >= m) || K[k + 1] != key;
            uint32_t j = valid ? U[k] : 0;
            uint32_t hp = block_incl_scan_max<uint32_t>(nh ? j : 0u, sm.scan);
            uint32_t cm = carry[0];
            hp = hp > cm ? hp : cm;
            if (valid) {
                uint32_t sa = Vv[k];
                SA[j] = sa;
                RK[sa] = hp;
            }
            bool keep = valid && !(nh && nexth);
            uint32_t tot, gtot;
            uint32_t pre = block_excl_scan_add<uint32_t>(keep ? 1u : 0u, sm.scan, &tot);
            if (keep) U2[carry[1] + pre] = j;
            (void)block_excl_scan_add<uint32_t>(nh ? 1u : 0u, sm.scan, &gtot);
            if (tid == BT - 1) { carry[0] = hp; carry[1] += tot; carry[2] += gtot; }
            __syncthreads();
        }
        uint32_t new_groups = carry[2];
        uint32_t nm = carry[1];
        __syncthreads();
        if (new_groups == groups) { periodic = true; break; }   // nothing split: true ties
        // groups still unresolved for the next round
        groups = 0;
        {
            uint32_t* t = U; U = U2; U2 = t;
        }
        m = nm;
        // count heads among the remaining unresolved positions
        if (tid == 0) carry[3] = 0;
        __syncthreads();
        uint32_t local = 0;
        for (uint32_t k = tid; k < m; k += BT) {
            uint32_t j = U[k];
            uint32_t r = RK[SA[j]];
            local += (r == j) ? 1u : 0u;
        }
        local = wave_reduce_add(local);
        if ((tid & 63) == 0) atomicAdd(&carry[3], local);
        __syncthreads();
        groups = carry[3];
        __syncthreads();
        h *= 2;
        if (h >= 2ull * n + (uint64_t)D) { periodic = (m > 0); break; }
    }
    __syncthreads();
    for (uint32_t j = tid; j < n; j += BT)
        if (SA[j] == 0) blocks[b].orig_ptr = j;
    if (tid == 0) {
        blocks[b].flags = periodic ? 1u : 0u;
        blocks[b].n_in_use = n_in_use;
        atomicAdd(stats, (unsigned long long)rounds);
        if (periodic) atomicAdd(stats + 1, 1ull);
    }
}

// ---------------------------------------------------------------------------
// Exact fallbackSort restatement for periodic blocks (bz:blocksort.c:30-329).
// ---------------------------------------------------------------------------
__device__ void fb_simple(uint32_t* fmap, const uint32_t* ecls, int32_t lo, int32_t hi)
{
    if (lo == hi) return;
    if (hi - lo > 3) {
        for (int32_t a = hi - 4; a >= lo; --a) {
            uint32_t x = fmap[a], kx = ecls[x];
            int32_t q = a + 4;
            while (q <= hi && kx > ecls[fmap[q]]) { fmap[q - 4] = fmap[q]; q += 4; }
            fmap[q - 4] = x;
        }
    }
    for (int32_t a = hi - 1; a >= lo; --a) {
        uint32_t x = fmap[a], kx = ecls[x];
        int32_t q = a + 1;
        while (q <= hi && kx > ecls[fmap[q]]) { fmap[q - 1] = fmap[q]; ++q; }
        fmap[q - 1] = x;
    }
}

__device__ void fb_qsort3(uint32_t* fmap, const uint32_t* ecls, int32_t lo0, int32_t hi0)
{
    int32_t slo[100], shi[100];
    int32_t sp = 0;
    uint32_t r = 0;
    slo[sp] = lo0; shi[sp] = hi0; ++sp;
    while (sp > 0) {
        --sp;
        int32_t lo = slo[sp], hi = shi[sp];
        if (hi - lo < 10) { fb_simple(fmap, ecls, lo, hi); continue; }
        r = (r * 7621u + 1u) % 32768u;
        uint32_t pv;
        uint32_t r3 = r % 3u;
        if (r3 == 0) pv = ecls[fmap[lo]]; else if (r3 == 1) pv = ecls[fmap[(lo + hi) >> 1]]; else pv = ecls[fmap[hi]];
        int32_t ulo = lo, lt = lo, uhi = hi, gt = hi;
        for (;;) {
            while (ulo <= uhi) {
                int64_t dd = (int64_t)ecls[fmap[ulo]] - (int64_t)pv;
                if (dd == 0) { uint32_t t = fmap[ulo]; fmap[ulo] = fmap[lt]; fmap[lt] = t; ++lt; ++ulo; continue; }
                if (dd > 0) break;
                ++ulo;
            }
            while (ulo <= uhi) {
                int64_t dd = (int64_t)ecls[fmap[uhi]] - (int64_t)pv;
                if (dd == 0) { uint32_t t = fmap[uhi]; fmap[uhi] = fmap[gt]; fmap[gt] = t; --gt; --uhi; continue; }
                if (dd < 0) break;
                --uhi;
            }
            if (ulo > uhi) break;
            uint32_t t = fmap[ulo]; fmap[ulo] = fmap[uhi]; fmap[uhi] = t;
            ++ulo; --uhi;
        }
        if (gt < lt) continue;
        int32_t k = (lt - lo < ulo - lt) ? lt - lo : ulo - lt;
        for (int32_t a = lo, bb = ulo - k; k > 0; --k, ++a, ++bb) { uint32_t t = fmap[a]; fmap[a] = fmap[bb]; fmap[bb] = t; }
        int32_t mm = (hi - gt < gt - uhi) ? hi - gt : gt - uhi;
        for (int32_t a = ulo, bb = hi - mm + 1; mm > 0; --mm, ++a, ++bb) { uint32_t t = fmap[a]; fmap[a] = fmap[bb]; fmap[bb] = t; }
        int32_t ahi = lo + ulo - lt - 1;
        int32_t blo = hi - (gt - uhi) + 1;
        if (ahi - lo > hi - blo) {
            slo[sp] = lo; shi[sp] = ahi; ++sp;
            slo[sp] = blo; shi[sp] = hi; ++sp;
        } else {
            slo[sp] = blo; shi[sp] = hi; ++sp;
            slo[sp] = lo; shi[sp] = ahi; ++sp;
        }
    }
}

// ---------------------------------------------------------------------------
// fallbackSort for periodic blocks, round by round on the whole GPU.
//
// The reference's tie order is the output here, so every step is the exact
// bz:blocksort.c:211-329 procedure; only the work placement is new:
//   * per doubling round H, grid-wide kernels: eclass from the bucket heads
//     (a max-scan of head positions), then key[i] = eclass[fmap[i]] next to
//     fmap (eclass does not change while a round's buckets are sorted, so the
//     sort moves (key, fmap) pairs and never gathers), mixed-bucket detection
//     and the count of not-done elements (nNotDone), then new heads;
//   * fallbackQSort3 (bz:blocksort.c:93-180) on each MIXED bucket -- an
//     all-equal bucket is left exactly as it is by it -- one wave per bucket,
//     buckets in parallel (r restarts at 0 per call, bz:blocksort.c:104): a
//     bucket of <= FB_CAP elements is staged in the wave's LDS and sorted
//     there by lane 0 (the whole call, stack and LCG included); a larger one
//     is partitioned by lane 0 in HBM until the range it pops fits, then that
//     range's whole subtree is sorted in LDS, so the order of partition steps
//     -- and with it the LCG sequence -- is the serial one.
// fmap lives in SA, eclass in RK, key in V, head flags in U, mixed stamps in
// U2, the head-position scan in K, the mixed-bucket list in K2, counters in V2.
// ---------------------------------------------------------------------------
constexpr int FB_WAVES = 4;
constexpr uint32_t FB_CAP = 4096;          // pairs per wave in LDS (32 KB)

// fallbackSimpleSort (bz:blocksort.c:30-59) on (key, fmap) pairs
__device__ __forceinline__ void fbp_simple(uint32_t* key, uint32_t* fm, int32_t lo, int32_t hi)
{
    if (lo == hi) return;
    if (hi - lo > 3) {
        for (int32_t a = hi - 4; a >= lo; --a) {
            const uint32_t x = fm[a], kx = key[a];
            int32_t q = a + 4;
            while (q <= hi && kx > key[q]) { fm[q - 4] = fm[q]; key[q - 4] = key[q]; q += 4; }
            fm[q - 4] = x;
            key[q - 4] = kx;
        }
    }
    for (int32_t a = hi - 1; a >= lo; --a) {
        const uint32_t x = fm[a], kx = key[a];
        int32_t q = a + 1;
        while (q <= hi && kx > key[q]) { fm[q - 1] = fm[q]; key[q - 1] = key[q]; ++q; }
        fm[q - 1] = x;
        key[q - 1] = kx;
    }
}

__device__ __forceinline__ void fbp_swap(uint32_t* key, uint32_t* fm, int32_t a, int32_t b)
{
    const uint32_t t = fm[a], k = key[a];
    fm[a] = fm[b];
    key[a] = key[b];
    fm[b] = t;
    key[b] = k;
}

// one partition step of fallbackQSort3 on [lo, hi] (hi - lo >= 10): the LCG
// advance, the pivot, the 3-way partition and the two vswaps; returns the
// two sub-ranges [lo, *n] and [*m, hi] (n < lo / m > hi: empty) in the order
// they are pushed (a first), or false when every key equals the pivot
__device__ __forceinline__ bool fbp_partition(uint32_t* key, uint32_t* fm, int32_t lo, int32_t hi, uint32_t& r, int32_t& alo,
                              int32_t& ahi, int32_t& blo, int32_t& bhi)
{
    r = (r * 7621u + 1u) % 32768u;                              // bz:blocksort.c:126-130
    const uint32_t r3 = r % 3u;
    const uint32_t med = r3 == 0 ? key[lo] : r3 == 1 ? key[(lo + hi) >> 1] : key[hi];
    int32_t unLo = lo, ltLo = lo, unHi = hi, gtHi = hi;
    for (;;) {
        while (unLo <= unHi) {
            const uint32_t k = key[unLo];
            if (k == med) { fbp_swap(key, fm, unLo, ltLo); ++ltLo; ++unLo; continue; }
            if (k > med) break;
            ++unLo;
        }
        while (unLo <= unHi) {
            const uint32_t k = key[unHi];
            if (k == med) { fbp_swap(key, fm, unHi, gtHi); --gtHi; --unHi; continue; }
            if (k < med) break;
            --unHi;
        }
        if (unLo > unHi) break;
        fbp_swap(key, fm, unLo, unHi);
        ++unLo;
        --unHi;
    }
    if (gtHi < ltLo) return false;
    int32_t n = ltLo - lo < unLo - ltLo ? ltLo - lo : unLo - ltLo;
    for (int32_t a = lo, b = unLo - n; n > 0; --n, ++a, ++b) fbp_swap(key, fm, a, b);
    int32_t m = hi - gtHi < gtHi - unHi ? hi - gtHi : gtHi - unHi;
    for (int32_t a = unLo, b = hi - m + 1; m > 0; --m, ++a, ++b) fbp_swap(key, fm, a, b);
    const int32_t nn = lo + unLo - ltLo - 1, mm = hi - (gtHi - unHi) + 1;
    if (nn - lo > hi - mm) { alo = lo; ahi = nn; blo = mm; bhi = hi; }   // larger pushed first
    else { alo = mm; ahi = hi; blo = lo; bhi = nn; }
    return true;
}

// the whole fallbackQSort3 call on [lo0, hi0] (any memory), continuing LCG r
__device__ __forceinline__ void fbp_qsort3(uint32_t* key, uint32_t* fm, int32_t lo0, int32_t hi0, uint32_t& r)
{
    int32_t slo[100], shi[100];                                  // FALLBACK_QSORT_STACK_SIZE
    int32_t sp = 0;
    slo[sp] = lo0; shi[sp] = hi0; ++sp;
    while (sp > 0) {
        --sp;
        const int32_t lo = slo[sp], hi = shi[sp];
        if (hi - lo < 10) { fbp_simple(key, fm, lo, hi); continue; }   // FALLBACK_QSORT_SMALL_THRESH
        int32_t alo, ahi, blo, bhi;
        if (!fbp_partition(key, fm, lo, hi, r, alo, ahi, blo, bhi)) continue;
        slo[sp] = alo; shi[sp] = ahi; ++sp;
        slo[sp] = blo; shi[sp] = bhi; ++sp;
    }
}

// 1-byte bucket sort of the block (bz:blocksort.c:240-249: indices descending
// inside a bucket) and the first heads; one workgroup
__global__ void __launch_bounds__(BT) k_fb_init(const uint8_t* __restrict__ blk, uint32_t n, BwtScratch scr,
                                                 uint64_t so)
{
    __shared__ RadixSmem sm;
    const int tid = threadIdx.x;
    uint64_t* K = scr.K + so;
    uint64_t* K2 = scr.K2 + so;
    uint32_t* V = scr.V + so;
    uint32_t* V2 = scr.V2 + so;
    uint32_t* fmap = scr.SA + so;
    uint32_t* head = scr.U + so;
    for (uint32_t i = tid; i < n; i += BT) { K[i] = blk[i]; V[i] = i; }
    __syncthreads();
    uint64_t* Kp = K; uint64_t* K2p = K2; uint32_t* Vp = V; uint32_t* V2p = V2;
    radix_sort<uint32_t>(Kp, Vp, K2p, V2p, n, 8, sm);          // stable ascending
    for (int i = tid; i < 256; i += BT) sm.hist[i] = 0;
    __syncthreads();
    for (uint32_t i = tid; i < n; i += BT) atomicAdd(&sm.hist[blk[i]], 1u);
    __syncthreads();
    if (tid == 0) { uint32_t a = 0; for (int c = 0; c < 256; ++c) { sm.base[c] = a; a += sm.hist[c]; } }
    __syncthreads();
    for (uint32_t j = tid; j < n; j += BT) {
        const uint32_t c = (uint32_t)Kp[j];
        const uint32_t bs = sm.base[c], be = bs + sm.hist[c];
        fmap[bs + be - 1 - j] = Vp[j];
        head[j] = 0;
    }
    __syncthreads();
    for (int c = tid; c < 256; c += BT) if (sm.hist[c]) head[sm.base[c]] = 1;
}

// The same 1-byte bucket sort over the whole GPU (the one-workgroup radix
// sort above took most of a period-2 block's time): per-tile byte counts, one
// scan, then per tile one wave places its bytes in order -- a byte's rank
// among its equals from the tile's offset, the 8-ballot peer set of its
// 64-byte step and the step's running counters -- at bucket end - 1 - rank
// (indices descending inside a bucket, bz:blocksort.c:240-249).
constexpr uint32_t FB_TILE = 4096;

__global__ void __launch_bounds__(256) k_fb_cnt(const uint8_t* __restrict__ blk, uint32_t n, uint32_t* __restrict__ cnt)
{
    __shared__ uint32_t h[256];
    h[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t a = blockIdx.x * FB_TILE, e = a + FB_TILE < n ? a + FB_TILE : n;
    for (uint32_t i = a + threadIdx.x; i < e; i += 256) atomicAdd(&h[blk[i]], 1u);
    __syncthreads();
    cnt[(uint64_t)blockIdx.x * 256 + threadIdx.x] = h[threadIdx.x];
}

// one workgroup of 256: bucket starts and totals, per-tile offsets in place
__global__ void __launch_bounds__(256) k_fb_cscan(uint32_t* __restrict__ cnt, uint32_t ntile, uint32_t* __restrict__ bstart,
                                                   uint32_t* __restrict__ btot, uint32_t* __restrict__ head, uint32_t n)
{
    __shared__ uint32_t sh[256 / 64 + 1];
    const uint32_t c = threadIdx.x;
    uint32_t t = 0;
    for (uint32_t k = 0; k < ntile; ++k) {
        uint32_t& x = cnt[(uint64_t)k * 256 + c];
        const uint32_t v = x;
        x = t;
        t += v;
    }
    uint32_t tot = 0;
    const uint32_t st = block_excl_scan_add<uint32_t>(t, sh, &tot);
    bstart[c] = st;
    btot[c] = t;
    if (t && st < n) head[st] = 1;
}

__global__ void __launch_bounds__(64) k_fb_place(const uint8_t* __restrict__ blk, uint32_t n,
                                                  const uint32_t* __restrict__ cnt, const uint32_t* __restrict__ bstart,
                                                  const uint32_t* __restrict__ btot, uint32_t* __restrict__ fmap)
{
    __shared__ uint32_t run[256];
    const int lane = threadIdx.x;
    for (int c = lane; c < 256; c += 64) run[c] = cnt[(uint64_t)blockIdx.x * 256 + c];
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
    const uint64_t lt = lanemask_lt();
    const uint32_t a = blockIdx.x * FB_TILE, e = a + FB_TILE < n ? a + FB_TILE : n;
    for (uint32_t i0 = a; i0 < e; i0 += 64) {
        const uint32_t i = i0 + lane;
        const bool ok = i < e;
        const uint32_t c = ok ? blk[i] : 0u;
        uint64_t peers = __ballot(ok);
#pragma unroll
        for (int bb = 0; bb < 8; ++bb) {
            const uint64_t bal = __ballot((c >> bb) & 1u);
            peers &= ((c >> bb) & 1u) ? bal : ~bal;
        }
        const uint32_t below = (uint32_t)__popcll(peers & lt);
        const uint32_t base = ok ? run[c] : 0u;     // all peers read the same counter
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
        if (ok && below == 0) run[c] = base + (uint32_t)__popcll(peers);   // the first peer advances it
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
        if (ok) {
            const uint32_t r = base + below;             // rank among the bucket's bytes, ascending index
            fmap[bstart[c] + btot[c] - 1u - r] = i;
        }
    }
}

// (and the round's counters zeroed: no separate memset launch per round)
__global__ void k_fb_hp(const uint32_t* __restrict__ head, uint64_t* __restrict__ hp, uint32_t n,
                        uint32_t* __restrict__ ctr)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < 4) ctr[i] = 0;
    if (i < n) hp[i] = head[i] ? i : 0u;
}

// eclass[fmap[i] - H mod n] = bucket start of i (bz:blocksort.c:258-263)
__global__ void k_fb_eclass(const uint32_t* __restrict__ fmap, const uint64_t* __restrict__ hp,
                            uint32_t* __restrict__ ecls, uint32_t n, uint32_t hmod)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t k = fmap[i] + (n - hmod);
    if (k >= n) k -= n;
    ecls[k] = (uint32_t)hp[i];
}

// key[i] = eclass[fmap[i]]; mixed buckets stamped; not-done elements counted
__global__ void __launch_bounds__(256) k_fb_key(const uint32_t* __restrict__ fmap, const uint32_t* __restrict__ ecls,
                                                const uint32_t* __restrict__ head, const uint64_t* __restrict__ hp,
                                                uint32_t* __restrict__ key, uint32_t* __restrict__ mixed,
                                                uint32_t* __restrict__ ctr, uint32_t n, uint32_t stamp)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t nd = 0;
    if (i < n) {
        const uint32_t k = ecls[fmap[i]];
        key[i] = k;
        const uint32_t l = (uint32_t)hp[i];
        if (!head[i] && k != ecls[fmap[l]]) mixed[l] = stamp;
        nd = (head[i] && (i + 1 == n || head[i + 1])) ? 0u : 1u;   // in a bucket of >= 2
    }
    nd = wave_reduce_add<uint32_t>(nd);
    if ((threadIdx.x & 63) == 0 && nd) atomicAdd(ctr, nd);
}

// list the mixed buckets [l, r] (packed l << 32 | r)
__global__ void k_fb_list(const uint32_t* __restrict__ head, const uint64_t* __restrict__ hp,
                          const uint32_t* __restrict__ mixed, uint64_t* __restrict__ list, uint32_t* __restrict__ ctr,
                          uint32_t n, uint32_t stamp)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x + 1;   // bucket ending at i - 1
    if (i > n) return;
    if (i < n && !head[i]) return;
    const uint32_t l = (uint32_t)hp[i - 1];
    if (mixed[l] != stamp) return;
    list[atomicAdd(ctr, 1u)] = ((uint64_t)l << 32) | (i - 1);
}

// One fallbackQSort3 partition step (fbp_partition, same pivot `med`) on a
// range too large for the wave's LDS, computed by the whole wave as a
// permutation instead of lane 0's serial scan.  The serial loop decomposes:
// * the left scan stops at the k-th '>' (g_k), the right scan at the k-th '<'
//   from the right (l_k), and the two swap while g_k < l_k; the scans meet at
//   p = the first non-'=' position with (# non-'=' before it) >= n('<'); the
//   left scan owns [lo, p), the right [p, hi], every '>' left of p is paired;
// * in the left part the '=' keys collect at lo in arrival order and the
//   '<' run [ltLo, unLo) behaves as a queue on the positions themselves: cell
//   c receives the arriving '<' (own or paired element), or, for a '=' of rank
//   h (h '=' before it), the element cell h received -- chains resolved by
//   pointer jumping; the right part is the mirror image;
// * the two vswaps are a fixed block exchange.
// Scratch: A (list of '<' then '>' offsets, then the gather indices) and B
// (the pointer array, then a staging copy), m words each, indexed by offset.
constexpr uint32_t FB_RES = 0x80000000u;

__device__ __forceinline__ void fbw_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
}

__device__ bool fbw_partition(uint32_t* __restrict__ key, uint32_t* __restrict__ fm, int32_t lo, int32_t hi, uint32_t med,
                              uint32_t* __restrict__ A, uint32_t* __restrict__ B, int32_t& alo, int32_t& ahi, int32_t& blo,
                              int32_t& bhi)
{
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t lt = lanemask_lt();
    const uint32_t m = (uint32_t)(hi - lo + 1);
    uint32_t* kk = key + lo;
    uint32_t* ff = fm + lo;
    uint32_t cl = 0, cg = 0;
    for (uint32_t j = lane; j < m; j += 64) {
        const uint32_t k = kk[j];
        cl += k < med;
        cg += k > med;
    }
    const uint32_t nL = wave_reduce_add<uint32_t>(cl), nG = wave_reduce_add<uint32_t>(cg), nE = m - nL - nG;
    if (nL + nG == 0) return false;                      // every key equals the pivot: nothing moves
    // lists of '<' and '>' offsets; the meeting point p
    uint32_t rL = 0, rG = 0, p = m, lbp = nL, gbp = nG;
    for (uint32_t j0 = 0; j0 < m; j0 += 64) {
        const uint32_t j = j0 + lane;
        const bool ok = j < m;
        const uint32_t k = ok ? kk[j] : med;
        const bool isL = k < med, isG = k > med;
        const uint64_t bL = __ballot(isL), bG = __ballot(isG);
        const uint32_t lb = rL + (uint32_t)__popcll(bL & lt), gb = rG + (uint32_t)__popcll(bG & lt);
        if (isL) A[lb] = j;
        if (isG) A[nL + gb] = j;
        if (p == m) {
            const uint64_t hit = __ballot((isL || isG) && lb + gb >= nL);
            if (hit) {
                const int h = __ffsll((unsigned long long)hit) - 1;
                p = j0 + (uint32_t)h;
                lbp = (uint32_t)__shfl((int)lb, h, 64);
                gbp = (uint32_t)__shfl((int)gb, h, 64);
            }
        }
        rL += (uint32_t)__popcll(bL);
        rG += (uint32_t)__popcll(bG);
    }
    const uint32_t nEL = p - lbp - gbp, nER = nE - nEL;
    fbw_sync();
    // the pointer array: resolved cells carry FB_RES | source offset
    rL = rG = 0;
    uint32_t rE = 0;
    for (uint32_t j0 = 0; j0 < m; j0 += 64) {
        const uint32_t j = j0 + lane;
        const bool ok = j < m;
        const uint32_t k = ok ? kk[j] : 0u;
        const bool isL = ok && k < med, isG = ok && k > med, isE = ok && k == med;
        const uint64_t bL = __ballot(isL), bG = __ballot(isG), bE = __ballot(isE);
        const uint32_t lb = rL + (uint32_t)__popcll(bL & lt), gb = rG + (uint32_t)__popcll(bG & lt),
                       eb = rE + (uint32_t)__popcll(bE & lt);
        if (ok) {
            uint32_t v;
            if (j < p) {
                if (isE) v = eb == j ? FB_RES : eb;                  // eb == j: no '<' queued yet, stays put
                else if (isL) v = FB_RES | j;
                else v = FB_RES | A[nL - 1 - gb];                   // paired with the (gb+1)-th '<' from the right
            } else {
                const uint32_t ea = nE - eb - 1;                    // '=' after it (for a '=')
                if (isE) v = ea == m - 1 - j ? FB_RES : m - 1 - ea;
                else if (isG) v = FB_RES | j;
                else v = FB_RES | A[2 * nL - lb - 1];               // paired with the (nL-lb)-th '>' from the left
            }
            B[j] = v;
        }
        rL += (uint32_t)__popcll(bL);
        rG += (uint32_t)__popcll(bG);
        rE += (uint32_t)__popcll(bE);
    }
    for (;;) {                                                       // pointer jumping (chains only go down)
        fbw_sync();
        bool un = false;
        for (uint32_t j = lane; j < m; j += 64) {
            const uint32_t v = B[j];
            if (!(v & FB_RES)) {
                const uint32_t w = B[v];
                B[j] = w;
                un |= !(w & FB_RES);
            }
        }
        if (!__any(un)) break;
    }
    fbw_sync();
    // gather indices after the vswaps (bz:blocksort.c:166-167)
    const uint32_t n1 = nEL < p - nEL ? nEL : p - nEL;
    const uint32_t ul = m - p, m1 = nER < ul - nER ? nER : ul - nER;
    auto phi = [&](uint32_t q) -> uint32_t {
        if (q < n1) return q + (p - n1);
        if (q < p && q >= p - n1) return q - (p - n1);
        if (q >= p && q < p + m1) return q + (m - m1 - p);
        if (q >= m - m1) return q - (m - m1 - p);
        return q;
    };
    rE = 0;
    for (uint32_t j0 = 0; j0 < m; j0 += 64) {
        const uint32_t j = j0 + lane;
        const bool ok = j < m;
        const bool isE = ok && kk[j] == med;
        const uint64_t bE = __ballot(isE);
        const uint32_t eb = rE + (uint32_t)__popcll(bE & lt);
        if (ok) {
            if (j < p) {
                if (isE) A[phi(eb)] = j;
                if (j >= nEL) A[phi(j)] = B[j] & ~FB_RES;
            } else {
                if (isE) A[phi(m - 1 - (nE - eb - 1))] = j;
                if (m - 1 - j >= nER) A[phi(j)] = B[j] & ~FB_RES;
            }
        }
        rE += (uint32_t)__popcll(bE);
    }
    fbw_sync();
    for (uint32_t j = lane; j < m; j += 64) B[j] = kk[A[j]];
    fbw_sync();
    for (uint32_t j = lane; j < m; j += 64) kk[j] = B[j];
    fbw_sync();
    for (uint32_t j = lane; j < m; j += 64) B[j] = ff[A[j]];
    fbw_sync();
    for (uint32_t j = lane; j < m; j += 64) ff[j] = B[j];
    fbw_sync();
    const int32_t nn = lo + (int32_t)nL - 1, mm = hi - (int32_t)nG + 1;
    if (nn - lo > hi - mm) { alo = lo; ahi = nn; blo = mm; bhi = hi; }   // larger pushed first
    else { alo = mm; ahi = hi; blo = lo; bhi = nn; }
    return true;
}

// fallbackQSort3 on every listed bucket: one wave per bucket (persistent)
__global__ void __launch_bounds__(64 * FB_WAVES) k_fb_sort(uint32_t* __restrict__ fmap, uint32_t* __restrict__ key,
                                                           const uint64_t* __restrict__ list,
                                                           const uint32_t* __restrict__ nlist, uint32_t* __restrict__ next,
                                                           uint32_t* __restrict__ sa, uint32_t* __restrict__ sb, int wave_part)
{
    __shared__ uint32_t sk_all[FB_WAVES][FB_CAP], sf_all[FB_WAVES][FB_CAP];
    __shared__ int32_t cmd_all[FB_WAVES][4];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t* sk = sk_all[w];
    uint32_t* sf = sf_all[w];
    int32_t* cmd = cmd_all[w];
    const uint32_t total = *nlist;
    for (;;) {
        uint32_t idx = 0;
        if (lane == 0) idx = atomicAdd(next, 1u);
        idx = (uint32_t)__shfl((int)idx, 0, 64);
        if (idx >= total) break;
        const uint64_t e = list[idx];
        const int32_t l = (int32_t)(e >> 32), rr = (int32_t)(uint32_t)e;
        // lane 0 drives the call's stack; the wave stages ranges that fit the LDS
        int32_t slo[100], shi[100];
        int32_t sp = 0;
        uint32_t lcg = 0;
        if (lane == 0) { slo[0] = l; shi[0] = rr; sp = 1; }
        for (;;) {
            if (lane == 0) {
                cmd[0] = 0;
                while (sp > 0) {
                    --sp;
                    const int32_t lo = slo[sp], hi = shi[sp];
                    if (hi - lo < 10) { fbp_simple(key, fmap, lo, hi); continue; }
                    if ((uint32_t)(hi - lo + 1) <= FB_CAP) { cmd[0] = 1; cmd[1] = lo; cmd[2] = hi; break; }
                    if (wave_part) {     // a large range: the wave partitions it (fbw_partition)
                        lcg = (lcg * 7621u + 1u) % 32768u;                   // as fbp_partition
                        const uint32_t r3 = lcg % 3u;
                        cmd[0] = 3; cmd[1] = lo; cmd[2] = hi;
                        cmd[3] = (int32_t)(r3 == 0 ? key[lo] : r3 == 1 ? key[(lo + hi) >> 1] : key[hi]);
                        break;
                    }
                    int32_t alo, ahi, blo, bhi;
                    if (!fbp_partition(key, fmap, lo, hi, lcg, alo, ahi, blo, bhi)) continue;
                    slo[sp] = alo; shi[sp] = ahi; ++sp;
                    slo[sp] = blo; shi[sp] = bhi; ++sp;
                }
            }
            fbw_sync();
            if (cmd[0] == 0) break;                                // the call is done
            if (cmd[0] == 3) {
                const int32_t lo = cmd[1], hi = cmd[2];
                const uint32_t med = (uint32_t)cmd[3];
                int32_t alo = 0, ahi = 0, blo = 0, bhi = 0;
                const bool split = fbw_partition(key, fmap, lo, hi, med, sa + lo, sb + lo, alo, ahi, blo, bhi);
                if (lane == 0 && split) {
                    slo[sp] = alo; shi[sp] = ahi; ++sp;
                    slo[sp] = blo; shi[sp] = bhi; ++sp;
                }
                fbw_sync();
                continue;
            }
            const int32_t lo = cmd[1], hi = cmd[2], m = hi - lo + 1;
            for (int32_t q = lane; q < m; q += 64) { sk[q] = key[lo + q]; sf[q] = fmap[lo + q]; }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            if (lane == 0) fbp_qsort3(sk, sf, 0, m - 1, lcg);      // the range's whole subtree, in order
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            for (int32_t q = lane; q < m; q += 64) { key[lo + q] = sk[q]; fmap[lo + q] = sf[q]; }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
    }
}

// new heads where the key changes inside a sorted mixed bucket (bz:blocksort.c:299-306)
__global__ void k_fb_heads(const uint32_t* __restrict__ key, const uint64_t* __restrict__ hp,
                           const uint32_t* __restrict__ mixed, uint32_t* __restrict__ head, uint32_t n, uint32_t stamp)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i == 0 || i >= n || head[i]) return;
    if (mixed[(uint32_t)hp[i]] == stamp && key[i] != key[i - 1]) head[i] = 1;
}

__global__ void k_fb_origptr(const uint32_t* __restrict__ fmap, BlockDesc* __restrict__ blocks, uint32_t b, uint32_t n)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && fmap[i] == 0) blocks[b].orig_ptr = i;
}

void launch_bwt(BlockDesc* blocks, uint32_t b0, uint32_t nb, const uint8_t* blkbytes, uint64_t stride,
                const BwtScratch& scr, unsigned long long* stats, hipStream_t st)
{
    hipLaunchKernelGGL(k_bwt, dim3(nb), dim3(BT), 0, st, blocks, b0, blkbytes, stride, scr, stats);
    HIP_CHECK(hipGetLastError());
}

void FbPool::init(int device)
{
    if (dev == device) return;
    if (dev >= 0) throw StarchError(-10, "FbPool: device changed");
    for (int i = 0; i < kStreams; ++i) HIP_CHECK(hipStreamCreateWithFlags(&st[i], hipStreamNonBlocking));
    for (int i = 0; i <= kStreams; ++i) HIP_CHECK(hipEventCreateWithFlags(&ev[i], hipEventDisableTiming));
    dev = device;
}

FbPool::~FbPool()
{
    for (int i = 0; i < kStreams; ++i)
        if (st[i]) { (void)hipStreamSynchronize(st[i]); (void)hipStreamDestroy(st[i]); }
    for (int i = 0; i <= kStreams; ++i)
        if (ev[i]) (void)hipEventDestroy(ev[i]);
}

void launch_fallback(BlockDesc* blocks, uint32_t b0, const uint32_t* which_host, const uint32_t* n_host,
                     uint32_t nwhich, const uint8_t* blkbytes, uint64_t stride, const BwtScratch& scr, FbPool& pool,
                     hipStream_t st)
{
    int dev = 0, ncu = 256;
    HIP_CHECK(hipGetDevice(&dev));
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) == hipSuccess && prop.multiProcessorCount > 0) ncu = prop.multiProcessorCount;
    pool.init(dev);
    static const bool wave_part = [] { const char* e = getenv("STARCH_FB_WAVE"); return !(e && !strcmp(e, "0")); }();
    struct Blk {
        uint32_t slot, b, n;
        uint64_t so;
        hipStream_t s;
        DevBuf* tmp;
        uint64_t H;
        uint32_t stamp;
        bool active;
    };
    std::vector<Blk> bl;
    for (uint32_t q = 0; q < nwhich; ++q) {
        if (n_host[q] == 0) continue;
        const int k = (int)(bl.size() % FbPool::kStreams);
        bl.push_back(Blk{which_host[q], b0 + which_host[q], n_host[q], (uint64_t)which_host[q] * scr.stride,
                         pool.st[k], &pool.tmp[k], 1, 0, true});
    }
    if (bl.empty()) return;
    const int nst = (int)std::min<size_t>(bl.size(), FbPool::kStreams);
    // the sort's results on st come first
    HIP_CHECK(hipEventRecord(pool.ev[FbPool::kStreams], st));
    for (int k = 0; k < nst; ++k) HIP_CHECK(hipStreamWaitEvent(pool.st[k], pool.ev[FbPool::kStreams], 0));
    uint32_t* hc = static_cast<uint32_t*>(pool.ctr.get(bl.size() * 2 * sizeof(uint32_t) + 64));
    for (auto& x : bl) {   // 1-byte bucket sort and the first heads, over the whole GPU
        const uint32_t n = x.n;
        uint32_t* fmap = scr.SA + x.so;
        uint32_t* ecls = scr.RK + x.so;
        uint32_t* head = scr.U + x.so;
        uint32_t* mixed = scr.U2 + x.so;
        const uint8_t* blk = blkbytes + (uint64_t)x.b * stride;
        const uint32_t ntile = (n + FB_TILE - 1) / FB_TILE;
        uint32_t* cnt = reinterpret_cast<uint32_t*>(scr.K2 + x.so);             // ntile x 256 (free until the rounds)
        uint32_t* bst = ecls;                                                     // bucket starts / totals in RK
        HIP_CHECK(hipMemsetAsync(head, 0, (uint64_t)n * sizeof(uint32_t), x.s));
        hipLaunchKernelGGL(k_fb_cnt, dim3(ntile), dim3(256), 0, x.s, blk, n, cnt);
        hipLaunchKernelGGL(k_fb_cscan, dim3(1), dim3(256), 0, x.s, cnt, ntile, bst, bst + 256, head, n);
        hipLaunchKernelGGL(k_fb_place, dim3(ntile), dim3(64), 0, x.s, blk, n, cnt, bst, bst + 256, fmap);
        HIP_CHECK(hipMemsetAsync(mixed, 0, (uint64_t)n * sizeof(uint32_t), x.s));
        HIP_CHECK(hipGetLastError());
    }
    // rounds H = 1, 2, 4, ... (bz:blocksort.c:252-327): every active block's
    // round is issued on its stream, then one wait for all of them
    for (;;) {
        bool any = false;
        for (size_t q = 0; q < bl.size(); ++q) {
            Blk& x = bl[q];
            if (!x.active) continue;
            any = true;
            const uint32_t n = x.n;
            uint32_t* fmap = scr.SA + x.so;
            uint32_t* ecls = scr.RK + x.so;
            uint32_t* key = scr.V + x.so;
            uint32_t* head = scr.U + x.so;
            uint32_t* mixed = scr.U2 + x.so;
            uint64_t* hp = scr.K + x.so;
            uint64_t* list = scr.K2 + x.so;
            uint32_t* ctr = scr.V2 + x.so;                      // [0] not done, [1] mixed buckets, [2] next bucket
            const dim3 g((n + 255) / 256), g1((n + 256) / 256);
            ++x.stamp;
            hipLaunchKernelGGL(k_fb_hp, g, dim3(256), 0, x.s, head, hp, n, ctr);
            scan::incl_max_u64(hp, n, *x.tmp, x.s);
            hipLaunchKernelGGL(k_fb_eclass, g, dim3(256), 0, x.s, fmap, hp, ecls, n, (uint32_t)(x.H % n));
            hipLaunchKernelGGL(k_fb_key, g, dim3(256), 0, x.s, fmap, ecls, head, hp, key, mixed, ctr, n, x.stamp);
            hipLaunchKernelGGL(k_fb_list, g1, dim3(256), 0, x.s, head, hp, mixed, list, ctr + 1, n, x.stamp);
            HIP_CHECK(hipGetLastError());
            HIP_CHECK(hipMemcpyAsync(hc + 2 * q, ctr, 2 * sizeof(uint32_t), hipMemcpyDeviceToHost, x.s));
        }
        if (!any) break;
        for (int k = 0; k < nst; ++k) HIP_CHECK(hipStreamSynchronize(pool.st[k]));
        for (size_t q = 0; q < bl.size(); ++q) {
            Blk& x = bl[q];
            if (!x.active) continue;
            const uint32_t n = x.n, not_done = hc[2 * q], nmixed = hc[2 * q + 1];
            uint32_t* fmap = scr.SA + x.so;
            uint32_t* ecls = scr.RK + x.so;
            uint32_t* key = scr.V + x.so;
            uint32_t* head = scr.U + x.so;
            uint32_t* mixed = scr.U2 + x.so;
            uint64_t* hp = scr.K + x.so;
            uint64_t* list = scr.K2 + x.so;
            uint32_t* ctr = scr.V2 + x.so;
            const dim3 g((n + 255) / 256);
            if (nmixed) {
                const uint32_t wg = std::min<uint32_t>((nmixed + FB_WAVES - 1) / FB_WAVES, (uint32_t)ncu);
                hipLaunchKernelGGL(k_fb_sort, dim3(wg), dim3(64 * FB_WAVES), 0, x.s, fmap, key, list, ctr + 1, ctr + 2,
                                   ecls, reinterpret_cast<uint32_t*>(list) + n, wave_part ? 1 : 0);
                hipLaunchKernelGGL(k_fb_heads, g, dim3(256), 0, x.s, key, hp, mixed, head, n, x.stamp);
                HIP_CHECK(hipGetLastError());
            }
            if (2 * x.H > n || not_done == 0) {                 // H *= 2; if (H > nblock || nNotDone == 0) break
                hipLaunchKernelGGL(k_fb_origptr, g, dim3(256), 0, x.s, fmap, blocks, x.b, n);
                HIP_CHECK(hipGetLastError());
                x.active = false;
            }
            x.H *= 2;
        }
    }
    // st continues after every block's replay
    for (int k = 0; k < nst; ++k) {
        HIP_CHECK(hipEventRecord(pool.ev[k], pool.st[k]));
        HIP_CHECK(hipStreamWaitEvent(st, pool.ev[k], 0));
    }
}

}  // namespace bz
