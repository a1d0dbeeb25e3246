// starch_amd/csrc/bz2_tables.hip -- coding-table selection and Huffman code
// lengths on MI355X (restates sendMTFValues' table part, bz:compress.c:266-
// 489, and BZ2_hbMakeCodeLengths / BZ2_hbAssignCodes, bz:huffman.c:63-166).
//
// One 1024-thread workgroup per block.  Per refinement pass the 50-symbol
// groups are costed against every table in parallel (lengths in LDS, first
// minimum wins as in bz:compress.c:399-401) and the chosen table's symbol
// frequencies are accumulated with LDS atomics; then one lane per table
// rebuilds that table's lengths with the exact heap algorithm (weights carry
// depth in the low byte, maxLen 17, halving retry).  The block's exact bit
// length (header + selectors + tables + data) is produced here, so stream
// offsets are known before any bit is written.
#include "bz2_bwt.hpp"

namespace bz {

constexpr int TT = 1024;

struct HuffSmem {
    int32_t heap[6][262];
    int32_t weight[6][516];
    int32_t parent[6][516];
};

__device__ void hb_make_lengths(uint8_t* len, const uint32_t* freq, int32_t alpha, int32_t max_len, int32_t* heap,
                                int32_t* weight, int32_t* parent)
{
    for (int32_t i = 0; i < alpha; ++i) weight[i + 1] = (int32_t)((freq[i] == 0 ? 1u : freq[i]) << 8);
    for (;;) {
        int32_t nodes = alpha, nheap = 0;
        heap[0] = 0; weight[0] = 0; parent[0] = -2;
        for (int32_t i = 1; i <= alpha; ++i) {
            parent[i] = -1;
            heap[++nheap] = i;
            int32_t zz = nheap, t = heap[zz];                       // UPHEAP
            while (weight[t] < weight[heap[zz >> 1]]) { heap[zz] = heap[zz >> 1]; zz >>= 1; }
            heap[zz] = t;
        }
        while (nheap > 1) {
            int32_t pick[2];
            for (int q = 0; q < 2; ++q) {
                pick[q] = heap[1];
                heap[1] = heap[nheap--];
                int32_t zz = 1, t = heap[zz];                       // DOWNHEAP
                for (;;) {
                    int32_t yy = zz << 1;
                    if (yy > nheap) break;
                    if (yy < nheap && weight[heap[yy + 1]] < weight[heap[yy]]) ++yy;
                    if (weight[t] < weight[heap[yy]]) break;
                    heap[zz] = heap[yy];
                    zz = yy;
                }
                heap[zz] = t;
            }
            ++nodes;
            parent[pick[0]] = parent[pick[1]] = nodes;
            int32_t wa = weight[pick[0]], wb = weight[pick[1]];
            int32_t da = wa & 0xff, db = wb & 0xff;
            weight[nodes] = (int32_t)(((uint32_t)wa & 0xffffff00u) + ((uint32_t)wb & 0xffffff00u)) |
                            (1 + (da > db ? da : db));
            parent[nodes] = -1;
            heap[++nheap] = nodes;
            int32_t zz = nheap, t = heap[zz];
            while (weight[t] < weight[heap[zz >> 1]]) { heap[zz] = heap[zz >> 1]; zz >>= 1; }
            heap[zz] = t;
        }
        bool too_long = false;
        for (int32_t i = 1; i <= alpha; ++i) {
            int32_t d = 0, k = i;
            while (parent[k] >= 0) { k = parent[k]; ++d; }
            len[i - 1] = (uint8_t)d;
            if (d > max_len) too_long = true;
        }
        if (!too_long) break;
        for (int32_t i = 1; i <= alpha; ++i) weight[i] = (1 + ((weight[i] >> 8) / 2)) << 8;
    }
}

// The same algorithm for alphabets <= 32 run by one whole wave, with the heap,
// the weights and the parents in registers: node k's weight and parent in
// lane k (2 * alpha - 1 <= 63 nodes), heap position z in lane z.  The control
// flow is wave-uniform and every heap step reads and writes single lanes
// (v_readlane with scalar indices, one v_cndmask per write), so the serial heap runs on
// scalar-latency steps instead of one lane's chain of LDS round trips; the
// depth walk is lane-parallel.  Same heap, same ties, same lengths.
__device__ __forceinline__ int32_t rl(int32_t v, int32_t i) { return __builtin_amdgcn_readlane(v, i); }
__device__ __forceinline__ int32_t wl(int32_t v, int32_t x, int32_t i) { return (int32_t)(threadIdx.x & 63) == i ? x : v; }

__device__ void hb_make_lengths_wave(uint8_t* len, const uint32_t* freq, int32_t alpha, int32_t max_len)
{
    const int32_t lane = (int32_t)(threadIdx.x & 63);
    const bool sym = lane >= 1 && lane <= alpha;
    int32_t W = 0;                                             // weight of node `lane`
    if (sym) W = (int32_t)((freq[lane - 1] == 0 ? 1u : freq[lane - 1]) << 8);
    for (;;) {
        int32_t P = lane == 0 ? -2 : -1;                       // parent of node `lane`
        int32_t H = 0;                                         // heap entry at position `lane`
        W = lane == 0 ? 0 : W;
        int32_t nodes = alpha, nheap = 0;
        auto upheap = [&](int32_t t) {
            const int32_t wt = rl(W, t);
            int32_t zz = nheap;
            for (;;) {
                const int32_t hp = rl(H, zz >> 1);
                if (!(wt < rl(W, hp))) break;
                H = wl(H, hp, zz);
                zz >>= 1;
            }
            H = wl(H, t, zz);
        };
        for (int32_t i = 1; i <= alpha; ++i) {
            ++nheap;
            upheap(i);
        }
        while (nheap > 1) {
            int32_t pick[2];
            for (int q = 0; q < 2; ++q) {
                pick[q] = rl(H, 1);
                const int32_t t = rl(H, nheap);
                --nheap;
                const int32_t wt = rl(W, t);
                int32_t zz = 1;
                for (;;) {
                    int32_t yy = zz << 1;
                    if (yy > nheap) break;
                    int32_t hy = rl(H, yy), wy = rl(W, hy);
                    if (yy < nheap) {
                        const int32_t h1 = rl(H, yy + 1), w1 = rl(W, h1);
                        if (w1 < wy) { ++yy; hy = h1; wy = w1; }
                    }
                    if (wt < wy) break;
                    H = wl(H, hy, zz);
                    zz = yy;
                }
                H = wl(H, t, zz);
            }
            ++nodes;
            P = wl(P, nodes, pick[0]);
            P = wl(P, nodes, pick[1]);
            const int32_t wa = rl(W, pick[0]), wb = rl(W, pick[1]);
            const int32_t da = wa & 0xff, db = wb & 0xff;
            W = wl(W, (int32_t)(((uint32_t)wa & 0xffffff00u) + ((uint32_t)wb & 0xffffff00u)) | (1 + (da > db ? da : db)),
                   nodes);
            P = wl(P, -1, nodes);
            ++nheap;
            upheap(nodes);
        }
        // depth of every symbol: all lanes walk their parent chains at once
        int32_t d = 0, k = lane;
        bool walking = sym;
        while (__ballot(walking)) {
            const int32_t pk = __shfl(P, k, 64);
            if (walking && pk >= 0) { k = pk; ++d; } else walking = false;
        }
        if (sym) len[lane - 1] = (uint8_t)d;
        if (!__ballot(sym && d > max_len)) break;
        if (sym) W = (1 + ((W >> 8) / 2)) << 8;
    }
}

__global__ void __launch_bounds__(TT) k_tables(BlockDesc* __restrict__ blocks, uint32_t b0,
                                                const uint16_t* __restrict__ mtfv_all, uint64_t mtf_stride,
                                                Tables* __restrict__ tabs, uint8_t* __restrict__ sel_all,
                                                uint32_t* __restrict__ gbits_all, uint8_t* __restrict__ hist_all,
                                                uint64_t hist_stride)
{
    __shared__ HuffSmem hs;
    __shared__ uint8_t len[6][258];
    __shared__ uint32_t rfreq[6][258];
    __shared__ uint32_t freq[258];
    __shared__ uint32_t scan_sh[TT / 64 + 1];
    __shared__ uint32_t info[4];
    __shared__ unsigned long long hdr_bits;

    const int tid = threadIdx.x;
    const uint32_t b = b0 + blockIdx.x;
    const uint16_t* mtfv = mtfv_all + (uint64_t)b * mtf_stride;
    uint8_t* sel = sel_all + (uint64_t)b * (2 * kMaxSelectors);
    uint8_t* selmtf = sel + kMaxSelectors;
    uint32_t* gbits = gbits_all + (uint64_t)b * kMaxSelectors;
    const uint32_t n_mtf = blocks[b].n_mtf;
    const int32_t alpha = (int32_t)blocks[b].n_in_use + 2;
    if (alpha <= 32) return;                       // uniform: k_tables32
    const int ng = n_mtf < 200 ? 2 : n_mtf < 600 ? 3 : n_mtf < 1200 ? 4 : n_mtf < 2400 ? 5 : 6;
    const uint32_t nsel = (n_mtf + 49) / 50;

    if (tid < 258) freq[tid] = tabs[b].freq[tid];
    for (int i = tid; i < 6 * 258; i += TT) (&len[0][0])[i] = 15;   // BZ_GREATER_ICOST
    __syncthreads();
    if (tid == 0) {   // initial equal-frequency bands (bz:compress.c:280-317)
        int32_t parts = ng, rem = (int32_t)n_mtf, gs = 0;
        while (parts > 0) {
            int32_t target = rem / parts, ge = gs - 1, acc = 0;
            while (acc < target && ge < alpha - 1) { ++ge; acc += (int32_t)freq[ge]; }
            if (ge > gs && parts != ng && parts != 1 && ((ng - parts) % 2 == 1)) { acc -= (int32_t)freq[ge]; --ge; }
            for (int32_t v = 0; v < alpha; ++v) len[parts - 1][v] = (v >= gs && v <= ge) ? 0 : 15;
            --parts;
            gs = ge + 1;
            rem -= acc;
        }
    }
    __syncthreads();
    // Small alphabets: per-group symbol histograms (u8, <= 50) built once, so a
    // group's cost against a table is alpha multiply-adds and the per-table
    // frequencies are a reduction over groups by (symbol, group chunk) lanes
    // instead of 50 contended LDS atomics per group.
    const bool use_hist = alpha <= 64;
    uint8_t* hist = hist_all + (uint64_t)blockIdx.x * hist_stride;
    if (use_hist) {
        // layout [symbol][group]: lanes of a wave touch consecutive bytes
        for (uint32_t g = tid; g < nsel; g += TT) {
            for (int32_t v = 0; v < alpha; ++v) hist[(uint64_t)v * nsel + g] = 0;
            uint32_t gs = g * 50, ge = gs + 50;
            if (ge > n_mtf) ge = n_mtf;
            const uint32_t* m32 = reinterpret_cast<const uint32_t*>(mtfv + gs);   // gs even: 4-B aligned
            for (uint32_t i = gs; i < ge; i += 2) {
                uint32_t w = m32[(i - gs) >> 1];
                hist[(uint64_t)(w & 0xffffu) * nsel + g]++;
                if (i + 1 < ge) hist[(uint64_t)(w >> 16) * nsel + g]++;
            }
        }
    }
    __syncthreads();
    for (int iter = 0; iter < 4; ++iter) {                         // BZ_N_ITERS
        for (int i = tid; i < 6 * 258; i += TT) (&rfreq[0][0])[i] = 0;
        __syncthreads();
        for (uint32_t g = tid; g < nsel; g += TT) {
            uint32_t cost[6] = {0, 0, 0, 0, 0, 0};
            if (use_hist) {
                for (int32_t v = 0; v < alpha; ++v) {
                    uint32_t c = hist[(uint64_t)v * nsel + g];
                    if (!c) continue;
#pragma unroll
                    for (int t = 0; t < 6; ++t) cost[t] += c * len[t][v];
                }
            } else {
                uint32_t gs = g * 50, ge = gs + 50;
                if (ge > n_mtf) ge = n_mtf;
                for (uint32_t i = gs; i < ge; ++i) {
                    uint32_t v = mtfv[i];
#pragma unroll
                    for (int t = 0; t < 6; ++t) cost[t] += len[t][v];
                }
            }
            int bt = 0;
            uint32_t bc = cost[0];
            for (int t = 1; t < ng; ++t) if (cost[t] < bc) { bc = cost[t]; bt = t; }
            sel[g] = (uint8_t)bt;
            if (!use_hist) {
                uint32_t gs = g * 50, ge = gs + 50;
                if (ge > n_mtf) ge = n_mtf;
                for (uint32_t i = gs; i < ge; ++i) atomicAdd(&rfreq[bt][mtfv[i]], 1u);
            }
        }
        __syncthreads();
        if (use_hist) {
            const uint32_t nchunk = TT / (uint32_t)alpha;
            const uint32_t v = tid % alpha, c = tid / alpha;
            if (c < nchunk) {
                const uint32_t per = (nsel + nchunk - 1) / nchunk;
                uint32_t acc[6] = {0, 0, 0, 0, 0, 0};
                const uint32_t g1 = (c + 1) * per < nsel ? (c + 1) * per : nsel;
                for (uint32_t g = c * per; g < g1; ++g) {
                    uint32_t cnt = hist[(uint64_t)v * nsel + g];
                    uint32_t t = sel[g];
#pragma unroll
                    for (int q = 0; q < 6; ++q) acc[q] += (t == (uint32_t)q) ? cnt : 0u;
                }
                for (int q = 0; q < ng; ++q) if (acc[q]) atomicAdd(&rfreq[q][v], acc[q]);
            }
        }
        __syncthreads();
        if (tid < ng) hb_make_lengths(len[tid], rfreq[tid], alpha, 17, hs.heap[tid], hs.weight[tid], hs.parent[tid]);
        __syncthreads();
    }
    // selector MTF (bz:compress.c:461-478) and header size
    if (tid == 0) {
        uint8_t pos[6];
        for (int i = 0; i < ng; ++i) pos[i] = (uint8_t)i;
        uint64_t sbits = 0;
        for (uint32_t i = 0; i < nsel; ++i) {
            uint8_t want = sel[i];
            int j = 0;
            uint8_t carry_v = pos[0];
            while (carry_v != want && j < 5) { ++j; uint8_t t = pos[j]; pos[j] = carry_v; carry_v = t; }
            pos[0] = carry_v;
            selmtf[i] = (uint8_t)j;
            sbits += (uint64_t)j + 1;
        }
        uint32_t used16 = 0;
        for (int i = 0; i < 16; ++i) {
            uint32_t w = blocks[b].in_use[i >> 1];
            uint32_t half = (i & 1) ? (w >> 16) : (w & 0xffffu);
            if (half) ++used16;
        }
        uint64_t tbits = 0;
        for (int t = 0; t < ng; ++t) {
            int32_t cur = len[t][0];
            tbits += 5;
            for (int32_t i = 0; i < alpha; ++i) {
                int32_t d = (int32_t)len[t][i] - cur;
                tbits += 1 + 2 * (uint64_t)(d < 0 ? -d : d);
                cur = len[t][i];
            }
        }
        hdr_bits = 48 + 32 + 1 + 24 + 16 + 16ull * used16 + 3 + 15 + sbits + tbits;
        blocks[b].hdr_bits = (uint32_t)hdr_bits;
    }
    // canonical codes (bz:huffman.c:152-166)
    if (tid < ng) {
        int32_t mn = 32, mx = 0;
        for (int32_t i = 0; i < alpha; ++i) {
            int32_t l = len[tid][i];
            if (l > mx) mx = l;
            if (l < mn) mn = l;
        }
        int32_t v = 0;
        for (int32_t L = mn; L <= mx; ++L) {
            for (int32_t i = 0; i < alpha; ++i) if (len[tid][i] == L) tabs[b].code[tid][i] = (uint32_t)v++;
            v <<= 1;
        }
        for (int32_t i = 0; i < alpha; ++i) tabs[b].len[tid][i] = len[tid][i];
    }
    __syncthreads();
    // data bits per group
    uint64_t local = 0;
    for (uint32_t g = tid; g < nsel; g += TT) {
        const uint8_t* L = len[sel[g]];
        uint32_t bits = 0;
        if (use_hist) {
            for (int32_t v = 0; v < alpha; ++v) bits += (uint32_t)hist[(uint64_t)v * nsel + g] * L[v];
        } else {
            uint32_t gs = g * 50, ge = gs + 50;
            if (ge > n_mtf) ge = n_mtf;
            for (uint32_t i = gs; i < ge; ++i) bits += L[mtfv[i]];
        }
        gbits[g] = bits;
        local += bits;
    }
    local = wave_reduce_add(local);
    if ((tid & 63) == 0) atomicAdd(&hdr_bits, (unsigned long long)local);
    __syncthreads();
    if (tid == 0) {
        blocks[b].bits = hdr_bits;
        blocks[b].n_groups = (uint32_t)ng;
        blocks[b].n_sel = nsel;
    }
}

// ---------------------------------------------------------------------------
// k_tables32: the same computation for alphabets <= 32 (every BED transform).
// Each 50-symbol group's histogram (32 u8 counts) is built once and kept in
// HBM; a group's cost against table t is then sum_v count_v * len_t[v], four
// symbols per v_dot4_u32_u8 (the packed-cost idea of bz:compress.c:379-398
// applied to byte lanes); the first minimum wins (bz:compress.c:399-401).
// Per-table symbol frequencies: per-table wave reductions into per-wave rows.
// ---------------------------------------------------------------------------
// 256 threads and small LDS: several blocks per CU, so one block's serial
// phases (Huffman construction, band setup) overlap other blocks' work
#ifndef STARCH_TABLES_WPE
#define STARCH_TABLES_WPE 4
#endif
#ifdef STARCH_TABLES_PROF
__device__ unsigned long long g_tprof[8];
#define TPROF(k) do { __syncthreads(); if (threadIdx.x == 0) { const uint64_t t_ = wall_clock64(); \
    atomicAdd(&g_tprof[k], (unsigned long long)(t_ - tp_last)); tp_last = t_; } } while (0)
#else
#define TPROF(k) do {} while (0)
#endif

__device__ __forceinline__ uint32_t byte_of(const uint32_t (&h)[8], int v)
{
    return (h[v >> 2] >> (8 * (v & 3))) & 0xffu;
}

// Sum over the wave of 32 u8 counts per lane (each <= 50; a lane adds only
// when `mine`), by recursive halving, all on the VALU: at lane bits 5 and 4
// (gfx950 v_permlane32_swap / v_permlane16_swap) a lane keeps half of its
// packed u8 words (<= 4 x 50 per byte) plus its partner's copy of that half;
// the two words left become u16 pairs, bit 3 halves again (DPP row_ror:8) and
// three DPP row shifts sum each 8-lane run.  Lanes 7 and 15 of every row then
// hold symbols 4q..4q+3, q = 4 * bit5 + 2 * bit4 + bit3, summed over the wave:
// ev = counts of 4q | 4q+2 << 16, od = 4q+1 | 4q+3 << 16.  ~30 VALU ops
// where 16 wave reductions took ~110.
__device__ __forceinline__ void wave_sum_u8x32(const uint32_t (&h)[8], bool mine, int lane, uint32_t& ev,
                                               uint32_t& od, uint32_t& q)
{
    uint32_t a[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] = mine ? h[k] : 0u;
#pragma unroll
    for (int i = 0; i < 4; ++i) {                  // bit 5: words k (lo half) | k + 4 (hi half)
        const auto r = __builtin_amdgcn_permlane32_swap(a[i], a[4 + i], false, false);
        a[i] = r[0] + r[1];
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {                  // bit 4: words k | k + 2
        const auto r = __builtin_amdgcn_permlane16_swap(a[i], a[2 + i], false, false);
        a[i] = r[0] + r[1];
    }
    const bool b3 = (lane & 8) != 0;               // bit 3: words q0 | q0 + 1, as u16 pairs
    const uint32_t src = b3 ? a[0] : a[1], own = b3 ? a[1] : a[0];
    ev = own & 0x00ff00ffu;
    od = (own >> 8) & 0x00ff00ffu;
    ev += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(src & 0x00ff00ffu), 0x128, 0xf, 0xf, false);
    od += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)((src >> 8) & 0x00ff00ffu), 0x128, 0xf, 0xf, false);
    ev += dpp_up(ev, 1); od += dpp_up(od, 1);      // 8-lane runs: lanes 7, 15 of a row
    ev += dpp_up(ev, 2); od += dpp_up(od, 2);
    ev += dpp_up(ev, 4); od += dpp_up(od, 4);
    q = ((uint32_t)lane >> 5) * 4u + (((uint32_t)lane >> 4) & 1u) * 2u + (b3 ? 1u : 0u);
}

// T32 threads per block: 256 when the batch fills the GPU with blocks (their
// serial phases overlap other blocks'), 1024 for a batch of few blocks (each
// block's group loops and its six heaps spread over 16 waves: per-block latency)
template <int T32>
__global__ void __launch_bounds__(T32) __attribute__((amdgpu_waves_per_eu(STARCH_TABLES_WPE))) k_tables32(BlockDesc* __restrict__ blocks, uint32_t b0,
                                                   const uint16_t* __restrict__ mtfv_all, uint64_t mtf_stride,
                                                   Tables* __restrict__ tabs, uint8_t* __restrict__ sel_all,
                                                   uint32_t* __restrict__ gbits_all, uint4* __restrict__ hist_all,
                                                   uint64_t hist_stride)
{
    constexpr int NW32 = T32 / 64;
    // phase-disjoint scratch shares one LDS region (histograms, then the four
    // refinement passes, then the selector MTF) and the per-table rows are
    // alpha <= 32 wide: ~27 KB, so LDS no longer caps residency; registers do
    // (STARCH_TABLES_WPE blocks per CU; 4 measured best: 5 spills the hoisted
    // packed lengths, profiles/r01_v24_tables_wpe.json)
    union Scratch {
        uint32_t hl[8][T32];
        struct { uint32_t rf[NW32][6][32]; uint32_t rfreq[6][32]; } it;
        NibState nst[T32];
    };
    __shared__ Scratch u;
    __shared__ uint8_t len[6][32];
    __shared__ uint32_t pl4[6][8];                 // table t's code lengths, 4 symbols per word
    __shared__ uint32_t freq[258];
    __shared__ uint8_t sel_l[kMaxSelectors];
    __shared__ unsigned long long hdr_bits, sbits_sh;
    auto& hl = u.hl;
    auto& rf = u.it.rf;
    auto& rfreq = u.it.rfreq;
    auto& nst = u.nst;

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const uint32_t b = b0 + blockIdx.x;
    const int32_t alpha = (int32_t)blocks[b].n_in_use + 2;
    if (alpha > 32) return;                        // uniform: k_tables handles it
    // alphabets <= 32: the MTF values are bytes (k_mtf_emit / k_mtf_scan_runs)
    const uint8_t* mtfv = reinterpret_cast<const uint8_t*>(mtfv_all + (uint64_t)b * mtf_stride);
    uint8_t* sel = sel_all + (uint64_t)b * (2 * kMaxSelectors);
    uint8_t* selmtf = sel + kMaxSelectors;
    uint32_t* gbits = gbits_all + (uint64_t)b * kMaxSelectors;
    uint4* hist = hist_all + (uint64_t)blockIdx.x * hist_stride;     // [group][2] x uint4
    const uint32_t n_mtf = blocks[b].n_mtf;
    const int ng = n_mtf < 200 ? 2 : n_mtf < 600 ? 3 : n_mtf < 1200 ? 4 : n_mtf < 2400 ? 5 : 6;
    const uint32_t nsel = (n_mtf + 49) / 50;

#ifdef STARCH_TABLES_PROF
    uint64_t tp_last = wall_clock64();
#endif
    for (int i = tid; i < 258; i += T32) freq[i] = 0;
    for (int i = tid; i < 6 * 32; i += T32) (&len[0][0])[i] = 15;   // BZ_GREATER_ICOST
    __syncthreads();
    // ---- per-group histograms (+ mtfFreq) ----
    for (uint32_t g0 = 0; g0 < nsel; g0 += T32) {
        const uint32_t g = g0 + tid;
        uint32_t h[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (g < nsel) {
#pragma unroll
            for (int q = 0; q < 8; ++q) hl[q][tid] = 0;
            const uint32_t gs = g * 50;
            const uint32_t cnt = gs + 50 < n_mtf ? 50u : n_mtf - gs;
            // the group's 50 bytes by four aligned 16-B loads over its 64-byte
            // window (the block's base is 32-B aligned and gs = 50 g is even,
            // so the group starts at byte o <= 14 of the window)
            const uintptr_t ga = reinterpret_cast<uintptr_t>(mtfv + gs);
            const uint4* w4 = reinterpret_cast<const uint4*>(ga & ~(uintptr_t)15);
            const uint32_t o = (uint32_t)(ga & 15u), bend = o + cnt;          // bytes [o, bend)
            uint32_t wv[16];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint4 x = 16u * k < bend ? w4[k] : make_uint4(0, 0, 0, 0);   // all loads in flight
                wv[4 * k] = x.x; wv[4 * k + 1] = x.y; wv[4 * k + 2] = x.z; wv[4 * k + 3] = x.w;
            }
#pragma unroll
            for (int k = 0; k < 64; ++k) {
                const uint32_t j = (uint32_t)k - o;                          // byte of the group (wraps if k < o)
                const uint32_t v = (wv[k >> 2] >> (8 * (k & 3))) & 0xffu;
                if (j < cnt) atomicAdd(&hl[v >> 2][tid], 1u << (8 * (v & 3)));
            }
#pragma unroll
            for (int q = 0; q < 8; ++q) h[q] = hl[q][tid];
            hist[2 * g] = make_uint4(h[0], h[1], h[2], h[3]);
            hist[2 * g + 1] = make_uint4(h[4], h[5], h[6], h[7]);
        }
        // mtfFreq: wave sums (wave_sum_u8x32), its 8 result lanes add
        {
            uint32_t ev, od, q;
            wave_sum_u8x32(h, true, lane, ev, od, q);
            if ((lane & 7) == 7) {
                if (ev & 0xffffu) atomicAdd(&freq[4 * q], ev & 0xffffu);
                if (od & 0xffffu) atomicAdd(&freq[4 * q + 1], od & 0xffffu);
                if (ev >> 16) atomicAdd(&freq[4 * q + 2], ev >> 16);
                if (od >> 16) atomicAdd(&freq[4 * q + 3], od >> 16);
            }
        }
    }
    __syncthreads();
    if (wid == 0) {   // initial equal-frequency bands (bz:compress.c:280-317), wave-uniform
        const int32_t fv = lane < alpha ? (int32_t)freq[lane] : 0;
        int32_t parts = ng, rem = (int32_t)n_mtf, gs = 0;
        while (parts > 0) {
            int32_t target = rem / parts, ge = gs - 1, acc = 0;
            while (acc < target && ge < alpha - 1) { ++ge; acc += rl(fv, ge); }
            if (ge > gs && parts != ng && parts != 1 && ((ng - parts) % 2 == 1)) { acc -= rl(fv, ge); --ge; }
            if (lane < alpha) len[parts - 1][lane] = (lane >= gs && lane <= ge) ? 0 : 15;
            --parts;
            gs = ge + 1;
            rem -= acc;
        }
    }
    for (int i = tid; i < 258; i += T32) tabs[b].freq[i] = freq[i];
    __syncthreads();
    TPROF(0);
    for (int iter = 0; iter < 4; ++iter) {                         // BZ_N_ITERS
        if (tid < 48) {
            const int t = tid >> 3, q = tid & 7;
            uint32_t w = 0;
            for (int b = 0; b < 4; ++b)
                if (4 * q + b < alpha && t < ng) w |= (uint32_t)len[t][4 * q + b] << (8 * b);
            pl4[t][q] = w;
        }
        for (int i = tid; i < NW32 * 6 * 32; i += T32) (&rf[0][0][0])[i] = 0;
        __syncthreads();
        uint4 n0 = make_uint4(0, 0, 0, 0), n1 = n0;
        if ((uint32_t)tid < nsel) { n0 = hist[2 * tid]; n1 = hist[2 * tid + 1]; }
        // wave-uniform trip count: every lane runs every round (the rfreq
        // reduction below needs the whole wave); lanes past nsel carry h = 0
        for (uint32_t gb = 0; gb < nsel; gb += T32) {
            const uint32_t g = gb + (uint32_t)tid;
            const bool valid = g < nsel;
            const uint4 h0 = n0, h1 = n1;
            if (g + T32 < nsel) { n0 = hist[2 * (g + T32)]; n1 = hist[2 * (g + T32) + 1]; }   // prefetch
            const uint32_t h[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
            // cost of the group under table t = sum_v count_v * len_t[v]: byte
            // counts (<= 50) and lengths (<= 17) packed 4 per word, one
            // v_dot4_u32_u8 per 4 symbols; first minimum wins (bz:compress.c:399-401)
            int bt = 0;
            uint32_t bc = ~0u;
#pragma unroll
            for (int t = 0; t < 6; ++t) {
                if (t < ng) {
                    uint32_t ct = 0;
#pragma unroll
                    for (int q = 0; q < 8; ++q)
                        if (4 * q < alpha) ct = __builtin_amdgcn_udot4(h[q], pl4[t][q], ct, false);
                    if (ct < bc) { bc = ct; bt = t; }
                }
            }
            if (valid) sel_l[g] = (uint8_t)bt;
            // rfreq: once per distinct table chosen in this wave, sum the lanes'
            // byte histograms as u16 pairs (<= 64 x 50 per field) into the
            // wave's private rows -- no same-address LDS atomics (a wave's 64
            // groups mostly pick one or two tables), summed over the wave by
            // wave_sum_u8x32; its 8 result lanes add them to the wave's rows
            uint32_t rem = valid ? (uint32_t)bt : 7u;
            for (;;) {
                const uint64_t act = __ballot(rem != 7u);
                if (!act) break;
                const uint32_t t = (uint32_t)__builtin_amdgcn_readlane((int)rem, (int)(__ffsll((long long)act) - 1));
                const bool mine = rem == t;
                uint32_t ev, od, q;
                wave_sum_u8x32(h, mine, lane, ev, od, q);
                if ((lane & 7) == 7) {
                    rf[wid][t][4 * q] += ev & 0xffffu;
                    rf[wid][t][4 * q + 1] += od & 0xffffu;
                    rf[wid][t][4 * q + 2] += ev >> 16;
                    rf[wid][t][4 * q + 3] += od >> 16;
                }
                if (mine) rem = 7u;
            }
        }
        __syncthreads();
        TPROF(1);
        if (tid < 6 * 32) {
            const int t = tid >> 5, v = tid & 31;
            uint32_t a = 0;
            for (int w = 0; w < NW32; ++w) a += rf[w][t][v];
            if (v < alpha) rfreq[t][v] = a;
        }
        __syncthreads();
        for (int t = wid; t < ng; t += NW32) hb_make_lengths_wave(len[t], rfreq[t], alpha, 17);
        __syncthreads();
        TPROF(2);
    }
    for (uint32_t g = tid; g < nsel; g += T32) sel[g] = sel_l[g];
    // selector MTF (bz:compress.c:461-478): contiguous ranges per thread, start
    // lists by a scan of the recency-list composition (as in k_mtf_nib)
    {
        const uint32_t per = (nsel + T32 - 1) / T32;
        const uint32_t a = tid * per, e = a + per < nsel ? a + per : nsel;
        NibState loc;
        loc.list = 0; loc.set = 0; loc.cnt = 0;
        for (uint32_t i = e; i > a; --i) {
            const uint32_t sv = sel_l[i - 1];
            if (!((loc.set >> sv) & 1u)) { loc.set |= 1u << sv; loc.list |= (uint64_t)sv << (4 * loc.cnt); ++loc.cnt; }
        }
        nst[tid] = loc;
        __syncthreads();
        for (int d = 1; d < T32; d <<= 1) {
            NibState v = (tid >= d) ? nib_compose(nst[tid - d], nst[tid]) : nst[tid];
            __syncthreads();
            nst[tid] = v;
            __syncthreads();
        }
        NibState ident;
        ident.list = 0x543210ull & lowmask4((uint32_t)ng);
        ident.set = (1u << ng) - 1u;
        ident.cnt = (uint32_t)ng;
        uint64_t L = (tid ? nib_compose(ident, nst[tid - 1]) : ident).list;
        uint64_t sb = 0;
        for (uint32_t i = a; i < e; ++i) {
            const uint32_t j = nib_mtf(L, sel_l[i]);
            selmtf[i] = (uint8_t)j;
            sb += j + 1;
        }
        sb = wave_reduce_add(sb);
        if (tid == 0) sbits_sh = 0;
        __syncthreads();
        if (lane == 0) atomicAdd(&sbits_sh, (unsigned long long)sb);
        __syncthreads();
    }
    TPROF(3);
    if (wid == 0) {   // header bits: the tables' delta-coded lengths summed across lanes
        const uint64_t sbits = sbits_sh;
        uint32_t used16 = 0;
        for (int i = 0; i < 16; ++i) {
            uint32_t w = blocks[b].in_use[i >> 1];
            uint32_t half = (i & 1) ? (w >> 16) : (w & 0xffffu);
            if (half) ++used16;
        }
        uint32_t tb = 0;
        for (int t = 0; t < ng; ++t) {
            const int32_t l = lane < alpha ? (int32_t)len[t][lane] : 0;
            const int32_t pv = lane == 0 ? l : (lane < alpha ? (int32_t)len[t][lane - 1] : 0);
            const int32_t d = l - pv;
            tb += lane < alpha ? 1u + 2u * (uint32_t)(d < 0 ? -d : d) : 0u;
        }
        const uint64_t tbits = 5ull * (uint64_t)ng + wave_reduce_add(tb);
        if (lane == 0) {
            hdr_bits = 48 + 32 + 1 + 24 + 16 + 16ull * used16 + 3 + 15 + sbits + tbits;
            blocks[b].hdr_bits = (uint32_t)hdr_bits;
        }
    }
    // canonical codes (bz:huffman.c:152-166): for each length in increasing
    // order the symbols of that length take consecutive codes in symbol order
    // -- a ballot per length, the rank inside it by popcount
    for (int t = wid; t < ng; t += NW32) {
        const bool in = lane < alpha;
        const int32_t l = in ? (int32_t)len[t][lane] : 0;
        const uint64_t lt = (1ull << lane) - 1ull;
        uint32_t base = 0, code = 0;
        for (int32_t L = 1; L <= 17; ++L) {
            const uint64_t m = __ballot(in && l == L);
            if (in && l == L) code = base + (uint32_t)__popcll(m & lt);
            base = (base + (uint32_t)__popcll(m)) << 1;
        }
        if (in) {
            tabs[b].code[t][lane] = code;
            tabs[b].len[t][lane] = (uint8_t)l;
        }
    }
    __syncthreads();
    TPROF(4);
    // data bits per group with the final tables
    uint64_t local = 0;
    for (uint32_t g = tid; g < nsel; g += T32) {
        const uint4 h0 = hist[2 * g], h1 = hist[2 * g + 1];
        const uint32_t h[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
        const uint8_t* L = len[sel_l[g]];
        uint32_t bits = 0;
#pragma unroll
        for (int v = 0; v < 32; ++v) if (v < alpha) bits += byte_of(h, v) * L[v];
        gbits[g] = bits;
        local += bits;
    }
    local = wave_reduce_add(local);
    if (lane == 0) atomicAdd(&hdr_bits, (unsigned long long)local);
    __syncthreads();
    TPROF(5);
    if (tid == 0) {
        blocks[b].bits = hdr_bits;
        blocks[b].n_groups = (uint32_t)ng;
        blocks[b].n_sel = nsel;
    }
}

void launch_tables(BlockDesc* blocks, uint32_t b0, uint32_t nb, const uint16_t* mtfv, uint64_t mtf_stride,
                   Tables* tabs, uint8_t* sel, uint32_t* gbits, const BwtScratch& scr, hipStream_t st, uint32_t need)
{
    // per-group histograms live in the (now free) block-sort key scratch
    uint8_t* hist = reinterpret_cast<uint8_t*>(scr.K);
    const uint64_t hist_stride = scr.stride * sizeof(uint64_t);
#ifndef STARCH_TABLES_WIDE_NB
#define STARCH_TABLES_WIDE_NB 512
#endif
    // STARCH_TABLES_T=256 / 512 / 1024 forces the workgroup size (experiments)
    static const int t_force = [] { const char* e = getenv("STARCH_TABLES_T"); return e ? atoi(e) : 0; }();
    const int t32 = t_force == 256 || t_force == 512 || t_force == 1024 ? t_force : (nb < STARCH_TABLES_WIDE_NB ? 1024 : 256);
    if (!(need & (kMtfNib | kMtfByte3 | kMtfByte4))) {
        // no block of <= 30 symbols in the batch: k_tables32 has nothing to do
    } else if (t32 == 1024)
        hipLaunchKernelGGL(k_tables32<1024>, dim3(nb), dim3(1024), 0, st, blocks, b0, mtfv, mtf_stride, tabs, sel, gbits,
                           reinterpret_cast<uint4*>(scr.K), hist_stride / sizeof(uint4));
    else if (t32 == 512)
        hipLaunchKernelGGL(k_tables32<512>, dim3(nb), dim3(512), 0, st, blocks, b0, mtfv, mtf_stride, tabs, sel, gbits,
                           reinterpret_cast<uint4*>(scr.K), hist_stride / sizeof(uint4));
    else
        hipLaunchKernelGGL(k_tables32<256>, dim3(nb), dim3(256), 0, st, blocks, b0, mtfv, mtf_stride, tabs, sel, gbits,
                           reinterpret_cast<uint4*>(scr.K), hist_stride / sizeof(uint4));
    if (need & kMtfBig)
        hipLaunchKernelGGL(k_tables, dim3(nb), dim3(TT), 0, st, blocks, b0, mtfv, mtf_stride, tabs, sel, gbits, hist,
                           hist_stride);
    HIP_CHECK(hipGetLastError());
#ifdef STARCH_TABLES_PROF
    {
        unsigned long long h[8];
        HIP_CHECK(hipStreamSynchronize(st));
        HIP_CHECK(hipMemcpyFromSymbol(h, HIP_SYMBOL(g_tprof), sizeof(h)));
        static const unsigned long long zero[8] = {};
        HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_tprof), zero, sizeof(zero)));
        const char* nm[6] = {"hist+bands", "iter:cost+rfreq", "iter:heap", "selmtf", "hdr+codes", "gbits"};
        for (int q = 0; q < 6; ++q) fprintf(stderr, "[tprof] nb %u %-16s %.1f us/block\n", nb, nm[q], h[q] / 100.0 / nb);
    }
#endif
}

}  // namespace bz
