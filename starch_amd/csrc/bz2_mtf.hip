// starch_amd/csrc/bz2_mtf.hip -- last column, move-to-front and RUNA/RUNB
// coding on MI355X (restates makeMaps_e + generateMTFValues,
// bz:compress.c:105-231).
//
// One 1024-thread workgroup per block, the block split into C contiguous
// chunks.  MTF is made parallel by the chunk decomposition
//     state(c+1) = local(c) ++ (state(c) \ local(c)),
// where local(c) lists chunk c's symbols by last occurrence (most recent
// first).  The map L -> local ++ (L \ local) composes associatively, so every
// chunk's start state is an exclusive scan over chunks.  Alphabets of <= 16
// symbols (BED3 transforms) keep the whole list as 16 nibbles of a u64 in a
// register (C = 1024 chunks): finding a symbol is a SWAR zero-nibble search
// and the move-to-front is three masks and a shift.  Larger alphabets use
// byte lists in LDS (C = 256).  The zero runs of the index stream are then
// coded in bijective base 2 (RUNA = 0, RUNB = 1); a run may span chunks, so
// per-chunk (leading zeros, trailing zeros, all-zero, interior symbols)
// summaries are scanned once to place every chunk's output.
#include "bz2_bwt.hpp"

namespace bz {

constexpr int MT = 1024;
constexpr int NCH_BIG = 256;

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

__device__ __forceinline__ uint32_t nsym_run(uint32_t z) { return z ? (31 - __clz(z + 1)) : 0; }

struct ChunkSum {
    uint32_t lz, tz, len, inner;   // leading/trailing zero counts, length, output symbols after the first non-zero
    uint32_t has_nz;
    uint32_t zin;                  // zeros entering the chunk (filled by the scan)
    uint32_t out;                  // output offset (filled by the scan)
    uint32_t pad;
};

// NIB: alphabets <= 16 (register nibble lists); !NIB: byte lists in LDS.  A
// block is handled by exactly one of the two instantiations.
template <bool NIB>
__global__ void __launch_bounds__(MT) k_mtf(BlockDesc* __restrict__ blocks, uint32_t b0,
                                             const uint8_t* __restrict__ blkbytes, uint64_t stride, BwtScratch scr,
                                             uint16_t* __restrict__ mtfv_all, uint64_t mtf_stride,
                                             Tables* __restrict__ tabs)
{
    constexpr uint32_t C = NIB ? MT : NCH_BIG;
    constexpr int NF = 4;                      // frequency histogram copies
    __shared__ ChunkSum cs_sh[C];
    __shared__ uint8_t seq[256];
    __shared__ uint32_t freq[NF][258];
    __shared__ uint32_t scan_sh[MT / 64 + 1];
    __shared__ uint32_t tail[2];

    const int tid = threadIdx.x;
    const uint32_t slot = blockIdx.x;
    const uint32_t b = b0 + slot;
    const uint32_t n = blocks[b].n;
    const uint8_t* blk = blkbytes + (uint64_t)b * stride;
    const uint64_t so = slot * scr.stride;
    const uint32_t* SA = scr.SA + so;
    uint8_t* ll = reinterpret_cast<uint8_t*>(scr.K + so);
    uint8_t* idx = reinterpret_cast<uint8_t*>(scr.K2 + so);
    uint8_t* locl = reinterpret_cast<uint8_t*>(scr.V2 + so);
    uint8_t* sstate = reinterpret_cast<uint8_t*>(scr.U2 + so);
    uint16_t* mtfv = mtfv_all + (uint64_t)b * mtf_stride;

    if (tid < 256) {   // makeMaps_e: unseqToSeq
        uint32_t c = tid;
        uint32_t below = 0;
        for (uint32_t j = 0; j < (c >> 5); ++j) below += __popc(blocks[b].in_use[j]);
        below += __popc(blocks[b].in_use[c >> 5] & ((1u << (c & 31)) - 1u));
        seq[c] = (uint8_t)below;
    }
    for (int i = tid; i < NF * 258; i += MT) (&freq[0][0])[i] = 0;
    const uint32_t nin = blocks[b].n_in_use;
    if (NIB != (nin <= 16)) return;            // uniform per workgroup
    __syncthreads();
    for (uint32_t j = tid; j < n; j += MT) {   // last column (bz:compress.c:166-168)
        uint32_t p = SA[j];
        p = p ? p - 1 : n - 1;
        ll[j] = seq[blk[p]];
    }
    __syncthreads();

    // chunks are 16-byte aligned so every lane moves its bytes with 16-B loads
    const uint32_t csz = ((n + C - 1) / C + 15u) & ~15u;
    const uint32_t a = tid * csz;
    uint32_t e = a + csz;
    if (e > n) e = n;
    const bool mine = (uint32_t)tid < C && a < e;

    if constexpr (NIB) {
        __shared__ NibState nst[MT];
        // local recency list of this chunk
        NibState loc;
        loc.list = 0; loc.set = 0; loc.cnt = 0;
        if (mine) {
            for (uint32_t j0 = a + ((e - a - 1) & ~15u);; j0 -= 16) {
                const uint4 v = *reinterpret_cast<const uint4*>(ll + j0);
                const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int k = 15; k >= 0; --k) {
                    if (j0 + k < e) {
                        uint32_t s = (w[k >> 2] >> (8 * (k & 3))) & 0xffu;
                        if (!((loc.set >> s) & 1u)) {
                            loc.set |= 1u << s;
                            loc.list |= (uint64_t)s << (4 * loc.cnt);
                            ++loc.cnt;
                        }
                    }
                }
                if (j0 == a) break;
            }
        }
        nst[tid] = loc;
        __syncthreads();
        for (int d = 1; d < MT; d <<= 1) {      // inclusive scan of the composition
            NibState v = (tid >= d) ? nib_compose(nst[tid - d], nst[tid]) : nst[tid];
            __syncthreads();
            nst[tid] = v;
            __syncthreads();
        }
        // start state = (exclusive prefix) applied to the identity list 0..nin-1
        NibState ident;
        ident.list = 0;
        for (uint32_t i = 0; i < nin; ++i) ident.list |= (uint64_t)i << (4 * i);
        ident.set = nin >= 32 ? 0xffffffffu : ((1u << nin) - 1u);
        ident.cnt = nin;
        NibState pre = tid ? nib_compose(ident, nst[tid - 1]) : ident;
        uint64_t L = pre.list;
        ChunkSum cs;
        cs.lz = 0; cs.tz = 0; cs.len = e > a ? e - a : 0; cs.inner = 0; cs.has_nz = 0; cs.zin = 0; cs.out = 0;
        if (mine) {
            uint32_t z = 0;
            for (uint32_t j0 = a; j0 < e; j0 += 16) {
                const uint4 v = *reinterpret_cast<const uint4*>(ll + j0);
                const uint32_t w[4] = {v.x, v.y, v.z, v.w};
                uint32_t o[4] = {0, 0, 0, 0};
#pragma unroll
                for (int q = 0; q < 16; ++q) {
                    if (j0 + q < e) {
                        const uint32_t s = (w[q >> 2] >> (8 * (q & 3))) & 0xffu;
                        const uint64_t x = L ^ (0x1111111111111111ull * s);
                        const uint64_t t = x | (x >> 1) | (x >> 2) | (x >> 3);
                        const uint64_t zn = ~t & 0x1111111111111111ull;
                        const uint32_t k = (uint32_t)__builtin_ctzll(zn) >> 2;
                        L = (L & ~lowmask4(k + 1)) | ((L & lowmask4(k)) << 4) | (uint64_t)s;
                        o[q >> 2] |= k << (8 * (q & 3));
                        if (k == 0) {
                            ++z;
                        } else {
                            if (!cs.has_nz) { cs.lz = z; cs.has_nz = 1; } else { cs.inner += 1 + nsym_run(z); }
                            z = 0;
                        }
                    }
                }
                *reinterpret_cast<uint4*>(idx + j0) = make_uint4(o[0], o[1], o[2], o[3]);
            }
            if (!cs.has_nz) cs.lz = z;
            cs.tz = z;
        }
        if ((uint32_t)tid < C) cs_sh[tid] = cs;
    } else {
        // ---- alphabets > 16: byte lists in LDS, 256 chunks ----
        __shared__ uint8_t lst[256 * NCH_BIG];   // [pos][chunk]
        __shared__ uint32_t seen[NCH_BIG][8];
        __shared__ uint8_t st[256], st2[256], fl[256];
        __shared__ uint32_t lcnt[NCH_BIG];
        if (tid < NCH_BIG) for (int j = 0; j < 8; ++j) seen[tid][j] = 0;
        __syncthreads();
        if ((uint32_t)tid < C) {
            uint32_t cnt = 0;
            uint8_t* out = locl + (uint64_t)tid * 256;
            for (uint32_t j = e; j > a && a < e; --j) {
                uint32_t s = ll[j - 1];
                uint32_t bit = 1u << (s & 31);
                if (!(seen[tid][s >> 5] & bit)) { seen[tid][s >> 5] |= bit; out[cnt++] = (uint8_t)s; }
            }
            lcnt[tid] = cnt;
        }
        if (tid < 256) { st[tid] = (uint8_t)tid; fl[tid] = 0; }
        __syncthreads();
        for (uint32_t c = 0; c < C; ++c) {   // list state at each chunk start (sequential)
            const uint32_t cnt = lcnt[c];
            const uint8_t* lc = locl + (uint64_t)c * 256;
            if (tid < (int)nin) sstate[(uint64_t)c * 256 + tid] = st[tid];
            if (tid < (int)cnt) fl[lc[tid]] = 1;
            __syncthreads();
            uint32_t keep = (tid < (int)nin && !fl[st[tid]]) ? 1u : 0u;
            uint32_t pre = block_excl_scan_add<uint32_t>(keep, scan_sh, (uint32_t*)nullptr);
            if (keep) st2[cnt + pre] = st[tid];
            if (tid < (int)cnt) st2[tid] = lc[tid];
            __syncthreads();
            if (tid < (int)nin) st[tid] = st2[tid];
            if (tid < (int)cnt) fl[lc[tid]] = 0;
            __syncthreads();
        }
        ChunkSum cs;
        cs.lz = 0; cs.tz = 0; cs.len = e > a ? e - a : 0; cs.inner = 0; cs.has_nz = 0; cs.zin = 0; cs.out = 0;
        if (mine) {
            for (uint32_t k = 0; k < nin; ++k) lst[k * NCH_BIG + tid] = sstate[(uint64_t)tid * 256 + k];
            uint32_t z = 0;
            for (uint32_t j = a; j < e; ++j) {
                uint8_t s = ll[j];
                uint8_t cur = lst[tid];
                uint32_t k = 0;
                if (cur != s) {   // bz:compress.c:197-211
                    uint8_t carry_v = cur;
                    k = 1;
                    for (;;) {
                        uint8_t nxt = lst[k * NCH_BIG + tid];
                        lst[k * NCH_BIG + tid] = carry_v;
                        if (nxt == s || k >= 255) break;
                        carry_v = nxt;
                        ++k;
                    }
                    lst[tid] = s;
                }
                idx[j] = (uint8_t)k;
                if (k == 0) { ++z; continue; }
                if (!cs.has_nz) { cs.lz = z; cs.has_nz = 1; } else { cs.inner += 1 + nsym_run(z); }
                z = 0;
            }
            if (!cs.has_nz) cs.lz = z;
            cs.tz = z;
        }
        if ((uint32_t)tid < C) cs_sh[tid] = cs;
    }
    __syncthreads();
    // ---- place every chunk's output: zeros entering each chunk, output offsets ----
    if (tid == 0) {
        uint32_t zin = 0, out = 0;
        for (uint32_t c = 0; c < C; ++c) {
            ChunkSum& s = cs_sh[c];
            s.zin = zin;
            s.out = out;
            if (s.has_nz) {
                out += 1 + nsym_run(zin + s.lz) + s.inner;
                zin = s.tz;
            } else {
                zin += s.len;
            }
        }
        tail[0] = zin;     // zeros after the last non-zero
        tail[1] = out;
    }
    __syncthreads();
    const int wv = (tid >> 6) & (NF - 1);
    if (mine) {
        const ChunkSum cs = cs_sh[tid];
        uint32_t o = cs.out;
        uint32_t z = cs.zin;
        for (uint32_t j0 = a; j0 < e; j0 += 16) {
            const uint4 vv = *reinterpret_cast<const uint4*>(idx + j0);
            const uint64_t lo = ((uint64_t)vv.y << 32) | vv.x, hi = ((uint64_t)vv.w << 32) | vv.z;
            const uint32_t qn = (e - j0) < 16u ? (e - j0) : 16u;
            for (uint32_t q = 0; q < qn; ++q) {
                const uint32_t v = (uint32_t)((q < 8 ? (lo >> (8 * q)) : (hi >> (8 * (q - 8)))) & 0xffu);
                if (v == 0) { ++z; continue; }
                while (z) {
                    uint32_t d = ((z - 1) & 1u) ? 1u : 0u;       // RUNB : RUNA
                    mtfv[o++] = (uint16_t)d;
                    atomicAdd(&freq[wv][d], 1u);
                    z = (z - (d + 1)) >> 1;
                }
                mtfv[o++] = (uint16_t)(v + 1);
                atomicAdd(&freq[wv][v + 1], 1u);
            }
        }
    }
    __syncthreads();
    if (tid == 0) {
        uint32_t z = tail[0], o = tail[1];
        while (z) {
            uint32_t d = ((z - 1) & 1u) ? 1u : 0u;
            mtfv[o++] = (uint16_t)d;
            freq[0][d]++;
            z = (z - (d + 1)) >> 1;
        }
        mtfv[o++] = (uint16_t)(nin + 1);      // EOB
        freq[0][nin + 1]++;
        blocks[b].n_mtf = o;
    }
    __syncthreads();
    if (tid < 258) {
        uint32_t f = 0;
        for (int w = 0; w < NF; ++w) f += freq[w][tid];
        tabs[b].freq[tid] = f;
    }
}

void launch_mtf(BlockDesc* blocks, uint32_t b0, uint32_t nb, const uint8_t* blkbytes, uint64_t stride,
                const BwtScratch& scr, uint16_t* mtfv, uint64_t mtf_stride, Tables* tabs, hipStream_t st)
{
    hipLaunchKernelGGL(k_mtf<true>, dim3(nb), dim3(MT), 0, st, blocks, b0, blkbytes, stride, scr, mtfv, mtf_stride,
                       tabs);
    hipLaunchKernelGGL(k_mtf<false>, dim3(nb), dim3(MT), 0, st, blocks, b0, blkbytes, stride, scr, mtfv, mtf_stride,
                       tabs);
    HIP_CHECK(hipGetLastError());
}

}  // namespace bz
