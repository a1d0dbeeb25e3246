// starch_amd/csrc/bz2_mtf.hip -- last column, move-to-front and RUNA/RUNB
// coding on MI355X (restates makeMaps_e + generateMTFValues,
// bz:compress.c:105-231).
//
// One 1024-thread workgroup per block.  The MTF recurrence is made parallel
// by chunking: 256 chunks each record their local recency list (symbols by
// last occurrence); a short sequential pass composes the list state at every
// chunk start (state' = local list ++ state minus local list); then each
// chunk runs MTF from its own start state with its list in LDS (byte-
// interleaved by thread to spread banks).  Zero runs are then coded in
// bijective base 2 (RUNA=0, RUNB=1), positions from a workgroup scan, and
// symbol frequencies (mtfFreq) accumulated in LDS.
#include "bz2_bwt.hpp"

namespace bz {

constexpr int MT = 1024;
constexpr int NCH = 256;

__global__ void __launch_bounds__(MT) k_mtf(BlockDesc* __restrict__ blocks, uint32_t b0,
                                             const uint8_t* __restrict__ blkbytes, uint64_t stride, BwtScratch scr,
                                             uint16_t* __restrict__ mtfv_all, uint64_t mtf_stride,
                                             Tables* __restrict__ tabs)
{
    __shared__ uint8_t lst[256 * NCH];     // per-chunk MTF lists, [pos][chunk]
    __shared__ uint32_t seen[NCH][8];
    __shared__ uint8_t seq[256];
    __shared__ uint8_t st[256], nst[256], fl[256];
    __shared__ uint32_t lcnt[NCH];
    __shared__ uint32_t freq[258];
    __shared__ uint32_t scan_sh[MT / 64 + 1];
    __shared__ uint32_t mbuf[MT];
    __shared__ uint32_t carry[4];

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

    // makeMaps_e: unseqToSeq
    if (tid < 256) {
        uint32_t c = tid;
        uint32_t below = 0;
        for (uint32_t j = 0; j < (c >> 5); ++j) below += __popc(blocks[b].in_use[j]);
        below += __popc(blocks[b].in_use[c >> 5] & ((1u << (c & 31)) - 1u));
        seq[c] = (uint8_t)below;
    }
    if (tid < 258) freq[tid] = 0;
    if (tid < NCH) for (int j = 0; j < 8; ++j) seen[tid][j] = 0;
    __syncthreads();
    const uint32_t nin = blocks[b].n_in_use;
    // last column (bz:compress.c:166-168)
    for (uint32_t j = tid; j < n; j += MT) {
        uint32_t p = SA[j];
        p = p ? p - 1 : n - 1;
        ll[j] = seq[blk[p]];
    }
    __syncthreads();
    const uint32_t cs = (n + NCH - 1) / NCH;
    // phase 1: local recency lists
    if (tid < NCH) {
        uint32_t a = tid * cs, e = a + cs;
        if (e > n) e = n;
        uint32_t cnt = 0;
        uint8_t* out = locl + (uint64_t)tid * 256;
        for (uint32_t j = e; j > a; --j) {
            uint32_t s = ll[j - 1];
            uint32_t bit = 1u << (s & 31);
            if (!(seen[tid][s >> 5] & bit)) { seen[tid][s >> 5] |= bit; out[cnt++] = (uint8_t)s; }
        }
        lcnt[tid] = cnt;
    }
    if (tid < 256) { st[tid] = (uint8_t)tid; fl[tid] = 0; }
    __syncthreads();
    // phase 2: list state at each chunk start
    for (int c = 0; c < NCH; ++c) {
        const uint32_t cnt = lcnt[c];
        const uint8_t* lc = locl + (uint64_t)c * 256;
        if (tid < (int)nin) sstate[(uint64_t)c * 256 + tid] = st[tid];
        if (tid < (int)cnt) fl[lc[tid]] = 1;
        __syncthreads();
        uint32_t keep = (tid < (int)nin && !fl[st[tid]]) ? 1u : 0u;
        uint32_t pre = block_excl_scan_add<uint32_t>(keep, scan_sh, (uint32_t*)nullptr);
        if (keep) nst[cnt + pre] = st[tid];
        if (tid < (int)cnt) nst[tid] = lc[tid];
        __syncthreads();
        if (tid < (int)nin) st[tid] = nst[tid];
        if (tid < (int)cnt) fl[lc[tid]] = 0;
        __syncthreads();
    }
    // phase 3: MTF per chunk
    if (tid < NCH) {
        for (uint32_t k = 0; k < nin; ++k) lst[k * NCH + tid] = sstate[(uint64_t)tid * 256 + k];
        uint32_t a = tid * cs, e = a + cs;
        if (e > n) e = n;
        for (uint32_t j = a; j < e; ++j) {
            uint8_t s = ll[j];
            uint8_t cur = lst[tid];
            uint32_t k = 0;
            if (cur != s) {
                // shift right until s is found (bz:compress.c:197-211)
                uint8_t carry_v = cur;
                k = 1;
                for (;;) {
                    uint8_t nxt = lst[k * NCH + tid];
                    lst[k * NCH + tid] = carry_v;
                    if (nxt == s || k >= 255) break;   // k >= 255 cannot happen for a consistent list
                    carry_v = nxt;
                    ++k;
                }
                lst[tid] = s;
            }
            idx[j] = (uint8_t)k;
        }
    }
    __syncthreads();
    // phase 4: zero-run coding, EOB, frequencies
    if (tid == 0) { carry[0] = 0; carry[1] = 0; }
    __syncthreads();
    for (uint32_t t0 = 0; t0 < n; t0 += MT) {
        const uint32_t j = t0 + tid;
        const bool valid = j < n;
        const uint32_t v = valid ? idx[j] : 0;
        const bool nz = valid && v != 0;
        uint32_t M = block_incl_scan_max<uint32_t>(nz ? j + 1 : 0u, scan_sh);
        uint32_t cm = carry[0];
        M = M > cm ? M : cm;
        mbuf[tid] = M;
        __syncthreads();
        uint32_t L = tid ? mbuf[tid - 1] : cm;     // start of the zero run ending at j-1
        uint32_t z = nz ? j - L : 0;
        uint32_t nsym = z ? (31 - __clz(z + 1)) : 0;
        uint32_t c = nz ? nsym + 1 : 0;
        uint32_t tot;
        uint32_t pre = block_excl_scan_add<uint32_t>(c, scan_sh, &tot);
        if (nz) {
            uint32_t o = carry[1] + pre;
            while (z) {
                uint32_t d = ((z - 1) & 1u) ? 1u : 0u;       // RUNB : RUNA
                mtfv[o++] = (uint16_t)d;
                atomicAdd(&freq[d], 1u);
                z = (z - (d + 1)) >> 1;
            }
            mtfv[o] = (uint16_t)(v + 1);
            atomicAdd(&freq[v + 1], 1u);
        }
        __syncthreads();
        if (tid == MT - 1) { carry[0] = M; carry[1] += tot; }
        __syncthreads();
    }
    if (tid == 0) {
        uint32_t o = carry[1];
        uint32_t z = n - carry[0];
        while (z) {
            uint32_t d = ((z - 1) & 1u) ? 1u : 0u;
            mtfv[o++] = (uint16_t)d;
            freq[d]++;
            z = (z - (d + 1)) >> 1;
        }
        mtfv[o++] = (uint16_t)(nin + 1);      // EOB
        freq[nin + 1]++;
        blocks[b].n_mtf = o;
    }
    __syncthreads();
    if (tid < 258) tabs[b].freq[tid] = freq[tid];
}

void launch_mtf(BlockDesc* blocks, uint32_t b0, uint32_t nb, const uint8_t* blkbytes, uint64_t stride,
                const BwtScratch& scr, uint16_t* mtfv, uint64_t mtf_stride, Tables* tabs, hipStream_t st)
{
    hipLaunchKernelGGL(k_mtf, dim3(nb), dim3(MT), 0, st, blocks, b0, blkbytes, stride, scr, mtfv, mtf_stride, tabs);
    HIP_CHECK(hipGetLastError());
}

}  // namespace bz
