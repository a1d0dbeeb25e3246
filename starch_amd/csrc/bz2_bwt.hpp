// starch_amd/csrc/bz2_bwt.hpp -- block-sort scratch (per batch slot, HBM).
#pragma once
#include "bz2_int.hpp"

namespace bz {

struct BwtScratch {            // 40 (+18 with bwt_kmat) bytes per rotation per batch slot
    uint64_t* K;
    uint64_t* K2;
    uint64_t* KM0;             // round 0 (bwt3, bwt_kmat() only, else null): every rotation's key window next to SA, and the
    uint64_t* KM1;             //   partition ping-pong copy (no key gathers in the round-0 sorts)
    uint8_t* LS0;              // round 0: the rotation's last-column symbol next to SA, ping-pong
    uint8_t* LS1;
    uint32_t* V;
    uint32_t* V2;
    uint32_t* SA;              // sorted rotation order (ptr[] of bz:blocksort.c)
    uint32_t* RK;
    uint32_t* U;
    uint32_t* U2;
    uint8_t* LL;               // last column bytes, sorted order (block[(ptr[i]-1) mod n])
    uint64_t stride;           // elements per slot
};

// STARCH_KMAT=1: round 0 materialises keys + last symbols next to SA (measured
// slower on cfg2: 25.9 vs 23.7 ms, the extra 18 B/rotation of writes cost more
// than the gathers they save); the encoder allocates KM0..LS1 only when set
bool bwt_kmat();
bool bwt_kgather();
void launch_bwt(BlockDesc* blocks, uint32_t b0, uint32_t nb, const uint8_t* blkbytes, uint64_t stride,
                const BwtScratch& scr, unsigned long long* stats, hipStream_t st);
// v3 (default): batch-wide segmented sort + doubling on ties (bz2_bwt3.hip).
// hctr: pinned host memory of >= 16 u32; stats[0..2] += rounds, periodic, tied rotations.
// Returns false when no block needed prefix doubling (then none is periodic).
bool launch_bwt3(BlockDesc* blocks, uint32_t b0, uint32_t nb, const uint8_t* blkbytes, uint64_t stride,
                 const BwtScratch& scr, DevBuf& meta, uint32_t* hctr, unsigned long long* stats, hipStream_t st,
                 bool wide = false);   // wide: some block has 17..20 symbols (8192-bin mixed-radix top digit)
// periodic blocks: bzip2's exact fallbackSort tie order (bz:blocksort.c:211-329),
// round by round on the GPU; which_host / n_host: batch slots and block sizes;
// hctr: pinned host memory (>= 2 u32)
void launch_fallback(BlockDesc* blocks, uint32_t b0, const uint32_t* which_host, const uint32_t* n_host,
                     uint32_t nwhich, const uint8_t* blkbytes, uint64_t stride, const BwtScratch& scr, FbPool& pool,
                     hipStream_t st);
// last column for blocks whose SA was produced elsewhere (fallback / LSD path)
void launch_last_col(const BlockDesc* blocks, uint32_t b0, const uint32_t* which, uint32_t nwhich,
                     const uint8_t* blkbytes, uint64_t stride, const BwtScratch& scr, hipStream_t st);
// alphabet classes of a batch (nInUse 1..16 / 17..24 / 25..30 / > 30): the
// MTF and table kernels of a class are launched only when a block needs them
constexpr uint32_t kMtfNib = 1, kMtfByte3 = 2, kMtfByte4 = 4, kMtfBig = 8, kMtfAll = 15;
inline uint32_t mtf_class(uint32_t nin)
{
    return nin <= 16 ? kMtfNib : nin <= 24 ? kMtfByte3 : nin <= 30 ? kMtfByte4 : kMtfBig;
}
void launch_mtf(BlockDesc* blocks, uint32_t b0, uint32_t nb, const uint8_t* blkbytes, uint64_t stride,
                const BwtScratch& scr, uint16_t* mtfv, uint64_t mtf_stride, Tables* tabs, hipStream_t st,
                uint32_t need = kMtfAll);
void launch_tables(BlockDesc* blocks, uint32_t b0, uint32_t nb, const uint16_t* mtfv, uint64_t mtf_stride,
                   Tables* tabs, uint8_t* sel, uint32_t* gbits, const BwtScratch& scr, hipStream_t st, uint32_t need = kMtfAll);
// src_of (nullable): block b's MTF values / tables / selectors / group sizes
// live at data index src_of[b] (exact block reuse, bz2_dedupe.hip); gpre has
// one kMaxSelectors row per block.
void launch_emit_blocks(const BlockDesc* blocks, uint32_t nb, const uint16_t* mtfv, uint64_t mtf_stride,
                        const Tables* tabs, const uint8_t* sel, const uint32_t* gbits, uint32_t* gpre,
                        const uint32_t* src_of, uint32_t* out32, hipStream_t st);
// exact block reuse (bz2_dedupe.hip)
void launch_block_equal(const uint8_t* blkbytes, uint64_t stride, const uint32_t* pairs, uint32_t npairs,
                        const BlockDesc* blocks, uint32_t* mismatch, hipStream_t st);
void launch_gather_blocks(const uint8_t* src, uint64_t stride, const uint32_t* idx, uint32_t n, uint8_t* dst,
                          hipStream_t st);
void launch_stream_frame(const StreamOut* souts, const BlockDesc* blocks, uint32_t nstreams, int bs100k,
                         uint64_t out_base, uint32_t* out32, hipStream_t st);

}  // namespace bz
