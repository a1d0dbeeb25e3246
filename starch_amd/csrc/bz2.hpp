// starch_amd/csrc/bz2.hpp -- host interface of the GPU bzip2 block pipeline.
//
// One bzip2 stream per input segment (a chromosome's transformed text, or a
// raw byte range for the bzlib ABI).  Byte-exact with bzip2-1.0.6
// BZ2_bzCompress(..., BZ_FINISH) at blockSize100k = 1..9 (the reference's
// vendored libbz2, third-party/bzip2-1.0.6.tar.gz).
#pragma once
#include "common.hpp"
#include <vector>

namespace bz {

constexpr int kMaxSelectors = 18002 + 8;   // BZ_MAX_SELECTORS (bz:bzlib_private.h:125)

struct StreamIn {          // one RLE1 piece: a stream, or the part of a stream between BZ_FLUSHes
    uint64_t text_off;     // offset of its bytes in the device text buffer
    uint64_t text_len;
    uint32_t final_run_joins;  // 1: its last byte arrived with the FLUSH/FINISH call (bz:bzlib.c:393-397)
    uint32_t group;        // output stream it belongs to (pieces of a stream are consecutive)
    // a stream encoded in pieces (streaming ingestion inside a chromosome):
    // all zero for a whole stream.  cont: not the stream's first piece (no
    // header; its bits start at bit `phase` of the first output byte, the
    // bits before belong to the previous piece).  open: the stream goes on
    // after this piece: its last, incomplete block is not encoded (its text
    // from Encoder::open_rest() on goes first in the next piece; a block
    // starts a fresh RLE1 run, bz:bzlib.c:266-280) and no trailer is written.
    // comb_in: combined CRC of the blocks before this piece.  Only the last
    // piece of a call may be open.
    uint32_t cont, open, phase, comb_in;
};

struct BlockDesc {         // one bzip2 block (bz:compress.c:602-667)
    uint64_t in_beg, in_end;   // text bytes covered (pre-RLE1)
    uint64_t w_beg;            // stream-relative RLE1 size before in_beg
    uint64_t bits;             // bits this block contributes (header + tables + data)
    uint64_t bit_off;          // absolute bit offset of the block in the output buffer
    uint32_t stream;           // index into StreamIn
    uint32_t n;                // nblock (RLE1 bytes)
    uint32_t crc;              // finalised blockCRC
    uint32_t orig_ptr;
    uint32_t n_in_use;
    uint32_t n_mtf;
    uint32_t flags;            // bit0: periodic (tie order from exact fallbackSort)
    uint32_t n_groups, n_sel;
    uint32_t in_use[8];        // 256-bit inUse map
    uint32_t hdr_bits;         // bits before the coded data (block header, map, selectors, tables)
    uint32_t pad;
};

struct StreamOut {
    uint64_t out_off;          // byte offset of the stream in the output buffer
    uint64_t bytes;            // stream length in bytes (a piece: its bytes, the last one partial unless closed)
    uint32_t first_block, n_blocks;
    uint32_t combined_crc;     // (emit: the CRC entering the piece; after emit: over all blocks so far)
    uint32_t frame;            // bit 0: header, bit 1: trailer, bits 8..10: phase (see StreamIn)
    uint64_t block_bits;       // bits of the blocks alone (no header, trailer or padding)
};

struct Stats {                 // per-stage device timings (ms) from HIP events
    float rle = 0, bwt = 0, mtf = 0, tables = 0, emit = 0;
    uint64_t n_blocks = 0, rle_bytes = 0, bwt_rounds = 0, periodic_blocks = 0, bwt_tied = 0;
    uint64_t dedup_blocks = 0;     // blocks that reused a byte-identical block's results
};

// Every periodic block of a batch replays at once: one HIP stream per block
// (from the pool, round-robin), each block's round issued on its stream, one
// host read-back per round for all of them.
struct FbPool {
    static constexpr int kStreams = 8;
    hipStream_t st[kStreams] = {};
    hipEvent_t ev[kStreams + 1] = {};
    DevBuf tmp[kStreams];          // scan scratch per stream
    PinnedBuf ctr;                 // per block: not-done, mixed-bucket count
    int dev = -1;
    void init(int device);
    ~FbPool();
};
class Encoder {
public:
    // Compress `streams` whose bytes live in d_text (device).  The result is
    // written to d_out (device) at out_base: stream k at out_base +
    // outs[k].out_off, streams back to back.  Capacity is checked.  Returns
    // the total number of bytes written after out_base.
    uint64_t plan_and_encode(const uint8_t* d_text, const std::vector<StreamIn>& streams, int bs100k,
                             uint8_t* d_out, uint64_t out_cap, uint64_t out_base, std::vector<StreamOut>& outs,
                             hipStream_t st, Stats* stats = nullptr);
    // Two-phase form used by the archive writer: plan() computes stream sizes;
    // emit() writes the bits once the caller has chosen out_base.
    void plan(const uint8_t* d_text, const std::vector<StreamIn>& streams, int bs100k, hipStream_t st,
              std::vector<StreamOut>& outs, Stats* stats = nullptr);
    void emit(uint8_t* d_out, uint64_t out_cap, uint64_t out_base, std::vector<StreamOut>& outs, hipStream_t st,
              Stats* stats = nullptr);
    // Bit length of the last code written for output stream g (its last
    // block's EOB symbol, bz:compress.c:580-593): libbz2 keeps the bits of its
    // last bsW call in its bit buffer when a block ends (bz:compress.c:37-52),
    // which decides how many bytes a BZ_FLUSH makes readable.  0: no blocks.
    uint32_t last_write_bits(uint32_t g, const StreamOut& so, hipStream_t st);
    // Per-block results of the last plan() + emit(), in block order: text
    // range (plan's d_text offsets), absolute bit offset and length in the
    // emitted buffer, block CRC, and the bit length of its last code (its
    // EOB: what libbz2's bit buffer keeps when the block ends).  One read-back.
    struct BlockOut {
        uint64_t in_beg, in_end, bit_off, bits;
        uint32_t crc, last_bits;
    };
    void block_results(std::vector<BlockOut>& out, hipStream_t st);
    // plan() and emit() record their stage timings as event pairs without
    // waiting on them; once the stream has synchronised, this adds them to
    // *stats (null: drops them).  plan() drops any left from an earlier call.
    void resolve_timers(Stats* stats);
    // the same timers as intervals, in ms after `ref` (an event recorded on a
    // stream before any of them), for a caller that merges several encoders'
    // stages; drops them
    struct Interval {
        int stage;
        float a, b;
    };
    void take_intervals(hipEvent_t ref, std::vector<Interval>& out);
    // free the device buffers (they grow again on the next plan); the caller
    // has synchronised the stream they were used on
    void release_device();
    // the part of the device's free memory plan() sizes its sort batches by
    // (1: all; encoder lanes planning concurrently take 1 / lanes each)
    void set_mem_share(double f) { mem_share_ = f > 0 && f <= 1 ? f : 1.0; }
    // text offset (in the plan's d_text) where an open last piece's unencoded
    // rest starts; its end is the piece's end
    uint64_t open_rest() const { return open_rest_; }
    struct PendTimer {
        hipEvent_t a, b;
        int stage;                 // 0 rle, 1 bwt, 2 mtf, 3 tables, 4 emit
    };

private:
    DevBuf b_streams, b_tiles, b_tile_sum, b_tile_carry, b_tile_w, b_tile_wpre, b_tile_block, b_cut_tab, b_seg_tile0, b_seg_nblk,
        b_blk_tmp, b_blk, b_blkbytes, b_scal, b_tmp, b_bwt, b_mtfv, b_freq, b_sel, b_tabs, b_gbits, b_souts,
        b_fallback, b_bwt3, b_crc, b_dedupe, b_rep_bytes, b_rep_blk, b_last;
    PinnedBuf h_wtot_, h_nblk_, h_blocks_, h_hr_, h_last_;
    FbPool fb_pool_;                        // periodic blocks' concurrent replays   // read-back targets (pinned)
    struct PinnedCtr {
        uint32_t* p = nullptr;
        uint32_t* get();
        ~PinnedCtr();
    } h_ctr_;
    const uint8_t* text_ = nullptr;
    int bs100k_ = 9;
    uint32_t nblocks_ = 0, nstreams_ = 0, ngroups_ = 0;
    uint64_t blk_stride_ = 0;
    uint64_t gpre_off_ = 0;                 // words: the per-block prefix rows in b_gbits
    const uint32_t* src_of_dev_ = nullptr;  // block -> data index (null: identity)
    std::vector<uint32_t> src_of_host_;     // the same on the host (empty: identity)
    std::vector<StreamIn> streams_;
    std::vector<BlockDesc> host_blocks_;
    std::vector<PendTimer> pend_;
    uint64_t open_rest_ = 0;
    double mem_share_ = 1.0;
};

}  // namespace bz
