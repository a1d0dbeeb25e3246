// starch_amd/csrc/bz2_decode.hpp -- host interface of the GPU bzip2 decoder
// (decompression / unstarch round trip).
#pragma once
#include "bz2.hpp"

namespace bz {

struct DecStream {            // one bzip2 stream of the input, as decoded
    uint64_t in_beg, in_end;  // its bytes in the input
    uint64_t out_off, out_len;
    uint32_t level;           // blockSize100k from its "BZh" header
    uint32_t n_blocks;
    uint32_t stored_crc;      // combined CRC from its end-of-stream trailer
    uint32_t combined_crc;    // recomputed from the decoded blocks
};

class Decoder {
public:
    // Decode every bzip2 stream of in[0, n) (device bytes, 16-byte aligned,
    // >= 64 readable bytes after n); h_in: the same bytes on the host, or
    // null (headers/trailers are then copied from the device as needed).
    // Output: the streams' decompressed bytes back to back in `out`.
    // Throws StarchError(STARCH_ERR_DATA-like -12) on malformed input or any
    // block / stream CRC mismatch.
    uint64_t decode(const uint8_t* d_in, uint64_t n, const uint8_t* h_in, hipStream_t st, DevBuf& out,
                    std::vector<DecStream>& streams);

private:
    DevBuf b_hits, b_cnt, b_blocks, b_ll, b_tt, b_rle, b_meta, b_bd, b_crc;
};

}  // namespace bz
