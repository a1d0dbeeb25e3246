// starch_amd/csrc/gz.hpp -- the gzip method (-g): one gzip member per segment,
// fixed-Huffman deflate built on the GPU (gz_deflate.hip).  Same two-phase
// shape as bz::Encoder: plan() sizes the members, emit() writes them.
#pragma once
#include "bz2.hpp"

namespace gz {

class Encoder {
public:
    void plan(const uint8_t* d_text, const std::vector<bz::StreamIn>& streams, hipStream_t st,
              std::vector<bz::StreamOut>& outs, bz::Stats* stats = nullptr);
    void emit(uint8_t* d_out, uint64_t out_cap, uint64_t out_base, std::vector<bz::StreamOut>& outs, hipStream_t st,
              bz::Stats* stats = nullptr);

private:
    DevBuf b_subs, b_bits, b_nbits, b_crc, b_sub0, b_slen, b_off, b_mo;
    uint32_t nseg_ = 0, nsub_ = 0;
    std::vector<uint32_t> sub0_, nbits_, crc_;
    std::vector<uint64_t> seg_len_;
    std::vector<bz::StreamOut> outs_;
};

}  // namespace gz
