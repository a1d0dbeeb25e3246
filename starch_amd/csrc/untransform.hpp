// starch_amd/csrc/untransform.hpp -- host interface of the inverse transform
// (segment texts -> BED lines).
#pragma once
#include <string>
#include <vector>

#include "common.hpp"

struct TransformWorkspace;

namespace ut {

class Untransform {
public:
    struct Seg {
        uint64_t text_off, text_len;   // the segment's transformed text in d_text
        std::string name;              // its chromosome
    };
    // BED lines of every segment, in order, into `out`; returns their bytes.
    // Throws StarchError(-12) on text the forward transform cannot have made.
    uint64_t run(TransformWorkspace& tf, const uint8_t* d_text, uint64_t n, const std::vector<Seg>& segs,
                 hipStream_t st, DevBuf& out);

private:
    DevBuf b_seg, b_names, b_segfirst, b_rec, b_key, b_cd, b_contrib, b_excl, b_stop, b_olen, b_tmp;
};

}  // namespace ut
