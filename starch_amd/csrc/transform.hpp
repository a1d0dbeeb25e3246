// starch_amd/csrc/transform.hpp -- host interface of the transform stage.
#pragma once
#include <vector>

#include "common.hpp"

struct SegInfo {            // one chromosome segment (hpp:393-407 flush unit)
    uint64_t first_line;
    uint64_t line_count;    // transform_state_t.line_count (hpp:503)
    uint64_t name_off;      // chr token offset in the input
    uint64_t name_len;      // strlen() of the chr token
    uint64_t text_off;      // offset of the segment's text in the text buffer
    uint64_t text_len;
};

struct TransformResult {
    uint64_t n_lines = 0, n_segments = 0, text_bytes = 0, ff_pos = ~0ull;
    bool general = false;   // some start/stop failed to parse: stale values were propagated
};

struct TransformWorkspace {
    DevBuf b_tile_cnt, b_tile_off, b_scal, b_tmp, b_line_end, b_start, b_stop, b_flags, b_rem_beg, b_rem_len,
        b_chr_len, b_idx, b_vcopy, b_out_len, b_seg_flag, b_out_off, b_seg_ord, b_seg_first, b_seg_info, b_text,
        b_fstatus, b_faggs, b_fx, b_arena, b_seg_arena;
    double text_ratio = 1.0;          // text bytes per input byte of the last run (single-pass capacity, path choice)
    bool ratio_seen = false;
    uint64_t seg_hint = 0;
    uint8_t* text = nullptr;          // device: transformed text (valid after run)
    SegInfo* seg_info_dev = nullptr;  // device: n_segments entries
    // init_start/init_stop: bed_t.start/stop before the first line (stale sscanf
    // values carried into a shard that starts mid-input, hpp:306-307)
    void run(const uint8_t* d_bed, uint64_t n, hipStream_t st, TransformResult& res, int64_t init_start = 0,
             int64_t init_stop = 0);
    // line-index based path (k_count_nl / k_index_nl, then k_tf1 + k_tf2 or the general path)
    void run_two_pass(const uint8_t* d_bed, uint64_t n, hipStream_t st, TransformResult& res, int64_t init_start,
                      int64_t init_stop);
    // line ends of the input up to the first 0xFF (b_line_end); returns the line count
    uint64_t index_lines(const uint8_t* d_bed, uint64_t n, hipStream_t st, uint64_t* ff_pos);
    // per-segment base counts, modulo 2^64; leaves text / seg_info_dev untouched
    void base_counts(const uint8_t* d_bed, uint64_t n, hipStream_t st, int64_t init_start, int64_t init_stop,
                     std::vector<uint64_t>& unique, std::vector<uint64_t>& nonunique);
};
