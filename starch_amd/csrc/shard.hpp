// starch_amd/csrc/shard.hpp -- host shard planning (shard.cpp).
#pragma once
#include <stdint.h>

#include <vector>

namespace shard {

struct Unit {              // same layout as starch_unit (include/starch_amd.h)
    uint64_t offset, length;
    int64_t init_start, init_stop;
};

// bytes before the first 0xFF (which reads as EOF, hpp:181)
uint64_t input_limit(const uint8_t* b, uint64_t n);
// split [0, input_limit) into at most max_units units whose boundaries are segment boundaries;
// (init_start0, init_stop0) = the sscanf values current before byte 0 (0, 0 at the input start)
void plan_units(const uint8_t* b, uint64_t n, uint64_t max_units, std::vector<Unit>& out, int64_t init_start0 = 0,
                int64_t init_stop0 = 0);
// the same over [0, lim) when the caller knows there is no 0xFF before lim (no scan)
void plan_units_upto(const uint8_t* b, uint64_t lim, uint64_t max_units, std::vector<Unit>& out,
                     int64_t init_start0 = 0, int64_t init_stop0 = 0);
// the sscanf values current before the line starting at pos: those of the
// last lines in [lo, pos) whose fields parse; (start, stop) on entry are the
// values current before lo (hpp:306-307)
void values_before(const uint8_t* b, uint64_t lo, uint64_t pos, int64_t* start, int64_t* stop);
// longest-processing-time assignment of units to shards by byte length
void assign_lpt(const std::vector<Unit>& units, int nshards, std::vector<int32_t>& shard_of);
// archive order of gathered segments (stable by unit) and their byte offsets from `base`
void layout(const uint64_t* unit_of, const uint64_t* bytes, uint64_t nseg, uint64_t base, std::vector<uint64_t>& order,
            std::vector<uint64_t>& offset, uint64_t* end);

}  // namespace shard
