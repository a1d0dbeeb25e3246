// starch_amd/csrc/ctx.hpp -- the context behind the C ABI's opaque
// starch_ctx (include/starch_amd.h), shared by starch_api.hip (encode,
// stream, decode entry points) and gather.hip (the multi-rank archive gather).
#pragma once
#include <stdint.h>

#include <condition_variable>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/starch_amd.h"
#include "bz2.hpp"
#include "bz2_decode.hpp"
#include "gz.hpp"
#include "transform.hpp"
#include "untransform.hpp"

struct starch_ctx {
    int device = 0;
    hipStream_t own = nullptr;
    hipStream_t st = nullptr;
    TransformWorkspace tf;
    bz::Encoder enc;
    gz::Encoder genc;            // the gzip method (-g)
    DevBuf input, archive, part, raw_in, raw_out, text_all;
    // decompression / unstarch: the last result is out_dev[0, out_bytes)
    bz::Decoder dec;
    ut::Untransform untf;
    DevBuf dec_in, dec_out, ut_out;
    const uint8_t* out_dev = nullptr;
    uint64_t out_bytes = 0;
    bool have_out = false;
    std::vector<bz::DecStream> dstreams;
    std::string err;
    // last result
    bool have = false;
    uint64_t archive_bytes = 0;
    uint64_t part_bytes = 0;          // streams of a shard (starch_encode_units_device)
    uint64_t text_bytes = 0;
    const uint8_t* text_dev = nullptr;
    uint32_t bz_nblocks = 0, bz_crc = 0;    // first stream of the last starch_bz2_compress_* call
    std::vector<starch_segment> segs;
    std::vector<std::string> names;
    starch_stats stats{};
    bool streamed = false;            // the last result went out through starch_stream_read
    struct Streaming {                // starch_stream_* session
        bool active = false, eof = false;
        starch_options opt{};
        std::string note;
        // two pinned buffers: the caller's bytes go into buf[cur] (from a
        // segment boundary on); a finished prefix is handed to the encoder
        // thread while the tail moves to the other buffer (double buffering)
        uint8_t* buf[2] = {nullptr, nullptr};
        uint64_t cap[2] = {0, 0};
        int cur = 0;
        uint64_t held_n = 0, try_at = 0, batch = 0, batches = 0;
        int64_t init_start = 0, init_stop = 0;   // sscanf values current before buf[cur][0]
        // encoder thread and its one job slot
        std::thread worker;
        std::mutex mu;                // guards the job slot, ready, segs/names/stats, err
        std::condition_variable cv;
        bool job = false, busy = false, stop = false;
        const uint8_t* job_buf = nullptr;
        uint64_t job_n = 0;
        int64_t job_is = 0, job_ip = 0;
        int err = 0;
        std::string err_msg;
        std::vector<uint8_t> ready;   // archive bytes not yet read, from ready_off on
        uint64_t ready_off = 0, stream_end = 4;  // archive offset of the next stream
        std::vector<starch_segment> segs;
        std::vector<std::string> names;
        starch_stats stats{};
    } sm;
    void stream_shutdown()
    {
        if (sm.worker.joinable()) {
            {
                std::lock_guard<std::mutex> lk(sm.mu);
                sm.stop = true;
            }
            sm.cv.notify_all();
            sm.worker.join();
        }
        sm.stop = false;
        sm.active = false;
    }
    ~starch_ctx()
    {
        stream_shutdown();
        for (int i = 0; i < 2; ++i)
            if (sm.buf[i]) (void)hipHostFree(sm.buf[i]);
    }
};

namespace archive {
extern const uint8_t kMagic[4];   // hpp:907-910
// JSON index + 32-byte footer for segments already placed at
// their stream offsets; index_off = where the index starts
std::string build_index(const starch_segment* segs, const char* const* names, const uint64_t* nlens, uint64_t nseg,
                        uint64_t index_off, const char* note, int bs, bool base_counts = false, int method = 0);
}  // namespace archive
