// starch_amd/csrc/ctx.hpp -- the context behind the C ABI's opaque
// starch_ctx (include/starch_amd.h), shared by starch_api.hip (encode,
// stream, decode entry points) and gather.hip (the multi-rank archive gather).
#pragma once
#include <stdint.h>

#include <string.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <memory>
#include <map>
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

// A few persistent host threads for large memcpys (streamed input lands in
// pinned memory at several times one core's copy bandwidth).
struct CopyPool {
    std::vector<std::thread> th;
    std::mutex mu;
    std::condition_variable cv, done;
    uint8_t* dst = nullptr;
    const uint8_t* src = nullptr;
    uint64_t n = 0, chunk = 0, gen = 0;
    std::atomic<uint64_t> next{0};
    std::atomic<uint64_t> ff{0};
    bool find_ff = false;
    int pending = 0;
    bool stop = false;
    void run(int id, uint64_t seen)
    {
        (void)id;
        for (;;) {
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return stop || gen != seen; });
                if (stop) return;
                seen = gen;
            }
            work();
            std::lock_guard<std::mutex> lk(mu);
            if (--pending == 0) done.notify_all();
        }
    }
    // take chunks until none is left; each chunk goes in 256 KiB steps, its
    // 0xFF search right after each step's copy (the bytes still in cache)
    void work()
    {
        for (;;) {
            const uint64_t k = next.fetch_add(1);
            const uint64_t o = k * chunk;
            if (o >= n) break;
            const uint64_t e = std::min(o + chunk, n);
            for (uint64_t p = o; p < e; p += kStep) {
                const uint64_t len = std::min(kStep, e - p);
                memcpy(dst + p, src + p, len);
                if (!find_ff) continue;
                const void* f = memchr(dst + p, 0xFF, len);
                if (f) {
                    const uint64_t at = p + (uint64_t)(static_cast<const uint8_t*>(f) - (dst + p));
                    uint64_t cur = ff.load();
                    while (at < cur && !ff.compare_exchange_weak(cur, at)) {}
                    break;   // a later 0xFF in this chunk cannot be the first
                }
            }
        }
    }
    static constexpr uint64_t kStep = 256ull << 10;
    // copy and return the offset of the first 0xFF in the bytes (len if none)
    uint64_t copy_find_ff(uint8_t* d, const uint8_t* s, uint64_t len)
    {
        if (len < (8ull << 20)) {
            memcpy(d, s, len);
            const void* f = memchr(d, 0xFF, len);
            return f ? (uint64_t)(static_cast<const uint8_t*>(f) - d) : len;
        }
        find_ff = true;
        ff = len;
        copy(d, s, len);
        find_ff = false;
        return ff.load();
    }
    void copy(uint8_t* d, const uint8_t* s, uint64_t len)
    {
        if (len < (8ull << 20)) { memcpy(d, s, len); return; }
        if (th.empty()) {   // the caller copies too: threads = the CPU share (OMP_NUM_THREADS) - 1
            unsigned hw = std::thread::hardware_concurrency();
            const char* e = getenv("OMP_NUM_THREADS");
            unsigned want = e && atoi(e) > 0 ? (unsigned)atoi(e) : std::min(16u, std::max(1u, hw / 2));
            want = std::min(want, 32u);
            for (unsigned i = 1; i < want; ++i) th.emplace_back(&CopyPool::run, this, (int)i, (uint64_t)0);
        }
        {
            std::lock_guard<std::mutex> lk(mu);
            dst = d;
            src = s;
            n = len;
            chunk = 1ull << 20;
            next = 0;
            pending = (int)th.size();
            ++gen;
        }
        cv.notify_all();
        work();
        std::unique_lock<std::mutex> lk(mu);
        done.wait(lk, [&] { return pending == 0; });
    }
    ~CopyPool()
    {
        {
            std::lock_guard<std::mutex> lk(mu);
            stop = true;
        }
        cv.notify_all();
        for (auto& t : th) t.join();
    }
};

// One persistent host thread that runs jobs one at a time (an extra encoder
// lane's plan in the device path: no thread start per encode).
struct LaneWorker {
    std::thread th;
    std::mutex mu;
    std::condition_variable cv;
    std::function<void()> job;
    bool pending = false, stop = false;
    void start(std::function<void()> f)
    {
        {
            std::lock_guard<std::mutex> lk(mu);
            job = std::move(f);
            pending = true;
        }
        if (!th.joinable()) th = std::thread([this] { loop(); });
        cv.notify_all();
    }
    void wait()
    {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return !pending; });
    }
    void loop()
    {
        std::unique_lock<std::mutex> lk(mu);
        for (;;) {
            cv.wait(lk, [&] { return pending || stop; });
            if (!pending) return;
            std::function<void()> f = std::move(job);
            lk.unlock();
            f();                      // (catches its own errors)
            lk.lock();
            pending = false;
            cv.notify_all();
        }
    }
    void shutdown()
    {
        if (!th.joinable()) return;
        {
            std::lock_guard<std::mutex> lk(mu);
            stop = true;
        }
        cv.notify_all();
        th.join();
    }
    ~LaneWorker() { shutdown(); }
};

struct starch_ctx {
    int device = 0;
    hipStream_t own = nullptr;
    hipStream_t st = nullptr;
    hipStream_t cst = nullptr;       // copy stream: H2D of the next batch while one encodes (pipelined host input)
    DevBuf pin_in[2];                // the pipelined path's two device input slots
    DevBuf collect;                  // the pipelined path: this lane's finished streams, batch after batch
    std::vector<std::unique_ptr<starch_ctx>> lanes;   // the pipelined path's extra lanes (same device)
    LaneWorker worker;               // an extra lane's host thread (device-path encoder lanes)
    int dev_lanes = 0;               // device-path encoder lanes (starch_set_lanes; 0: default)
    TransformWorkspace tf;
    bz::Encoder enc;
    gz::Encoder genc;            // the gzip method (-g)
    DevBuf input, archive, part, raw_in, raw_out, text_all;
    DevBuf names_dev;                // segment names gathered on the device (one D2H per encode)
    PinnedBuf names_pin;             // ... their host copy, and the gather descriptors
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
    bool gathered = false;            // rank 0 after starch_gather_archive: segs are archive-order records
    hipEvent_t tev[3] = {nullptr, nullptr, nullptr};   // encode timers (created once, reused)
    hipEvent_t* timers()
    {
        for (auto& e : tev)
            if (!e && hipEventCreate(&e) != hipSuccess) { e = nullptr; throw StarchError(STARCH_ERR_DEVICE, "hipEventCreate"); }
        return tev;
    }
    struct Streaming {                // starch_stream_* session
        bool active = false, eof = false;
        starch_options opt{};
        std::string note;
        // three pinned buffers: the caller's bytes go into buf[cur] (from a
        // segment boundary on); a finished prefix is handed to one of two
        // encoder lanes while the tail moves to a free buffer, so two batches
        // encode while the third fills
        static constexpr int NBUF = 3, NLANE = 2;
        uint8_t* buf[NBUF] = {nullptr, nullptr, nullptr};
        uint64_t cap[NBUF] = {0, 0, 0};
        // device mirrors: every committed piece is copied to dbuf[cur] at once
        // (copy stream), so a batch is in HBM when it is handed over and the
        // lane only encodes
        DevBuf dbuf[NBUF];
        hipEvent_t buf_ev[NBUF] = {nullptr, nullptr, nullptr};   // the handed-over bytes are in HBM
        bool buf_busy[NBUF] = {false, false, false};            // handed to a lane, not finished
        CopyPool pool;
        // buffers other than the first are pinned by this thread while the
        // first batch is read (pinning 1 GiB took ~0.3 s of the CLI's set-up);
        // joined before any of them is touched
        std::thread prepin;
        int cur = 0;
        uint64_t held_n = 0, try_at = 0, batch = 0, batches = 0;
        double t_copy = 0, t_commit = 0;   // STARCH_TRACE: feed-side time
        uint64_t fed = 0;
        int64_t init_start = 0, init_stop = 0;   // sscanf values current before buf[cur][0]
        // buf[cur] starts with ctx_len bytes of context: the last line of a
        // batch cut inside a chromosome, re-parsed for the transform state of
        // the lines after it (its own output is dropped)
        uint64_t ctx_len = 0;
        // encoder lanes (lane 0: the context itself, lane 1: an extra context
        // on the same device), one job slot each
        struct Job {
            bool pending = false, busy = false;
            int bufi = 0;
            uint64_t n = 0, ctx = 0, seq = 0;
            bool open = false;          // the batch ends inside a chromosome
            bool cont = false;          // ... the batch before it did
            int64_t is = 0, ip = 0;
        } lj[NLANE];
        std::thread workers[NLANE];
        std::mutex mu;                // guards the job slots, buffers' busy flags, ready, segs/names/stats, err
        std::condition_variable cv;
        bool stop = false;
        bool last_open = false;       // the last batch handed over ends inside a chromosome
        // batches are appended to `ready` in hand-over order: seq_commit is the
        // next one; a lane that finishes out of order parks its result
        uint64_t seq_next = 0, seq_commit = 0;
        struct Done {
            std::vector<uint8_t> bytes;
            std::vector<starch_segment> segs;
            std::vector<std::string> names;
            starch_stats stats{};
        };
        std::map<uint64_t, Done> done;
        PinnedBuf back[NLANE];        // a lane's streams come back here (pinned D2H)
        struct OpenStream {             // a chromosome's bzip2 stream encoded batch by batch (encoder thread)
            bool active = false;
            std::string name;
            DevBuf rest;                // its text after the last complete block
            uint64_t rest_len = 0;
            uint32_t phase = 0, comb = 0, n_blocks = 0;
            uint8_t carry = 0;          // the first `phase` bits of its next byte
            uint64_t lines = 0, text_bytes = 0, off = 0, bytes = 0;
            void clear()                // everything but the rest's allocation and length
            {
                active = false;
                name.clear();
                phase = comb = n_blocks = 0;
                carry = 0;
                lines = text_bytes = off = bytes = 0;
            }
        } os;
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
        if (sm.prepin.joinable()) sm.prepin.join();
        {
            std::lock_guard<std::mutex> lk(sm.mu);
            sm.stop = true;
        }
        sm.cv.notify_all();
        for (auto& w : sm.workers)
            if (w.joinable()) w.join();
        sm.stop = false;
        sm.active = false;
    }
    bool is_lane = false;             // an extra lane: owns its streams (starch_destroy does the others')
    ~starch_ctx()
    {
        stream_shutdown();
        for (auto& l : lanes) l->worker.shutdown();
        worker.shutdown();
        lanes.clear();
        if (is_lane) {
            (void)hipSetDevice(device);
            if (own) (void)hipStreamSynchronize(own);
            if (cst) (void)hipStreamDestroy(cst);
            if (own) (void)hipStreamDestroy(own);
        }
        for (int i = 0; i < Streaming::NBUF; ++i) {
            if (sm.buf[i]) (void)hipHostFree(sm.buf[i]);
            if (sm.buf_ev[i]) (void)hipEventDestroy(sm.buf_ev[i]);
        }
        for (auto& e : tev)
            if (e) (void)hipEventDestroy(e);
    }
};

namespace archive {
extern const uint8_t kMagic[4];   // hpp:907-910
// JSON index + 32-byte footer for segments already placed at
// their stream offsets; index_off = where the index starts
std::string build_index(const starch_segment* segs, const char* const* names, const uint64_t* nlens, uint64_t nseg,
                        uint64_t index_off, const char* note, int bs, bool base_counts = false, int method = 0);
}  // namespace archive
