// starch_amd/csrc/bzlib_abi.hip -- the patched-libbz2 streaming ABI
// (include/starch_bzlib.h) on top of the GPU encoder.
//
// Mirrors the state machine of bz:bzlib.c:148-500 (modes RUNNING / FLUSHING /
// FINISHING / IDLE, avail_in_expect, return codes, total_in/out counters,
// block_close_functor at BZ_STREAM_END), but instead of compressing a block
// at a time on the CPU it records the input and the BZ_FLUSH boundaries and
// encodes the whole stream on the GPU when BZ_FINISH arrives.  The bytes are
// those of the patched library for the same call sequence: each flush-
// delimited piece is RLE1-coded and block-cut on its own (flush_RL resets the
// run state, bz:bzlib.c:393-397), and a piece's final single-byte run joins a
// full block only when the terminating FLUSH/FINISH call supplied input.
#include <string.h>

#include <condition_variable>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "../../include/starch_bzlib.h"
#include "bz2.hpp"

namespace {

enum Mode { M_IDLE = 1, M_RUNNING = 2, M_FLUSHING = 3, M_FINISHING = 4, M_FAILED = 5 };

struct GpuStreamState {
    bz_stream* strm;
    int bs100k;
    int mode;
    std::vector<uint8_t> input;
    std::vector<bz::StreamIn> pieces;   // closed pieces
    uint64_t piece_start = 0;
    std::vector<uint8_t> output;
    uint64_t out_pos = 0;
    bool encoded = false;
};

// Encoder slots: each stream borrows one for its BZ_FINISH encode, so
// streams of different threads encode concurrently (up to kSlots at once per
// process) on their own HIP streams.  A slot belongs to one device.
constexpr int kSlots = 4;
struct Slot {
    int device = 0;
    bool busy = false;
    hipStream_t st = nullptr;
    bz::Encoder enc;
    DevBuf in, out;
};
struct Pool {
    std::mutex mu;
    std::condition_variable cv;
    std::vector<std::unique_ptr<Slot>> slots;
};
Pool g_pool;

int target_device()
{
    const char* e = getenv("STARCH_DEVICE");
    return e ? atoi(e) : 0;
}

// device guard: the encode runs on the slot's device; the caller thread's
// current device is restored afterwards
struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev)
    {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        HIP_CHECK(hipSetDevice(dev));
    }
    ~DeviceGuard() { if (prev >= 0) (void)hipSetDevice(prev); }
};

Slot* acquire(int dev)
{
    std::unique_lock<std::mutex> lk(g_pool.mu);
    for (;;) {
        int n = 0;
        for (auto& s : g_pool.slots) {
            if (s->device != dev) continue;
            ++n;
            if (!s->busy) { s->busy = true; return s.get(); }
        }
        if (n < kSlots) {
            g_pool.slots.emplace_back(new Slot());
            Slot* s = g_pool.slots.back().get();
            s->device = dev;
            s->busy = true;
            return s;
        }
        g_pool.cv.wait(lk);
    }
}

void release(Slot* s)
{
    {
        std::lock_guard<std::mutex> lk(g_pool.mu);
        s->busy = false;
    }
    g_pool.cv.notify_all();
}

void* default_bzalloc(void*, int items, int size) { return malloc((size_t)items * (size_t)size); }   // bz:bzlib.c:151-156
void default_bzfree(void*, void* addr) { free(addr); }

void add_in(bz_stream* s, uint64_t n)
{
    uint64_t t = ((uint64_t)s->total_in_hi32 << 32 | s->total_in_lo32) + n;
    s->total_in_lo32 = (unsigned)t;
    s->total_in_hi32 = (unsigned)(t >> 32);
}
void add_out(bz_stream* s, uint64_t n)
{
    uint64_t t = ((uint64_t)s->total_out_hi32 << 32 | s->total_out_lo32) + n;
    s->total_out_lo32 = (unsigned)t;
    s->total_out_hi32 = (unsigned)(t >> 32);
}

void consume(GpuStreamState* g)
{
    bz_stream* s = g->strm;
    if (s->avail_in) {
        g->input.insert(g->input.end(), (uint8_t*)s->next_in, (uint8_t*)s->next_in + s->avail_in);
        s->next_in += s->avail_in;
        add_in(s, s->avail_in);
        s->avail_in = 0;
    }
}

void close_piece(GpuStreamState* g, bool supplied)
{
    bz::StreamIn p;
    p.text_off = g->piece_start;
    p.text_len = g->input.size() - g->piece_start;
    p.final_run_joins = supplied ? 1u : 0u;
    p.group = 0;
    g->pieces.push_back(p);
    g->piece_start = g->input.size();
}

int encode_on_gpu(GpuStreamState* g)
{
    Slot* sl = nullptr;
    try {
        const int dev = target_device();
        DeviceGuard guard(dev);
        sl = acquire(dev);
        if (!sl->st) HIP_CHECK(hipStreamCreateWithFlags(&sl->st, hipStreamNonBlocking));
        uint64_t n = g->input.size();
        uint8_t* d_in = sl->in.as<uint8_t>(n + 64);
        if (n) HIP_CHECK(hipMemcpyAsync(d_in, g->input.data(), n, hipMemcpyHostToDevice, sl->st));
        std::vector<bz::StreamOut> outs;
        sl->enc.plan(d_in, g->pieces, g->bs100k, sl->st, outs, nullptr);
        uint64_t bytes = outs.empty() ? 0 : outs[0].bytes;
        uint64_t cap = (bytes + 64 + 255) / 256 * 256;
        uint8_t* d_out = sl->out.as<uint8_t>(cap);
        sl->enc.emit(d_out, cap, 0, outs, sl->st, nullptr);
        g->output.resize(bytes);
        if (bytes) HIP_CHECK(hipMemcpyAsync(g->output.data(), d_out, bytes, hipMemcpyDeviceToHost, sl->st));
        HIP_CHECK(hipStreamSynchronize(sl->st));
        release(sl);
    } catch (const std::exception&) {
        if (sl) release(sl);
        g->output.clear();
        return BZ_CONFIG_ERROR;
    }
    g->input.clear();
    g->input.shrink_to_fit();
    g->encoded = true;
    return BZ_OK;
}

bool drain(GpuStreamState* g)
{
    bz_stream* s = g->strm;
    uint64_t left = g->output.size() - g->out_pos;
    uint64_t k = left < s->avail_out ? left : s->avail_out;
    if (k) {
        memcpy(s->next_out, g->output.data() + g->out_pos, k);
        s->next_out += k;
        s->avail_out -= (unsigned)k;
        g->out_pos += k;
        add_out(s, k);
    }
    return k > 0;
}

GpuStreamState* state_of(bz_stream* s)
{
    if (!s || !s->state) return nullptr;
    GpuStreamState* g = static_cast<GpuStreamState*>(s->state);
    return g->strm == s ? g : nullptr;
}

}  // namespace

extern "C" {

int BZ2_bzCompressInit(bz_stream* strm, int blockSize100k, int verbosity, int workFactor)
{
    (void)verbosity;
    if (!strm || blockSize100k < 1 || blockSize100k > 9 || workFactor < 0 || workFactor > 250)
        return BZ_PARAM_ERROR;                                            // bz:bzlib.c:159-162
    if (!strm->bzalloc) strm->bzalloc = default_bzalloc;                 // bz:bzlib.c:165-166
    if (!strm->bzfree) strm->bzfree = default_bzfree;
    void* mem = strm->bzalloc(strm->opaque, (int)sizeof(GpuStreamState), 1);
    if (!mem) return BZ_MEM_ERROR;
    GpuStreamState* g = new (mem) GpuStreamState();
    g->strm = strm;
    g->bs100k = blockSize100k;
    g->mode = M_RUNNING;
    strm->state = g;
    strm->total_in_lo32 = strm->total_in_hi32 = 0;
    strm->total_out_lo32 = strm->total_out_hi32 = 0;
    strm->block_close_functor = nullptr;                                  // bz:bzlib.c:211-212
    strm->handler = nullptr;
    return BZ_OK;
}

int BZ2_bzCompress(bz_stream* strm, int action)
{
    GpuStreamState* g = state_of(strm);
    if (!g) return BZ_PARAM_ERROR;
    switch (g->mode) {
        case M_IDLE:
            return BZ_SEQUENCE_ERROR;
        case M_RUNNING:
            if (action == BZ_RUN) {
                bool progress = strm->avail_in > 0;
                consume(g);
                return progress ? BZ_RUN_OK : BZ_PARAM_ERROR;           // bz:bzlib.c:432-434
            }
            if (action == BZ_FLUSH) {
                bool supplied = strm->avail_in > 0;
                consume(g);
                close_piece(g, supplied);
                return BZ_RUN_OK;
            }
            if (action == BZ_FINISH) {
                bool supplied = strm->avail_in > 0;
                consume(g);
                close_piece(g, supplied);
                int rc = encode_on_gpu(g);
                if (rc != BZ_OK) {   // never report BZ_STREAM_END for a stream that was not encoded
                    g->mode = M_FAILED;
                    return rc;
                }
                g->mode = M_FINISHING;
                break;
            }
            return BZ_PARAM_ERROR;
        case M_FINISHING:
            if (action != BZ_FINISH) return BZ_SEQUENCE_ERROR;
            if (strm->avail_in != 0) return BZ_SEQUENCE_ERROR;          // avail_in_expect mismatch
            break;
        case M_FAILED:   // the input is still held: a BZ_FINISH retries the encode
            if (action != BZ_FINISH || strm->avail_in != 0) return BZ_SEQUENCE_ERROR;
            if (int rc = encode_on_gpu(g)) return rc;
            g->mode = M_FINISHING;
            break;
        default:
            return BZ_SEQUENCE_ERROR;
    }
    // FINISHING: drain the encoded stream
    bool progress = drain(g);
    if (g->out_pos < g->output.size()) return progress ? BZ_FINISH_OK : BZ_SEQUENCE_ERROR;
    g->mode = M_IDLE;
    if (strm->block_close_functor) strm->block_close_functor(strm->handler);   // bz:bzlib.c:470
    return BZ_STREAM_END;
}

int BZ2_bzCompressEnd(bz_stream* strm)
{
    GpuStreamState* g = state_of(strm);
    if (!g) return BZ_PARAM_ERROR;
    g->~GpuStreamState();
    strm->bzfree(strm->opaque, g);                                        // bz:bzlib.c:493-497
    strm->state = nullptr;
    return BZ_OK;
}

const char* BZ2_bzlibVersion(void) { return "1.0.6-starch-mi355x"; }

}  // extern "C"
