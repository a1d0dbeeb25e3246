// starch_amd/csrc/bzlib_abi.hip -- the patched-libbz2 streaming ABI
// (include/starch_bzlib.h) on top of the GPU encoder.
//
// Mirrors the state machine of bz:bzlib.c:148-500 (modes RUNNING / FLUSHING /
// FINISHING / IDLE, avail_in_expect, return codes, total_in/out counters,
// block_close_functor at BZ_STREAM_END).  Input is recorded until the caller
// ends a piece with BZ_FLUSH or BZ_FINISH; the piece is then RLE1-coded,
// block-cut, sorted and coded on the GPU on its own (flush_RL resets the run
// state, bz:bzlib.c:393-397; its final single-byte run joins a full block
// only when the terminating call supplied input), and its blocks' bits are
// appended to the stream's bit string: at BZ_FLUSH every whole byte so far is
// output, the last 0..7 bits stay pending (the library's bsBuff/bsLive carry
// across BZ2_compressBlock, bz:compress.c:609); BZ_FINISH appends the trailer
// with the combined CRC and pads to a byte (bz:compress.c:657-666).  The
// bytes and the total_out after every call are those of the patched library
// for the same call sequence; only BZ_RUN differs in timing (the library emits
// a block as soon as 900 k are buffered, here at the next FLUSH/FINISH).
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
    std::vector<uint8_t> input;         // bytes of the open piece
    std::vector<uint8_t> output;        // whole bytes not yet drained
    uint64_t out_pos = 0;
    uint64_t released = 0;              // output[0, released) may be drained (the library's numZ)
    uint64_t total_bits = 0;            // bits of the stream so far
    uint32_t last_n = 0;                // bits of the last write (bsW) so far
    uint32_t tail = 0, tail_bits = 0;   // bits not yet a whole byte (right-aligned, < 8)
    bool header = false;                // "BZh<level>" written (first BZ2_compressBlock)
    bool pending_piece = false;         // a FINISH failed: the closed piece is still to encode
    bool pending_supplied = false, pending_finish = false;
    uint32_t n_blocks = 0, combined = 0;
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

void put_bits(GpuStreamState* g, uint32_t v, uint32_t n)   // n <= 24, MSB first
{
    g->total_bits += n;
    g->tail = (g->tail << n) | (v & ((1u << n) - 1u));
    g->tail_bits += n;
    while (g->tail_bits >= 8) {
        g->tail_bits -= 8;
        g->output.push_back((uint8_t)(g->tail >> g->tail_bits));
    }
    g->tail &= (1u << g->tail_bits) - 1u;
}

// append bits [bit0, bit0 + nbits) of src (MSB-first bit string)
void put_stream_bits(GpuStreamState* g, const uint8_t* src, uint64_t bit0, uint64_t nbits)
{
    const uint64_t tb = g->total_bits;
    uint64_t b = bit0;
    const uint64_t e = bit0 + nbits;
    while (b < e && (b & 7)) {   // to a source byte boundary
        put_bits(g, (src[b >> 3] >> (7 - (b & 7))) & 1u, 1);
        ++b;
    }
    const uint64_t whole = (e - b) / 8;
    const uint8_t* p = src + (b >> 3);
    if (g->tail_bits == 0) {
        g->output.insert(g->output.end(), p, p + whole);
    } else {
        const uint32_t t = g->tail_bits;
        uint32_t acc = g->tail;
        const size_t o = g->output.size();
        g->output.resize(o + whole);
        for (uint64_t i = 0; i < whole; ++i) {
            acc = (acc << 8) | p[i];
            g->output[o + i] = (uint8_t)(acc >> t);
            acc &= (1u << t) - 1u;
        }
        g->tail = acc;
    }
    b += whole * 8;
    for (; b < e; ++b) put_bits(g, (src[b >> 3] >> (7 - (b & 7))) & 1u, 1);
    g->total_bits = tb + nbits;
}

// bytes libbz2 has emitted at the end of a block: bsW flushes whole bytes only
// BEFORE adding bits (bsNEEDW, bz:compress.c:37-52), so after the last write of
// n bits, ((T - n) mod 8) + n bits stay in its buffer
void release(GpuStreamState* g)
{
    const uint64_t keep = ((g->total_bits - g->last_n) & 7u) + g->last_n;
    g->released = (g->total_bits - keep) / 8;
}

// BZ2_compressBlock for the open piece (bz:compress.c:602-667): encode it on
// the GPU as a stream of its own and append its blocks' bits
int encode_piece(GpuStreamState* g, bool supplied)
{
    std::vector<uint8_t> tmp;
    bz::StreamOut so{};
    uint32_t last = 0;
    if (!g->input.empty()) {
        Slot* sl = nullptr;
        try {
            const int dev = target_device();
            DeviceGuard guard(dev);
            sl = acquire(dev);
            if (!sl->st) HIP_CHECK(hipStreamCreateWithFlags(&sl->st, hipStreamNonBlocking));
            const uint64_t n = g->input.size();
            uint8_t* d_in = sl->in.as<uint8_t>(n + 64);
            HIP_CHECK(hipMemcpyAsync(d_in, g->input.data(), n, hipMemcpyHostToDevice, sl->st));
            std::vector<bz::StreamIn> pieces(1);
            pieces[0].text_off = 0;
            pieces[0].text_len = n;
            pieces[0].final_run_joins = supplied ? 1u : 0u;
            pieces[0].group = 0;
            std::vector<bz::StreamOut> outs;
            sl->enc.plan(d_in, pieces, g->bs100k, sl->st, outs, nullptr);
            const uint64_t cap = (outs[0].bytes + 64 + 255) / 256 * 256;
            uint8_t* d_out = sl->out.as<uint8_t>(cap);
            sl->enc.emit(d_out, cap, 0, outs, sl->st, nullptr);
            so = outs[0];
            last = sl->enc.last_write_bits(0, so, sl->st);
            tmp.resize(so.bytes);
            HIP_CHECK(hipMemcpyAsync(tmp.data(), d_out, so.bytes, hipMemcpyDeviceToHost, sl->st));
            HIP_CHECK(hipStreamSynchronize(sl->st));
            release(sl);
        } catch (const std::exception&) {
            if (sl) release(sl);
            return BZ_CONFIG_ERROR;
        }
    }
    if (!g->header) {   // the first compressBlock writes the stream header, data or not
        put_bits(g, 'B', 8);
        put_bits(g, 'Z', 8);
        put_bits(g, 'h', 8);
        put_bits(g, (uint32_t)('0' + g->bs100k), 8);
        g->header = true;
        g->last_n = 8;
    }
    if (so.n_blocks) {
        put_stream_bits(g, tmp.data(), 32, so.block_bits);   // after the piece stream's own header
        // combined CRC over all blocks: c = rotl1(c) ^ blockCRC per block, so a
        // piece of k blocks folds in as rotl_k(c) ^ (its own combined CRC)
        const uint32_t k = so.n_blocks & 31u;
        g->combined = (k ? (g->combined << k) | (g->combined >> (32 - k)) : g->combined) ^ so.combined_crc;
        g->n_blocks += so.n_blocks;
        g->last_n = last;
    }
    release(g);
    g->input.clear();
    return BZ_OK;
}

void finish_stream(GpuStreamState* g)   // trailer + combined CRC + byte pad
{
    put_bits(g, 0x177245u, 24);
    put_bits(g, 0x385090u, 24);
    put_bits(g, g->combined >> 16, 16);
    put_bits(g, g->combined & 0xFFFFu, 16);
    if (g->tail_bits) put_bits(g, 0, 8 - g->tail_bits);
    g->released = g->output.size();   // bsFinishWrite
    g->input.shrink_to_fit();
}

bool drain(GpuStreamState* g)
{
    bz_stream* s = g->strm;
    uint64_t left = g->released - g->out_pos;
    uint64_t k = left < s->avail_out ? left : s->avail_out;
    if (k) {
        memcpy(s->next_out, g->output.data() + g->out_pos, k);
        s->next_out += k;
        s->avail_out -= (unsigned)k;
        g->out_pos += k;
        add_out(s, k);
    }
    if (g->out_pos == g->released && g->out_pos > (1u << 20)) {   // compact the drained prefix
        g->output.erase(g->output.begin(), g->output.begin() + (std::ptrdiff_t)g->out_pos);
        g->released -= g->out_pos;
        g->out_pos = 0;
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
            if (action == BZ_FLUSH || action == BZ_FINISH) {
                const bool supplied = strm->avail_in > 0;
                consume(g);
                if (int rc = encode_piece(g, supplied)) {   // input kept: the same call may be retried
                    g->mode = M_FAILED;
                    g->pending_piece = true;
                    g->pending_supplied = supplied;
                    g->pending_finish = action == BZ_FINISH;
                    return rc;
                }
                if (action == BZ_FLUSH) {
                    drain(g);
                    if (g->out_pos < g->released) { g->mode = M_FLUSHING; return BZ_FLUSH_OK; }   // bz:bzlib.c:451-459
                    return BZ_RUN_OK;
                }
                finish_stream(g);
                g->mode = M_FINISHING;
                break;
            }
            return BZ_PARAM_ERROR;
        case M_FLUSHING:   // avail_in_expect is 0: everything was consumed by the first FLUSH call
            if (action != BZ_FLUSH || strm->avail_in != 0) return BZ_SEQUENCE_ERROR;
            drain(g);
            if (g->out_pos < g->released) return BZ_FLUSH_OK;
            g->mode = M_RUNNING;
            return BZ_RUN_OK;
        case M_FINISHING:
            if (action != BZ_FINISH) return BZ_SEQUENCE_ERROR;
            if (strm->avail_in != 0) return BZ_SEQUENCE_ERROR;          // avail_in_expect mismatch
            break;
        case M_FAILED:   // the piece is still held: the same action retries its encode
            if ((action == BZ_FINISH) != g->pending_finish || action == BZ_RUN || strm->avail_in != 0)
                return BZ_SEQUENCE_ERROR;
            if (int rc = encode_piece(g, g->pending_supplied)) return rc;
            g->pending_piece = false;
            if (!g->pending_finish) {
                g->mode = M_RUNNING;
                drain(g);
                if (g->out_pos < g->released) { g->mode = M_FLUSHING; return BZ_FLUSH_OK; }
                return BZ_RUN_OK;
            }
            finish_stream(g);
            g->mode = M_FINISHING;
            break;
        default:
            return BZ_SEQUENCE_ERROR;
    }
    // FINISHING: drain the encoded stream
    bool progress = drain(g);
    if (g->out_pos < g->released) return progress ? BZ_FINISH_OK : BZ_SEQUENCE_ERROR;
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

int starch_bzstream_info(bz_stream* strm, unsigned int* n_blocks, unsigned int* combined_crc)
{
    GpuStreamState* g = state_of(strm);
    if (!g || !n_blocks || !combined_crc) return BZ_PARAM_ERROR;
    *n_blocks = g->n_blocks;
    *combined_crc = g->combined;
    return BZ_OK;
}

}  // extern "C"
