// starch_amd/csrc/bzlib_abi.hip -- the patched-libbz2 streaming ABI
// (include/starch_bzlib.h) on top of the GPU encoder.
//
// A step-for-step emulation of libbz2's compression state machine
// (bz:bzlib.c:148-500): modes RUNNING / FLUSHING / FINISHING / IDLE, the
// INPUT / OUTPUT states of handle_compress, avail_in_expect, return codes,
// total_in / total_out, block_close_functor at BZ_STREAM_END.  The input side
// keeps libbz2's RLE1 bookkeeping (state_in_ch / state_in_len / nblock,
// ADD_CHAR_TO_BLOCK bz:bzlib.c:269-293) so every block closes where the
// library closes it: under BZ_RUN as soon as nblockMAX RLE1 bytes are in it
// (bz:bzlib.c:297-338, 399-402), the pending run carried into the next block;
// at FLUSH / FINISH with the pending run flushed in (flush_RL).  Only the
// current block's input is held on the host (<= nblockMAX + a run).  Where
// the library calls BZ2_compressBlock the block's text is coded on the GPU
// and its bits are appended to the stream's bit string; the bytes that call
// makes readable (numZ) follow the library's bit buffer, which keeps the
// bits of its last bsW when a block ends (bz:compress.c:37-52, 609), so
// total_out after every call -- BZ_RUN included -- equals the library's.
//
// Blocks are coded ahead in batches (one GPU plan for many blocks) where the
// input they cover is certain to be consumed: FLUSH / FINISH input (the
// caller has committed it: avail_in_expect) and BZ_RUN input when avail_out
// is large enough that the library would drain every block of the call.
// Otherwise one block is coded when it closes.
#include <string.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "../../include/starch_bzlib.h"
#include "bz2.hpp"

namespace {

enum Mode { M_IDLE = 1, M_RUNNING = 2, M_FLUSHING = 3, M_FINISHING = 4, M_FAILED = 5 };
enum State { S_OUTPUT = 1, S_INPUT = 2 };

// a block coded ahead: its text is input [beg, end) (absolute offsets); a
// block closed by nblockMAX also consumed its closing byte `end` (the first
// byte of the run it left pending); a flushed block ends the committed input
struct Coded {
    uint64_t beg, end;
    uint64_t bit_off, bits;     // in GpuStreamState::enc
    uint32_t crc, last_bits;
    bool flushed;
};

struct GpuStreamState {
    bz_stream* strm;
    int bs100k;
    int mode;
    int state = S_INPUT;
    uint32_t expect = 0;                // avail_in_expect
    uint32_t nblock_max = 0;
    // RLE1 bookkeeping of the current block (EState, bz:bzlib.c:116-126, 269-293)
    uint32_t in_ch = 256, in_len = 0, nblock = 0;
    std::vector<uint8_t> blk;           // the block's input bytes, the pending run included
    uint64_t blk_beg = 0;               // absolute input offset of blk[0]
    // a coded-ahead block that arrived whole in one call is not copied: its
    // last `virt` bytes are counted here instead of held in blk (only its
    // closing byte, the next block's pending run, is kept: virt_last)
    uint64_t virt = 0;
    uint8_t virt_last = 0;
    // where those bytes are: the caller's input of the current call (the block
    // is compressed in the same call that counted them, copy_input ->
    // compress_block), for a block that must be coded again after all
    const uint8_t* virt_src = nullptr;
    uint64_t consumed = 0;              // input bytes consumed (total_in)
    // blocks coded ahead
    std::deque<Coded> ahead;
    RawBytes enc;                       // their GPU output
    // the stream's bits
    RawBytes output;                    // whole bytes from stream offset out_base on
    uint64_t out_base = 0;              // stream offset of output[0] (drained bytes are dropped)
    uint64_t out_pos = 0;               // stream offset of the next byte to drain
    uint64_t released = 0;              // stream bytes [0, released) may be drained (the library's numZ)
    uint64_t total_bits = 0;            // bits of the stream so far
    uint32_t last_n = 0;                // bits of the last write (bsW) so far
    uint32_t tail = 0, tail_bits = 0;   // bits not yet a whole byte (right-aligned, < 8)
    bool header = false;                // "BZh<level>" written (first BZ2_compressBlock)
    uint32_t n_blocks = 0, combined = 0;
};

// Encoder slots: a stream borrows one to code blocks, so streams of different
// threads encode concurrently (up to kSlots at once per process) on their
// own HIP streams.  A slot belongs to one device.
int slots_per_device()
{
    static const int n = [] { const char* e = getenv("STARCH_BZ_SLOTS"); return e && atoi(e) > 0 ? atoi(e) : 2; }();
    return n;
}
struct Slot {
    int device = 0;
    bool busy = false;
    hipStream_t st = nullptr;
    bz::Encoder enc;
    DevBuf in, out;
    PinnedBuf stage;
};
struct CodeReq;
struct Pool {
    std::mutex mu;
    std::condition_variable cv;
    std::vector<std::unique_ptr<Slot>> slots;
    std::deque<CodeReq*> queue;        // code_text requests not yet taken by a slot
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

// a free slot of the device (made if fewer than slots_per_device exist), or
// null; g_pool.mu held
Slot* try_acquire_locked(int dev)
{
    int n = 0;
    for (auto& s : g_pool.slots) {
        if (s->device != dev) continue;
        ++n;
        if (!s->busy) { s->busy = true; return s.get(); }
    }
    if (n < slots_per_device()) {
        g_pool.slots.emplace_back(new Slot());
        Slot* s = g_pool.slots.back().get();
        s->device = dev;
        s->busy = true;
        return s;
    }
    return nullptr;
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

void put_bits(GpuStreamState* g, uint32_t v, uint32_t n)   // n <= 24, MSB first
{
    g->total_bits += n;
    g->tail = (g->tail << n) | (v & ((1u << n) - 1u));
    g->tail_bits += n;
    while (g->tail_bits >= 8) {
        g->tail_bits -= 8;
        const size_t o = g->output.size();
        g->output.resize(o + 1);
        g->output.data()[o] = (uint8_t)(g->tail >> g->tail_bits);
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
    const size_t o = g->output.size();
    g->output.resize(o + whole);
    uint8_t* q = g->output.data() + o;
    if (g->tail_bits == 0) {
        if (whole) memcpy(q, p, whole);
    } else {   // shifted by t bits: 8 bytes per step (big-endian words), then bytewise
        const uint32_t t = g->tail_bits;
        uint64_t acc = g->tail;                    // t pending bits, right-aligned
        uint64_t i = 0;
        for (; i + 8 <= whole; i += 8) {
            uint64_t w;
            memcpy(&w, p + i, 8);
            w = __builtin_bswap64(w);
            const uint64_t out = (acc << (64 - t)) | (w >> t);
            acc = w & ((1ull << t) - 1ull);
            const uint64_t be = __builtin_bswap64(out);
            memcpy(q + i, &be, 8);
        }
        for (; i < whole; ++i) {
            acc = (acc << 8) | p[i];
            q[i] = (uint8_t)(acc >> t);
            acc &= (1ull << t) - 1ull;
        }
        g->tail = (uint32_t)acc;
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

// ---- RLE1 bookkeeping (ADD_CHAR_TO_BLOCK, bz:bzlib.c:269-293) --------------
inline void add_char(GpuStreamState* g, uint32_t c)
{
    if (c != g->in_ch && g->in_len == 1) {           // fast track: the pending single byte goes in
        ++g->nblock;
        g->in_ch = c;
    } else if (c != g->in_ch || g->in_len == 255) {  // add_pair_to_block (bz:bzlib.c:224-256)
        if (g->in_ch < 256) g->nblock += g->in_len <= 3 ? g->in_len : 5u;
        g->in_ch = c;
        g->in_len = 1;
    } else {
        ++g->in_len;
    }
}

bool empty_rl(const GpuStreamState* g) { return !(g->in_ch < 256 && g->in_len > 0); }   // isempty_RL

// consume input bytes [p, p + n) into the block, through the RLE1 bookkeeping,
// stopping once the block is full (copy_input_until_stop); returns the count
uint64_t track(GpuStreamState* g, const uint8_t* p, uint64_t n)
{
    uint64_t i = 0;
    while (i < n && g->nblock < g->nblock_max) {
        // eight bytes at a time while each differs from its predecessor: each
        // only pushes the pending single byte in (the fast track)
        if (g->in_len == 1 && n - i >= 8 && g->nblock + 8 < g->nblock_max) {
            uint64_t x;
            memcpy(&x, p + i, 8);
            const uint64_t prev = (x << 8) | (uint64_t)g->in_ch;
            const uint64_t d = x ^ prev;                  // a zero byte: a byte equal to its predecessor
            if (!((d - 0x0101010101010101ull) & ~d & 0x8080808080808080ull)) {
                g->nblock += 8;
                g->in_ch = (uint32_t)(x >> 56);
                i += 8;
                continue;
            }
        }
        add_char(g, p[i]);
        ++i;
    }
    return i;
}

// re-derive the bookkeeping of the current block from its bytes (after a
// partial consumption on the coded-ahead path)
void retrack(GpuStreamState* g)
{
    g->in_ch = 256;
    g->in_len = 0;
    g->nblock = 0;
    (void)track(g, g->blk.data(), g->blk.size());
}

// ---- GPU coding -------------------------------------------------------------
// Code text (host) as one piece on the GPU: closed (its last run flushed, the
// final block included) or open (complete blocks only).  Appends one Coded
// per block to g->ahead, with absolute offsets from `beg`.
//
// Requests of all threads go through one queue per process: a thread whose
// request is still queued when a slot (an encoder with its own HIP stream;
// STARCH_BZ_SLOTS, default 2 per device) is free takes every queued request
// of that device and block size -- up to 1 GiB of text, closed pieces in
// arrival order and at most one open piece, last (Encoder::plan's rule) --
// and codes them as the
// pieces of ONE plan; the others wait for their results.  Streams of
// different threads (one per chromosome in the process_tf_buffer hand-off)
// thus share the GPU's block sort instead of each running a plan of a few
// dozen blocks.
// STARCH_BZ_TRACE=1: process totals of the time BZ2_bzCompress spends coding
// on the GPU (code_text, waits for a batch included) and in all, printed at
// every BZ2_bzCompressEnd
std::atomic<uint64_t> g_tr_code{0}, g_tr_all{0};
bool bz_trace()
{
    static const bool on = [] { const char* e = getenv("STARCH_BZ_TRACE"); return e && !strcmp(e, "1"); }();
    return on;
}
uint64_t now_ns()
{
    return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::steady_clock::now().time_since_epoch()).count();
}
struct TraceSpan {
    std::atomic<uint64_t>& acc;
    uint64_t t0;
    explicit TraceSpan(std::atomic<uint64_t>& a) : acc(a), t0(bz_trace() ? now_ns() : 0) {}
    ~TraceSpan() { if (t0) acc += now_ns() - t0; }
};

struct CodeReq {
    GpuStreamState* g;
    const uint8_t *a, *b;
    uint64_t na, nb, beg;
    bool closed;
    int dev;
    bool taken = false, done = false;
    std::exception_ptr err;
};

void code_batch(Slot* sl, const std::vector<CodeReq*>& B)
{
    if (!sl->st) HIP_CHECK(hipStreamCreateWithFlags(&sl->st, hipStreamNonBlocking));
    const size_t nr = B.size();
    std::vector<uint64_t> off(nr);
    uint64_t total = 0, staged = 0;
    std::vector<std::unique_ptr<HostRegistration>> regs(nr);
    for (size_t i = 0; i < nr; ++i) {
        off[i] = total;
        total += B[i]->na + B[i]->nb;
        // a large piece of the caller's input is DMA'd straight from its buffer
        // (registered for this call, or page-locked by the caller); the rest
        // goes through the slot's pinned stage
        regs[i].reset(new HostRegistration(B[i]->b, B[i]->nb, 16ull << 20));
        staged += B[i]->na + (regs[i]->ok() ? 0 : B[i]->nb);
    }
    uint8_t* d_in = sl->in.as<uint8_t>(total + 64);
    uint8_t* h = static_cast<uint8_t*>(sl->stage.get(staged + 64));
    uint64_t hs = 0;
    for (size_t i = 0; i < nr; ++i) {   // one staged copy of each request's non-registered bytes
        const CodeReq& r = *B[i];
        const uint64_t h0 = hs;
        if (r.na) { memcpy(h + hs, r.a, r.na); hs += r.na; }
        if (r.nb && !regs[i]->ok()) { memcpy(h + hs, r.b, r.nb); hs += r.nb; }
        if (hs > h0) HIP_CHECK(hipMemcpyAsync(d_in + off[i], h + h0, hs - h0, hipMemcpyHostToDevice, sl->st));
        if (r.nb && regs[i]->ok()) regs[i]->h2d(d_in + off[i] + r.na, r.b, r.nb, sl->st);
    }
    std::vector<bz::StreamIn> pieces(nr);
    for (size_t i = 0; i < nr; ++i) {
        pieces[i] = bz::StreamIn{};
        pieces[i].text_off = off[i];
        pieces[i].text_len = B[i]->na + B[i]->nb;
        pieces[i].final_run_joins = 1;   // flush_RL adds the pending run to the block, full or not
        pieces[i].group = (uint32_t)i;
        pieces[i].open = B[i]->closed ? 0u : 1u;
    }
    std::vector<bz::StreamOut> outs;
    sl->enc.plan(d_in, pieces, B[0]->g->bs100k, sl->st, outs, nullptr);
    uint64_t cap = 0;
    for (const auto& o : outs) cap += o.bytes;
    cap = (cap + 64 * nr + 255) / 256 * 256;
    uint8_t* d_out = sl->out.as<uint8_t>(cap);
    sl->enc.emit(d_out, cap, 0, outs, sl->st, nullptr);
    std::vector<bz::Encoder::BlockOut> res;
    sl->enc.block_results(res, sl->st);
    for (size_t i = 0; i < nr; ++i) {
        GpuStreamState* g = B[i]->g;
        g->enc.resize(outs[i].bytes);
        if (outs[i].bytes)
            HIP_CHECK(hipMemcpyAsync(g->enc.data(), d_out + outs[i].out_off, outs[i].bytes, hipMemcpyDeviceToHost,
                                     sl->st));
    }
    HIP_CHECK(hipStreamSynchronize(sl->st));     // (the registrations' DMA is done before they unregister)
    size_t i = 0;
    for (size_t k = 0; k < res.size(); ++k) {    // blocks in piece order
        while (i + 1 < nr && res[k].in_beg >= off[i + 1]) ++i;
        const CodeReq& r = *B[i];
        const bool last = k + 1 == res.size() || res[k + 1].in_beg >= off[i] + r.na + r.nb;
        r.g->ahead.push_back(Coded{r.beg + (res[k].in_beg - off[i]), r.beg + (res[k].in_end - off[i]),
                                   res[k].bit_off - 8 * outs[i].out_off, res[k].bits, res[k].crc, res[k].last_bits,
                                   r.closed && last});
    }
}

void code_text(GpuStreamState* g, const uint8_t* a, uint64_t na, const uint8_t* b, uint64_t nb, uint64_t beg,
               bool closed)
{
    TraceSpan span(g_tr_code);
    if (na + nb == 0) return;
    CodeReq me;
    me.g = g;
    me.a = a;
    me.na = na;
    me.b = b;
    me.nb = nb;
    me.beg = beg;
    me.closed = closed;
    me.dev = target_device();
    DeviceGuard guard(me.dev);
    std::unique_lock<std::mutex> lk(g_pool.mu);
    g_pool.queue.push_back(&me);
    // if this thread leaves by an exception (a slot that could not be made)
    // while its request is still queued, the request goes with it
    struct Unqueue {
        CodeReq* r;
        std::unique_lock<std::mutex>& lk;
        ~Unqueue()
        {
            if (r->taken) return;
            if (!lk.owns_lock()) lk.lock();
            for (auto it = g_pool.queue.begin(); it != g_pool.queue.end(); ++it)
                if (*it == r) { g_pool.queue.erase(it); break; }
        }
    } unq{&me, lk};
    for (;;) {
        if (me.done) break;
        Slot* sl = me.taken ? nullptr : try_acquire_locked(me.dev);
        if (!sl) {
            g_pool.cv.wait(lk);
            continue;
        }
        // take the device's queued requests: closed ones in order, one open one last
        std::vector<CodeReq*> B;
        B.reserve(g_pool.queue.size());   // (no allocation once requests are marked taken)
        uint64_t bytes = 0;
        for (auto it = g_pool.queue.begin(); it != g_pool.queue.end();) {
            CodeReq* r = *it;
            const uint64_t n = r->na + r->nb;
            // (one plan has one block size: streams of another level wait for a plan of their own)
            if (r->dev != me.dev || (!B.empty() && (bytes + n > (1ull << 30) || r->g->bs100k != B[0]->g->bs100k))) {
                ++it;
                continue;
            }
            B.push_back(r);
            bytes += n;
            r->taken = true;
            it = g_pool.queue.erase(it);
            if (!r->closed) break;
        }
        lk.unlock();
        std::exception_ptr err;
        try {
            code_batch(sl, B);
        } catch (...) {
            err = std::current_exception();
        }
        lk.lock();
        for (CodeReq* r : B) {
            r->err = err;
            r->done = true;
        }
        sl->busy = false;
        g_pool.cv.notify_all();
    }
    lk.unlock();
    if (me.err) std::rethrow_exception(me.err);
}

// BZ2_compressBlock (bz:compress.c:602-667) at the current block: its text is
// the whole of blk when the pending run is flushed in (flush), else blk
// without the pending run (a block closed by nblockMAX)
void compress_block(GpuStreamState* g, bool flush, bool last)
{
    const uint64_t len = g->blk.size() + g->virt;
    const uint64_t text = flush ? len : len - g->in_len;
    if (text) {
        const bool have = !g->ahead.empty() && g->ahead.front().beg == g->blk_beg &&
                          g->ahead.front().end == g->blk_beg + text && g->ahead.front().flushed == flush;
        if (!have) {   // code this block alone
            g->ahead.clear();
            // (a block coded ahead as closed by nblockMAX that a FLUSH / FINISH
            // closes with its pending run instead: its counted bytes are the
            // last ones this call consumed, still in the caller's buffer)
            if (g->virt) {
                if (text < g->blk.size() || text - g->blk.size() > g->virt)
                    throw StarchError(-10, "bzlib: counted block bytes out of range");
                code_text(g, g->blk.data(), g->blk.size(), g->virt_src, text - g->blk.size(), g->blk_beg, true);
            } else {
                code_text(g, g->blk.data(), text, nullptr, 0, g->blk_beg, true);
            }
            if (g->ahead.size() != 1 || g->ahead.front().end != g->blk_beg + text)
                throw StarchError(-10, "bzlib: block cut differs from the RLE1 bookkeeping");
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
    if (text) {
        const Coded c = g->ahead.front();
        g->ahead.pop_front();
        put_stream_bits(g, g->enc.data(), c.bit_off, c.bits);
        g->combined = ((g->combined << 1) | (g->combined >> 31)) ^ c.crc;   // bz:compress.c:606-608
        ++g->n_blocks;
        g->last_n = c.last_bits;
    }
    if (last) {        // trailer + combined CRC + byte pad (bz:compress.c:657-666)
        put_bits(g, 0x177245u, 24);
        put_bits(g, 0x385090u, 24);
        put_bits(g, g->combined >> 16, 16);
        put_bits(g, g->combined & 0xFFFFu, 16);
        if (g->tail_bits) put_bits(g, 0, 8 - g->tail_bits);
        g->released = g->out_base + g->output.size();   // bsFinishWrite
    } else {
        release(g);
    }
    // the next block starts with the pending run (none after a flush: init_RL)
    if (flush) {
        g->blk.clear();
        g->virt = 0;
        g->blk_beg = g->consumed;
        g->in_ch = 256;
        g->in_len = 0;
    } else {
        if (g->virt) {   // (closed by nblockMAX: in_len is 1, its closing byte is the last one)
            g->blk.assign(1, g->virt_last);
            g->virt = 0;
        } else {
            g->blk.erase(g->blk.begin(), g->blk.begin() + (std::ptrdiff_t)text);
        }
        g->blk_beg += text;
    }
    g->nblock = 0;
    if (g->blk.capacity() > (4u << 20)) g->blk.shrink_to_fit();
}

// code the blocks of input that is certain to be consumed in one GPU plan
// (see the header comment); at most kAhead bytes of new input at a time
// (STARCH_BZ_AHEAD overrides it, for tests: a small limit exercises the open,
// non-final plans that larger FLUSH / FINISH / BZ_RUN commitments take)
uint64_t ahead_limit()
{
    const char* e = getenv("STARCH_BZ_AHEAD");
    const long long v = e ? atoll(e) : 0;
    return v > 0 ? (uint64_t)v : 64ull << 20;
}
void code_ahead(GpuStreamState* g)
{
    if (!g->ahead.empty()) return;
    const uint64_t kAhead = ahead_limit();
    bz_stream* s = g->strm;
    uint64_t avail = s->avail_in;
    bool closed = false;
    if (g->mode == M_RUNNING) {
        const uint64_t text = g->blk.size() + avail;
        if (text < 2ull * g->nblock_max) return;                // at most one block closes: code it when it does
        const uint64_t nbk = text / g->nblock_max + 2;
        const uint64_t worst = text + text / 3 + 1024 * nbk;    // > any bzip2 output of that text
        if ((uint64_t)s->avail_out + g->out_pos < g->released + worst) return;   // the library might stop early
        avail = std::min<uint64_t>(avail, kAhead);
    } else {
        avail = g->expect;
        if (g->blk.size() + avail < g->nblock_max && avail) return;   // one block: coded at the flush anyway
        if (avail <= kAhead) closed = true;
        else avail = kAhead;
    }
    code_text(g, g->blk.data(), g->blk.size(), reinterpret_cast<const uint8_t*>(s->next_in), avail, g->blk_beg,
              closed);
}

// copy_input_until_stop (bz:bzlib.c:297-338)
bool copy_input(GpuStreamState* g)
{
    bz_stream* s = g->strm;
    const bool running = g->mode == M_RUNNING;
    uint64_t lim = s->avail_in;
    if (!running) lim = std::min<uint64_t>(lim, g->expect);
    if (lim == 0 || g->nblock >= g->nblock_max) return false;
    const uint8_t* p = reinterpret_cast<const uint8_t*>(s->next_in);
    uint64_t took;
    if (!g->ahead.empty() && g->ahead.front().beg == g->blk_beg) {
        // the block's end is known: consume to its closing byte (or the end)
        const Coded& c = g->ahead.front();
        const uint64_t target = c.flushed ? c.end : c.end + 1;
        took = std::min<uint64_t>(lim, target - g->consumed);
        if (took && g->consumed + took == target) {   // the rest of the block, all in this call: counted, not copied
            if (g->virt) throw StarchError(-10, "bzlib: counted block bytes left over");
            g->virt = took;
            g->virt_last = p[took - 1];
            g->virt_src = p;
        } else {
            g->blk.insert(g->blk.end(), p, p + took);
        }
        if (g->consumed + took == target) {
            // closed by nblockMAX: full, its closing byte pending; flushed:
            // the committed input is in (the flush follows at once)
            g->in_ch = g->virt ? g->virt_last : g->blk.back();
            g->in_len = 1;
            g->nblock = c.flushed ? 0u : g->nblock_max;
        } else {
            retrack(g);
        }
    } else {
        took = track(g, p, lim);
        g->blk.insert(g->blk.end(), p, p + took);
    }
    s->next_in += took;
    s->avail_in -= (unsigned)took;
    add_in(s, took);
    g->consumed += took;
    if (!running) g->expect -= (uint32_t)took;
    return took > 0;
}

// copy_output_until_stop (bz:bzlib.c:342-365)
bool drain(GpuStreamState* g)
{
    bz_stream* s = g->strm;
    uint64_t left = g->released - g->out_pos;
    uint64_t k = left < s->avail_out ? left : s->avail_out;
    if (k) {
        memcpy(s->next_out, g->output.data() + (g->out_pos - g->out_base), k);
        s->next_out += k;
        s->avail_out -= (unsigned)k;
        g->out_pos += k;
        add_out(s, k);
    }
    const uint64_t dr = g->out_pos - g->out_base;
    if (dr > (1u << 20) && 2 * dr > g->output.size()) {   // drop the drained prefix (amortised: at most the kept half moves)
        const size_t keep = g->output.size() - dr;
        if (keep) memmove(g->output.data(), g->output.data() + dr, keep);
        g->output.resize(keep);
        g->out_base = g->out_pos;
    }
    return k > 0;
}

// handle_compress (bz:bzlib.c:369-412)
bool handle_compress(GpuStreamState* g)
{
    bz_stream* s = g->strm;
    bool pin = false, pout = false;
    for (;;) {
        if (g->state == S_OUTPUT) {
            pout |= drain(g);
            if (g->out_pos < g->released) break;
            if (g->mode == M_FINISHING && g->expect == 0 && empty_rl(g)) break;
            g->state = S_INPUT;                          // prepare_new_block
            if (g->mode == M_FLUSHING && g->expect == 0 && empty_rl(g)) break;
        }
        if (g->state == S_INPUT) {
            code_ahead(g);
            pin |= copy_input(g);
            if (g->mode != M_RUNNING && g->expect == 0) {
                compress_block(g, true, g->mode == M_FINISHING);
                g->state = S_OUTPUT;
            } else if (g->nblock >= g->nblock_max) {
                compress_block(g, false, false);
                g->state = S_OUTPUT;
            } else if (s->avail_in == 0) {
                break;
            }
        }
    }
    return pin || pout;
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
    g->nblock_max = 100000u * (uint32_t)blockSize100k - 19u;   // bz:bzlib.c:194
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
    TraceSpan span(g_tr_all);
    try {
        for (;;) {   // preswitch (bz:bzlib.c:420-471)
            switch (g->mode) {
                case M_IDLE:
                    return BZ_SEQUENCE_ERROR;
                case M_RUNNING:
                    if (action == BZ_RUN) {
                        const bool progress = handle_compress(g);
                        if (!g->ahead.empty()) { g->ahead.clear(); g->enc.clear(); }   // BZ_RUN input is not committed
                        return progress ? BZ_RUN_OK : BZ_PARAM_ERROR;                 // bz:bzlib.c:432-434
                    }
                    if (action == BZ_FLUSH || action == BZ_FINISH) {
                        g->expect = strm->avail_in;
                        g->mode = action == BZ_FLUSH ? M_FLUSHING : M_FINISHING;
                        continue;
                    }
                    return BZ_PARAM_ERROR;
                case M_FLUSHING: {
                    if (action != BZ_FLUSH) return BZ_SEQUENCE_ERROR;
                    if (g->expect != strm->avail_in) return BZ_SEQUENCE_ERROR;
                    handle_compress(g);
                    if (g->expect > 0 || !empty_rl(g) || g->out_pos < g->released) return BZ_FLUSH_OK;
                    g->mode = M_RUNNING;
                    return BZ_RUN_OK;
                }
                case M_FINISHING: {
                    if (action != BZ_FINISH) return BZ_SEQUENCE_ERROR;
                    if (g->expect != strm->avail_in) return BZ_SEQUENCE_ERROR;
                    if (!handle_compress(g)) return BZ_SEQUENCE_ERROR;
                    if (g->expect > 0 || !empty_rl(g) || g->out_pos < g->released) return BZ_FINISH_OK;
                    g->mode = M_IDLE;
                    g->ahead.clear();
                    g->enc.release();
                    std::vector<uint8_t>().swap(g->blk);
                    if (strm->block_close_functor) strm->block_close_functor(strm->handler);   // bz:bzlib.c:470
                    return BZ_STREAM_END;
                }
                default:
                    return BZ_SEQUENCE_ERROR;   // a GPU failure ended the stream
            }
        }
    } catch (const std::exception&) {
        g->mode = M_FAILED;
        return BZ_CONFIG_ERROR;
    }
}

int BZ2_bzCompressEnd(bz_stream* strm)
{
    GpuStreamState* g = state_of(strm);
    if (!g) return BZ_PARAM_ERROR;
    if (bz_trace())
        fprintf(stderr, "bz trace: BZ2_bzCompress %.1f ms, of which GPU coding (code_text) %.1f ms (all threads)\n",
                g_tr_all.load() / 1e6, g_tr_code.load() / 1e6);
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
