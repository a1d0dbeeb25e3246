// starch_amd/csrc/starch_api.hip -- the C ABI (include/starch_amd.h) and the
// archive writer.  Host orchestration only: every byte of the transform and
// of the bzip2 streams is produced by the HIP kernels in this directory.
#include <string.h>

#include <string>
#include <vector>

#include "../../include/starch_amd.h"
#include "bz2.hpp"
#include "transform.hpp"

struct starch_ctx {
    int device = 0;
    hipStream_t own = nullptr;
    hipStream_t st = nullptr;
    TransformWorkspace tf;
    bz::Encoder enc;
    DevBuf input, archive, raw_in, raw_out;
    std::string err;
    // last result
    bool have = false;
    uint64_t archive_bytes = 0;
    uint64_t text_bytes = 0;
    std::vector<starch_segment> segs;
    std::vector<std::string> names;
    starch_stats stats{};
};

namespace {

int fail(starch_ctx* c, const StarchError& e)
{
    if (c) c->err = e.what();
    return e.code;
}

struct Ctx {   // device guard
    int prev = -1;
    explicit Ctx(starch_ctx* c) { (void)hipGetDevice(&prev); (void)hipSetDevice(c->device); }
    ~Ctx() { if (prev >= 0) (void)hipSetDevice(prev); }
};

bool valid_utf8(const unsigned char* s, size_t n)
{
    for (size_t i = 0; i < n;) {
        unsigned char c = s[i];
        int k = c < 0x80 ? 0 : (c >> 5) == 6 ? 1 : (c >> 4) == 14 ? 2 : (c >> 3) == 30 ? 3 : -1;
        if (k < 0 || i + k >= n + (k == 0 ? 1 : 0)) return false;
        for (int j = 1; j <= k; ++j) if (i + j >= n || (s[i + j] & 0xc0) != 0x80) return false;
        i += 1 + k;
    }
    return true;
}

// Chromosome names are arbitrary bytes: escaped byte-wise as \u00XX so the
// original bytes are recovered as latin-1 code points.  Free text (the note)
// that is valid UTF-8 is kept as UTF-8.
void json_str(std::string& o, const char* p, size_t n, bool keep_utf8 = false)
{
    static const char* hx = "0123456789abcdef";
    const bool raw_hi = keep_utf8 && valid_utf8(reinterpret_cast<const unsigned char*>(p), n);
    o += '"';
    for (size_t i = 0; i < n; ++i) {
        unsigned char c = (unsigned char)p[i];
        if (c == '"') o += "\\\"";
        else if (c == '\\') o += "\\\\";
        else if (c >= 0x80 && raw_hi) o += (char)c;
        else if (c < 0x20 || c >= 0x7f) {   // control and non-ASCII bytes as latin-1 code points
            o += "\\u00";
            o += hx[c >> 4];
            o += hx[c & 15];
        } else o += (char)c;
    }
    o += '"';
}

std::string build_index(const starch_segment* segs, const char* const* names, const uint64_t* nlens, uint64_t nseg,
                        uint64_t index_off, const char* note, int bs)
{
    std::string j;
    j += "{\"archive\":{\"type\":\"starch\",\"format\":\"starch3-mi355x\",\"version\":{\"major\":3,\"minor\":0,"
         "\"revision\":0},\"compressionFormat\":\"bzip2\",\"blockSize100k\":";
    j += std::to_string(bs);
    j += ",\"note\":";
    json_str(j, note ? note : "", note ? strlen(note) : 0, true);
    j += "},\"streams\":[";
    for (uint64_t s = 0; s < nseg; ++s) {
        if (s) j += ',';
        j += "{\"chromosome\":";
        json_str(j, names[s], nlens[s]);
        j += ",\"offset\":" + std::to_string(segs[s].stream_offset);
        j += ",\"size\":" + std::to_string(segs[s].stream_bytes);
        j += ",\"uncompressedLineCount\":" + std::to_string(segs[s].line_count);
        j += ",\"transformedBytes\":" + std::to_string(segs[s].text_bytes);
        j += ",\"blocks\":" + std::to_string(segs[s].n_blocks);
        j += ",\"combinedCRC\":" + std::to_string(segs[s].combined_crc);
        j += '}';
    }
    j += "]}";
    // 32-byte footer: zero-padded decimal offset of the index, then padding + '\n'
    char foot[40];
    snprintf(foot, sizeof(foot), "%020llu", (unsigned long long)index_off);
    std::string f(foot);
    f.append(31 - f.size(), ' ');
    f += '\n';
    return j + f;
}

uint64_t align_up(uint64_t x, uint64_t a) { return (x + a - 1) / a * a; }

// transform + bzip2 + archive into ctx->archive (device)
void encode_device(starch_ctx* c, const uint8_t* d_bed, uint64_t n, const starch_options& opt)
{
    hipEvent_t e0, e1, e2;
    HIP_CHECK(hipEventCreate(&e0));
    HIP_CHECK(hipEventCreate(&e1));
    HIP_CHECK(hipEventCreate(&e2));
    HIP_CHECK(hipEventRecord(e0, c->st));
    c->have = false;
    c->stats = starch_stats{};
    c->stats.input_bytes = n;
    TransformResult tr;
    c->tf.run(d_bed, n, c->st, tr);
    HIP_CHECK(hipEventRecord(e1, c->st));
    std::vector<SegInfo> si(tr.n_segments);
    if (tr.n_segments)
        HIP_CHECK(hipMemcpyAsync(si.data(), c->tf.seg_info_dev, tr.n_segments * sizeof(SegInfo),
                                 hipMemcpyDeviceToHost, c->st));
    HIP_CHECK(hipStreamSynchronize(c->st));
    c->stats.n_lines = tr.n_lines;
    c->stats.n_segments = tr.n_segments;
    c->stats.text_bytes = tr.text_bytes;
    c->text_bytes = tr.text_bytes;
    // segment names (small host copies of the chr tokens)
    c->names.assign(tr.n_segments, std::string());
    for (uint64_t s = 0; s < tr.n_segments; ++s) {
        c->names[s].resize(si[s].name_len);
        if (si[s].name_len)
            HIP_CHECK(hipMemcpyAsync(&c->names[s][0], d_bed + si[s].name_off, si[s].name_len, hipMemcpyDeviceToHost,
                                     c->st));
    }
    c->segs.assign(tr.n_segments, starch_segment{});
    const uint64_t magic = 4;
    if (opt.reference_compat) {   // the reference writes only the magic (hpp:765-769)
        uint8_t* out = c->archive.as<uint8_t>(64);
        static const uint8_t mb[4] = {0xca, 0x5c, 0xad, 0x1a};
        HIP_CHECK(hipMemcpyAsync(out, mb, 4, hipMemcpyHostToDevice, c->st));
        HIP_CHECK(hipStreamSynchronize(c->st));
        c->archive_bytes = 4;
        for (uint64_t s = 0; s < tr.n_segments; ++s) {
            c->segs[s].line_count = si[s].line_count;
            c->segs[s].text_bytes = si[s].text_len;
            c->segs[s].name_len = si[s].name_len;
        }
        c->have = true;
        return;
    }
    std::vector<bz::StreamIn> sin(tr.n_segments);
    for (uint64_t s = 0; s < tr.n_segments; ++s) {
        sin[s].text_off = si[s].text_off;
        sin[s].text_len = si[s].text_len;
        sin[s].final_run_joins = 1;
        sin[s].group = (uint32_t)s;
    }
    std::vector<bz::StreamOut> outs;
    bz::Stats bst;
    c->enc.plan(c->tf.text, sin, opt.block_size_100k, c->st, outs, &bst);
    uint64_t streams_bytes = 0;
    for (auto& o : outs) streams_bytes = std::max(streams_bytes, o.out_off + o.bytes);
    for (uint64_t s = 0; s < tr.n_segments; ++s) {
        starch_segment& g = c->segs[s];
        g.line_count = si[s].line_count;
        g.text_bytes = si[s].text_len;
        g.stream_offset = magic + outs[s].out_off;
        g.stream_bytes = outs[s].bytes;
        g.name_len = si[s].name_len;
        g.n_blocks = outs[s].n_blocks;
    }
    // combined CRCs are known after emit; compute the index afterwards
    const uint64_t index_off = magic + streams_bytes;
    const uint64_t cap = align_up(index_off + 4 + (opt.emit_index ? 256 + 256 * tr.n_segments + 64 : 0) +
                                      [&] { uint64_t t = 0; for (auto& nm : c->names) t += 6 * nm.size(); return t; }() +
                                      (opt.note ? 6 * strlen(opt.note) : 0),
                                  256);
    uint8_t* out = c->archive.as<uint8_t>(cap);
    static const uint8_t mb[4] = {0xca, 0x5c, 0xad, 0x1a};
    HIP_CHECK(hipMemcpyAsync(out, mb, 4, hipMemcpyHostToDevice, c->st));
    c->enc.emit(out, cap, magic, outs, c->st, &bst);
    for (uint64_t s = 0; s < tr.n_segments; ++s) c->segs[s].combined_crc = outs[s].combined_crc;
    uint64_t total = index_off;
    std::string idx;
    if (opt.emit_index) {
        std::vector<const char*> np(tr.n_segments);
        std::vector<uint64_t> nl(tr.n_segments);
        for (uint64_t s = 0; s < tr.n_segments; ++s) { np[s] = c->names[s].data(); nl[s] = c->names[s].size(); }
        idx = build_index(c->segs.data(), np.data(), nl.data(), tr.n_segments, index_off, opt.note,
                          opt.block_size_100k);
        if (index_off + idx.size() > cap) throw StarchError(STARCH_ERR_INTERNAL, "index capacity");
        HIP_CHECK(hipMemcpyAsync(out + index_off, idx.data(), idx.size(), hipMemcpyHostToDevice, c->st));
        total += idx.size();
    }
    HIP_CHECK(hipEventRecord(e2, c->st));
    HIP_CHECK(hipStreamSynchronize(c->st));
    float ms_t = 0, ms_all = 0;
    HIP_CHECK(hipEventElapsedTime(&ms_t, e0, e1));
    HIP_CHECK(hipEventElapsedTime(&ms_all, e0, e2));
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    (void)hipEventDestroy(e2);
    c->archive_bytes = total;
    c->stats.archive_bytes = total;
    c->stats.n_blocks = bst.n_blocks;
    c->stats.rle_bytes = bst.rle_bytes;
    c->stats.bwt_rounds = bst.bwt_rounds;
    c->stats.periodic_blocks = bst.periodic_blocks;
    c->stats.bwt_tied = bst.bwt_tied;
    c->stats.dedup_blocks = bst.dedup_blocks;
    c->stats.ms_transform = ms_t;
    c->stats.ms_rle = bst.rle;
    c->stats.ms_bwt = bst.bwt;
    c->stats.ms_mtf = bst.mtf;
    c->stats.ms_tables = bst.tables;
    c->stats.ms_emit = bst.emit;
    c->stats.ms_total = ms_all;
    c->have = true;
}

}  // namespace

#define GUARD(c)                                         \
    if (!(c)) return STARCH_ERR_ARG;                     \
    try {                                                \
        Ctx _g(c);
#define END_GUARD(c)                                     \
    }                                                    \
    catch (const StarchError& e) { return fail(c, e); }  \
    catch (const std::exception& e) { (c)->err = e.what(); return STARCH_ERR_INTERNAL; }

extern "C" {

int starch_version(void) { return 0x000100; }

const char* starch_strerror(int code)
{
    switch (code) {
        case STARCH_OK: return "ok";
        case STARCH_ERR_ARG: return "invalid argument";
        case STARCH_ERR_MEM: return "out of memory or buffer too small";
        case STARCH_ERR_STATE: return "no result available";
        case STARCH_ERR_DEVICE: return "HIP device error";
        default: return "internal error";
    }
}

const char* starch_last_error(starch_ctx* ctx) { return ctx ? ctx->err.c_str() : "no context"; }

int starch_create(int device, starch_ctx** out)
{
    if (!out) return STARCH_ERR_ARG;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0 || device < 0 || device >= n) return STARCH_ERR_DEVICE;
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, device) != hipSuccess) return STARCH_ERR_DEVICE;
    if (strncmp(p.gcnArchName, "gfx950", 6) != 0) return STARCH_ERR_DEVICE;   // code objects are gfx950-only
    starch_ctx* c = new starch_ctx();
    c->device = device;
    int prev = 0;
    (void)hipGetDevice(&prev);
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return STARCH_ERR_DEVICE;
    }
    (void)hipSetDevice(prev);
    c->st = c->own;
    *out = c;
    return STARCH_OK;
}

void starch_destroy(starch_ctx* c)
{
    if (!c) return;
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->st);
    if (c->own) (void)hipStreamDestroy(c->own);
    delete c;
}

int starch_set_stream(starch_ctx* c, void* s)
{
    if (!c) return STARCH_ERR_ARG;
    c->st = s ? static_cast<hipStream_t>(s) : c->own;
    return STARCH_OK;
}

void starch_options_init(starch_options* o)
{
    if (!o) return;
    o->block_size_100k = 9;
    o->emit_index = 1;
    o->reference_compat = 0;
    o->note = nullptr;
}

int starch_encode_device(starch_ctx* c, const void* d_bed, uint64_t n, const starch_options* opt)
{
    GUARD(c)
    starch_options o;
    starch_options_init(&o);
    if (opt) o = *opt;
    if (o.block_size_100k < 1 || o.block_size_100k > 9) return STARCH_ERR_ARG;
    if (n && !d_bed) return STARCH_ERR_ARG;
    encode_device(c, static_cast<const uint8_t*>(d_bed), n, o);
    return STARCH_OK;
    END_GUARD(c)
}

int starch_encode_host(starch_ctx* c, const void* bed, uint64_t n, const starch_options* opt)
{
    GUARD(c)
    if (n && !bed) return STARCH_ERR_ARG;
    uint8_t* d = c->input.as<uint8_t>(n + 64);
    if (n) HIP_CHECK(hipMemcpyAsync(d, bed, n, hipMemcpyHostToDevice, c->st));
    HIP_CHECK(hipStreamSynchronize(c->st));
    starch_options o;
    starch_options_init(&o);
    if (opt) o = *opt;
    if (o.block_size_100k < 1 || o.block_size_100k > 9) return STARCH_ERR_ARG;
    encode_device(c, d, n, o);
    return STARCH_OK;
    END_GUARD(c)
}

int starch_archive_size(starch_ctx* c, uint64_t* n)
{
    if (!c || !n) return STARCH_ERR_ARG;
    if (!c->have) return STARCH_ERR_STATE;
    *n = c->archive_bytes;
    return STARCH_OK;
}

int starch_archive_device(starch_ctx* c, const void** p)
{
    if (!c || !p) return STARCH_ERR_ARG;
    if (!c->have) return STARCH_ERR_STATE;
    *p = c->archive.p;
    return STARCH_OK;
}

int starch_archive_copy(starch_ctx* c, void* dst, uint64_t cap)
{
    GUARD(c)
    if (!c->have) return STARCH_ERR_STATE;
    if (cap < c->archive_bytes || !dst) return STARCH_ERR_MEM;
    if (c->archive_bytes)
        HIP_CHECK(hipMemcpyAsync(dst, c->archive.p, c->archive_bytes, hipMemcpyDeviceToHost, c->st));
    HIP_CHECK(hipStreamSynchronize(c->st));
    return STARCH_OK;
    END_GUARD(c)
}

int starch_segment_count(starch_ctx* c, uint64_t* n)
{
    if (!c || !n) return STARCH_ERR_ARG;
    if (!c->have) return STARCH_ERR_STATE;
    *n = c->segs.size();
    return STARCH_OK;
}

int starch_segments(starch_ctx* c, starch_segment* out, uint64_t cap)
{
    if (!c || (!out && cap)) return STARCH_ERR_ARG;
    if (!c->have) return STARCH_ERR_STATE;
    if (cap < c->segs.size()) return STARCH_ERR_MEM;
    if (!c->segs.empty()) memcpy(out, c->segs.data(), c->segs.size() * sizeof(starch_segment));
    return STARCH_OK;
}

int starch_segment_name(starch_ctx* c, uint64_t i, char* buf, uint64_t cap, uint64_t* len)
{
    if (!c) return STARCH_ERR_ARG;
    if (!c->have) return STARCH_ERR_STATE;
    if (i >= c->names.size()) return STARCH_ERR_ARG;
    const std::string& s = c->names[i];
    if (len) *len = s.size();
    if (buf) {
        if (cap < s.size()) return STARCH_ERR_MEM;
        memcpy(buf, s.data(), s.size());
    }
    return STARCH_OK;
}

int starch_get_stats(starch_ctx* c, starch_stats* out)
{
    if (!c || !out) return STARCH_ERR_ARG;
    *out = c->stats;
    return STARCH_OK;
}

int starch_transform_host(starch_ctx* c, const void* bed, uint64_t n)
{
    GUARD(c)
    if (n && !bed) return STARCH_ERR_ARG;
    uint8_t* d = c->input.as<uint8_t>(n + 64);
    if (n) HIP_CHECK(hipMemcpyAsync(d, bed, n, hipMemcpyHostToDevice, c->st));
    TransformResult tr;
    c->tf.run(d, n, c->st, tr);
    std::vector<SegInfo> si(tr.n_segments);
    if (tr.n_segments)
        HIP_CHECK(hipMemcpyAsync(si.data(), c->tf.seg_info_dev, tr.n_segments * sizeof(SegInfo),
                                 hipMemcpyDeviceToHost, c->st));
    HIP_CHECK(hipStreamSynchronize(c->st));
    c->segs.assign(tr.n_segments, starch_segment{});
    c->names.assign(tr.n_segments, std::string());
    const uint8_t* hb = static_cast<const uint8_t*>(bed);
    for (uint64_t s = 0; s < tr.n_segments; ++s) {
        c->segs[s].line_count = si[s].line_count;
        c->segs[s].text_bytes = si[s].text_len;
        c->segs[s].stream_offset = si[s].text_off;   // transform-only: offset into the text
        c->segs[s].name_len = si[s].name_len;
        c->names[s].assign(reinterpret_cast<const char*>(hb + si[s].name_off), si[s].name_len);
    }
    c->text_bytes = tr.text_bytes;
    c->archive_bytes = 0;
    c->have = true;
    return STARCH_OK;
    END_GUARD(c)
}

int starch_text_size(starch_ctx* c, uint64_t* n)
{
    if (!c || !n) return STARCH_ERR_ARG;
    if (!c->have) return STARCH_ERR_STATE;
    *n = c->text_bytes;
    return STARCH_OK;
}

int starch_text_copy(starch_ctx* c, void* dst, uint64_t cap)
{
    GUARD(c)
    if (!c->have) return STARCH_ERR_STATE;
    if (cap < c->text_bytes) return STARCH_ERR_MEM;
    if (c->text_bytes) HIP_CHECK(hipMemcpyAsync(dst, c->tf.text, c->text_bytes, hipMemcpyDeviceToHost, c->st));
    HIP_CHECK(hipStreamSynchronize(c->st));
    return STARCH_OK;
    END_GUARD(c)
}

int starch_bz2_compress_many_device(starch_ctx* c, const void* d_in, const uint64_t* offs, const uint64_t* lens,
                                    uint64_t nstreams, int bs, void* d_out, uint64_t cap, uint64_t* out_offs,
                                    uint64_t* out_lens)
{
    GUARD(c)
    if (bs < 1 || bs > 9 || (nstreams && (!offs || !lens || !out_offs || !out_lens))) return STARCH_ERR_ARG;
    std::vector<bz::StreamIn> sin(nstreams);
    for (uint64_t s = 0; s < nstreams; ++s) {
        sin[s].text_off = offs[s];
        sin[s].text_len = lens[s];
        sin[s].final_run_joins = 1;
        sin[s].group = (uint32_t)s;
    }
    std::vector<bz::StreamOut> outs;
    c->enc.plan_and_encode(static_cast<const uint8_t*>(d_in), sin, bs, static_cast<uint8_t*>(d_out), cap, 0, outs,
                           c->st, nullptr);
    HIP_CHECK(hipStreamSynchronize(c->st));
    for (uint64_t s = 0; s < nstreams; ++s) { out_offs[s] = outs[s].out_off; out_lens[s] = outs[s].bytes; }
    return STARCH_OK;
    END_GUARD(c)
}

int starch_bz2_compress_host(starch_ctx* c, const void* in, uint64_t n, int bs, void* out, uint64_t cap,
                             uint64_t* out_len)
{
    GUARD(c)
    if (bs < 1 || bs > 9 || !out_len || (n && !in)) return STARCH_ERR_ARG;
    uint8_t* d = c->raw_in.as<uint8_t>(n + 64);
    if (n) HIP_CHECK(hipMemcpyAsync(d, in, n, hipMemcpyHostToDevice, c->st));
    uint64_t ocap = n + n / 50 + 4096;
    uint8_t* dout = c->raw_out.as<uint8_t>(ocap);
    uint64_t off = 0, len = 0, zero = 0;
    int rc = starch_bz2_compress_many_device(c, d, &zero, &n, 1, bs, dout, ocap, &off, &len);
    if (rc) return rc;
    *out_len = len;
    if (cap < len) return STARCH_ERR_MEM;
    HIP_CHECK(hipMemcpyAsync(out, dout + off, len, hipMemcpyDeviceToHost, c->st));
    HIP_CHECK(hipStreamSynchronize(c->st));
    return STARCH_OK;
    END_GUARD(c)
}

int starch_build_index(const starch_segment* segs, const char* const* names, const uint64_t* name_lens,
                       uint64_t nseg, uint64_t index_offset, const char* note, int bs, char* dst, uint64_t cap,
                       uint64_t* len)
{
    if (!len || (nseg && (!segs || !names || !name_lens))) return STARCH_ERR_ARG;
    std::string s = build_index(segs, names, name_lens, nseg, index_offset, note, bs);
    *len = s.size();
    if (!dst) return STARCH_OK;
    if (cap < s.size()) return STARCH_ERR_MEM;
    memcpy(dst, s.data(), s.size());
    return STARCH_OK;
}

}  // extern "C"
