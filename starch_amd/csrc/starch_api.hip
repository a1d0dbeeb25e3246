// starch_amd/csrc/starch_api.hip -- the C ABI (include/starch_amd.h) and the
// archive writer.  Host orchestration only: every byte of the transform and
// of the bzip2 streams is produced by the HIP kernels in this directory.
#include <string.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "ctx.hpp"
#include "shard.hpp"

namespace archive {
const uint8_t kMagic[4] = {0xca, 0x5c, 0xad, 0x1a};   // hpp:907-910
}  // namespace archive

namespace {

// STARCH_TRACE=1: host-side timeline of the batched paths on stderr
double trace_t0()
{
    static const auto t0 = std::chrono::steady_clock::now();
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}
bool tracing()
{
    static const bool on = getenv("STARCH_TRACE") != nullptr;
    return on;
}
#define STRACE(...)                                                              \
    do {                                                                         \
        if (tracing()) {                                                         \
            fprintf(stderr, "[starch %9.3f ms] ", trace_t0());                   \
            fprintf(stderr, __VA_ARGS__);                                        \
            fputc('\n', stderr);                                                \
        }                                                                        \
    } while (0)

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

}  // namespace

std::string archive::build_index(const starch_segment* segs, const char* const* names, const uint64_t* nlens, uint64_t nseg,
                        uint64_t index_off, const char* note, int bs, bool base_counts, int method)
{
    std::string j;
    j += "{\"archive\":{\"type\":\"starch\",\"format\":\"starch3-mi355x\",\"version\":{\"major\":3,\"minor\":0,"
         "\"revision\":0},\"compressionFormat\":";
    j += method == STARCH_METHOD_GZIP ? "\"gzip\",\"blockSize100k\":" : "\"bzip2\",\"blockSize100k\":";
    j += std::to_string(method == STARCH_METHOD_GZIP ? 0 : bs);
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
        if (base_counts) {   // hpp:61-62
            j += ",\"uniqueBaseCount\":" + std::to_string(segs[s].base_count_unique);
            j += ",\"nonUniqueBaseCount\":" + std::to_string(segs[s].base_count_nonunique);
        }
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


namespace {

uint64_t align_up(uint64_t x, uint64_t a) { return (x + a - 1) / a * a; }

using archive::build_index;
using archive::kMagic;

struct UnitIn {
    uint64_t off, len;           // byte range relative to the device base pointer
    int64_t init_start, init_stop;
    uint64_t id;                 // global unit index (archive order)
};

// chr token of the last line before `j` and of the line at `j`, read from small
// device windows; false when a line does not fit the window (the caller then
// takes the exact per-unit route)
bool junction_differs(starch_ctx* c, const uint8_t* d_base, uint64_t lo, uint64_t j, uint64_t hi)
{
    const uint64_t W = 1024;
    uint8_t a[W], b[W];
    const uint64_t a0 = (j - lo > W) ? j - W : lo, an = j - a0;
    const uint64_t bn = std::min<uint64_t>(W, hi - j);
    if (an) HIP_CHECK(hipMemcpyAsync(a, d_base + a0, an, hipMemcpyDeviceToHost, c->st));
    if (bn) HIP_CHECK(hipMemcpyAsync(b, d_base + j, bn, hipMemcpyDeviceToHost, c->st));
    HIP_CHECK(hipStreamSynchronize(c->st));
    if (an == 0 || bn == 0) return false;
    // previous line: [ls, an) in a (a[an-1] is its '\n')
    uint64_t ls = an - 1;
    while (ls > 0 && a[ls - 1] != '\n') --ls;
    if (ls == 0 && a0 > lo) return false;
    auto tok = [](const uint8_t* x, uint64_t beg, uint64_t n, bool complete, uint64_t* len) {
        uint64_t p = beg;
        while (p < n && x[p] != '\t' && x[p] != '\n') ++p;
        if (p == n && !complete) return false;
        uint64_t e = (p < n && x[p] == '\n') ? p + 1 : p;
        const void* z = memchr(x + beg, 0, e - beg);
        *len = z ? (uint64_t)(static_cast<const uint8_t*>(z) - (x + beg)) : e - beg;
        return true;
    };
    uint64_t la = 0, lb = 0;
    if (!tok(a, ls, an, true, &la) || !tok(b, 0, bn, j + bn >= hi, &lb)) return false;
    return la != lb || memcmp(a + ls, b, la) != 0;
}

struct FFInBatch {};   // transform_units(planned): the batch holds a 0xFF (hpp:181: EOF)

// Transform stage over units.  One launch sequence over the whole range when
// the units are back to back, every junction changes chromosome (so it is a
// segment start in the concatenation too) and no sscanf value goes stale;
// otherwise each unit runs on its own with its initial values.  Fills the host
// segment table (name_off relative to d_base, text_off into the returned text)
// and the unit of every segment.
const uint8_t* transform_units(starch_ctx* c, const uint8_t* d_base, const std::vector<UnitIn>& u,
                               std::vector<SegInfo>& si, std::vector<uint64_t>& unit_of, uint64_t& text_bytes,
                               uint64_t& n_lines, bool planned = false)
{
    si.clear();
    unit_of.clear();
    text_bytes = n_lines = 0;
    if (u.empty()) return nullptr;
    bool joint = true;
    for (size_t k = 1; k < u.size() && joint; ++k) joint = u[k].off == u[k - 1].off + u[k - 1].len;
    // units from shard::plan_units start a new chromosome by construction
    for (size_t k = 1; k < u.size() && joint && !planned; ++k)
        if (u[k].len && u[k - 1].len) joint = junction_differs(c, d_base, u[k - 1].off, u[k].off, u[k].off + u[k].len);
    if (joint) {
        const uint64_t beg = u[0].off, end = u.back().off + u.back().len;
        TransformResult tr;
        c->tf.run(d_base + beg, end - beg, c->st, tr, u[0].init_start, u[0].init_stop);
        if (planned && tr.ff_pos != ~0ull) throw FFInBatch{};
        if (u.size() > 1 && tr.ff_pos != ~0ull)
            throw StarchError(STARCH_ERR_ARG, "a unit contains byte 0xFF (plan units with starch_plan_units)");
        if (u.size() == 1 || !tr.general) {
            si.resize(tr.n_segments);
            if (tr.n_segments)
                HIP_CHECK(hipMemcpyAsync(si.data(), c->tf.seg_info_dev, tr.n_segments * sizeof(SegInfo),
                                         hipMemcpyDeviceToHost, c->st));
            HIP_CHECK(hipStreamSynchronize(c->st));
            unit_of.resize(si.size());
            size_t k = 0;
            for (size_t s = 0; s < si.size(); ++s) {
                si[s].name_off += beg;
                while (k + 1 < u.size() && si[s].name_off >= u[k + 1].off) ++k;
                unit_of[s] = u[k].id;
            }
            text_bytes = tr.text_bytes;
            n_lines = tr.n_lines;
            return c->tf.text;
        }
    }
    // exact per-unit route: each unit with the sscanf values current before it
    uint8_t* all = static_cast<uint8_t*>(c->text_all.p);   // staging text of all units
    uint64_t cap = c->text_all.cap;
    for (size_t k = 0; k < u.size(); ++k) {
        TransformResult tr;
        c->tf.run(d_base + u[k].off, u[k].len, c->st, tr, u[k].init_start, u[k].init_stop);
        if (planned && tr.ff_pos != ~0ull) throw FFInBatch{};
        if (tr.ff_pos != ~0ull)
            throw StarchError(STARCH_ERR_ARG, "a unit contains byte 0xFF (plan units with starch_plan_units)");
        std::vector<SegInfo> part(tr.n_segments);
        if (tr.n_segments)
            HIP_CHECK(hipMemcpyAsync(part.data(), c->tf.seg_info_dev, tr.n_segments * sizeof(SegInfo),
                                     hipMemcpyDeviceToHost, c->st));
        if (text_bytes + tr.text_bytes + 64 > cap) {   // grow the staging text, keeping what it holds
            const uint64_t ncap = std::max<uint64_t>(2 * cap, text_bytes + tr.text_bytes + 64);
            DevBuf nb;
            uint8_t* np = nb.as<uint8_t>(ncap);
            if (text_bytes) HIP_CHECK(hipMemcpyAsync(np, all, text_bytes, hipMemcpyDeviceToDevice, c->st));
            HIP_CHECK(hipStreamSynchronize(c->st));
            std::swap(c->text_all.p, nb.p);
            std::swap(c->text_all.cap, nb.cap);
            all = np;
            cap = ncap;
        }
        if (tr.text_bytes)
            HIP_CHECK(hipMemcpyAsync(all + text_bytes, c->tf.text, tr.text_bytes, hipMemcpyDeviceToDevice, c->st));
        HIP_CHECK(hipStreamSynchronize(c->st));
        for (auto& g : part) {
            g.name_off += u[k].off;
            g.text_off += text_bytes;
            g.first_line += n_lines;
            si.push_back(g);
            unit_of.push_back(u[k].id);
        }
        text_bytes += tr.text_bytes;
        n_lines += tr.n_lines;
    }
    return all;
}

// Segment names (the chr tokens, in the input) -> c->names.  One gather
// kernel packs them into a device buffer and ONE copy brings them to pinned
// host memory (one copy per name costs a host round trip each: ~20 us per
// segment).  fetch_names issues the work on c->st; finish_names fills
// c->names once the stream has passed it (the caller syncs or waits on ev).
struct NameDesc { uint64_t src, dst, len; };

__global__ void k_gather_names(const uint8_t* __restrict__ base, const NameDesc* __restrict__ d, uint8_t* __restrict__ out)
{
    const NameDesc x = d[blockIdx.x];
    for (uint64_t i = threadIdx.x; i < x.len; i += blockDim.x) out[x.dst + i] = base[x.src + i];
}

struct PendingNames {
    std::vector<uint64_t> at;    // nseg + 1 offsets into the packed bytes
    const uint8_t* host = nullptr;
    hipEvent_t ev = nullptr;
    ~PendingNames() { if (ev) (void)hipEventDestroy(ev); }
};

void fetch_names(starch_ctx* c, const uint8_t* d_base, const std::vector<SegInfo>& si, PendingNames& pn)
{
    const uint64_t nseg = si.size();
    pn.at.assign(nseg + 1, 0);
    for (uint64_t s = 0; s < nseg; ++s) pn.at[s + 1] = pn.at[s] + si[s].name_len;
    const uint64_t total = pn.at[nseg];
    if (!total) return;
    uint8_t* hp = static_cast<uint8_t*>(c->names_pin.get(total + nseg * sizeof(NameDesc) + 64));
    NameDesc* hd = reinterpret_cast<NameDesc*>(hp + align_up(total, 64));
    for (uint64_t s = 0; s < nseg; ++s) hd[s] = NameDesc{si[s].name_off, pn.at[s], si[s].name_len};
    uint8_t* dp = c->names_dev.as<uint8_t>(align_up(total, 64) + nseg * sizeof(NameDesc));
    NameDesc* dd = reinterpret_cast<NameDesc*>(dp + align_up(total, 64));
    HIP_CHECK(hipMemcpyAsync(dd, hd, nseg * sizeof(NameDesc), hipMemcpyHostToDevice, c->st));
    hipLaunchKernelGGL(k_gather_names, dim3((unsigned)nseg), dim3(64), 0, c->st, d_base, dd, dp);
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipMemcpyAsync(hp, dp, total, hipMemcpyDeviceToHost, c->st));
    HIP_CHECK(hipEventCreateWithFlags(&pn.ev, hipEventDisableTiming));
    HIP_CHECK(hipEventRecord(pn.ev, c->st));
    pn.host = hp;
}

void finish_names(starch_ctx* c, PendingNames& pn)
{
    const uint64_t nseg = pn.at.empty() ? 0 : pn.at.size() - 1;
    c->names.assign(nseg, std::string());
    if (pn.ev) {
        HIP_CHECK(hipEventSynchronize(pn.ev));
        (void)hipEventDestroy(pn.ev);
        pn.ev = nullptr;
        for (uint64_t s = 0; s < nseg; ++s)
            c->names[s].assign(reinterpret_cast<const char*>(pn.host) + pn.at[s], pn.at[s + 1] - pn.at[s]);
    }
}

enum Layout { L_ARCHIVE, L_STREAMS };

// transform + bzip2 over units.  L_ARCHIVE: magic + streams + index in
// c->archive (the whole-input result); L_STREAMS: the streams alone, back to
// back from offset 0 of c->part (one shard of a multi-GPU run).
// Encoder lanes of a one-transform encode (STARCH_DEV_LANES, default 2): the
// segments split into contiguous runs of about equal text, each planned
// (RLE1 .. tables) by its own encoder on its own stream and host thread, so
// one lane's host round trips and the drain of its persistent kernels are
// filled by the other lanes' kernels.  Returns the first segment of every
// lane (empty: one lane).  Streams keep their order; the archive is the same
// bytes.
starch_ctx* lane_ctx(starch_ctx* c, int i);

std::vector<uint64_t> lane_cuts(const std::vector<SegInfo>& si, uint64_t tbytes, int want)
{
    static const int nl_env = [] { const char* e = getenv("STARCH_DEV_LANES"); return e ? atoi(e) : 2; }();
    const int nl_req = want > 0 ? want : nl_env;
    static const uint64_t min_b = [] {
        const char* e = getenv("STARCH_DEV_LANES_MIN");
        return e ? (uint64_t)atoll(e) : (uint64_t)(16ull << 20);
    }();
    const uint64_t nseg = si.size();
    const uint64_t nl = std::min<uint64_t>({(uint64_t)std::max(nl_req, 1), nseg, 8});
    std::vector<uint64_t> cuts;
    if (nl < 2 || tbytes < min_b) return cuts;
    cuts.push_back(0);
    uint64_t acc = 0, k = 0;
    for (uint64_t i = 1; i < nl; ++i) {
        const uint64_t target = tbytes * i / nl;   // lane i starts at the segment whose middle passes it
        while (k < nseg && 2 * acc + si[k].text_len < 2 * target) acc += si[k++].text_len;
        if (k <= cuts.back()) acc += si[k++].text_len;
        if (k >= nseg) break;
        cuts.push_back(k);
    }
    if (cuts.size() < 2) cuts.clear();
    return cuts;
}

void merge_counters(bz::Stats& a, const bz::Stats& b)
{
    a.n_blocks += b.n_blocks;
    a.rle_bytes += b.rle_bytes;
    a.bwt_rounds += b.bwt_rounds;
    a.periodic_blocks += b.periodic_blocks;
    a.bwt_tied += b.bwt_tied;
    a.dedup_blocks += b.dedup_blocks;
}

// per stage, the wall time during which any lane ran it (union of intervals)
void stage_union(const std::vector<bz::Encoder::Interval>& iv, bz::Stats& st)
{
    float* f[5] = {&st.rle, &st.bwt, &st.mtf, &st.tables, &st.emit};
    for (int k = 0; k < 5; ++k) {
        std::vector<std::pair<float, float>> x;
        for (auto& v : iv)
            if (v.stage == k) x.emplace_back(v.a, v.b);
        std::sort(x.begin(), x.end());
        float tot = 0, ca = 0, cb = -1e30f;
        for (auto& p : x) {
            if (p.first > cb) {
                if (cb > ca) tot += cb - ca;
                ca = p.first;
                cb = p.second;
            } else if (p.second > cb) {
                cb = p.second;
            }
        }
        if (cb > ca) tot += cb - ca;
        *f[k] = tot;
    }
}

void encode_units(starch_ctx* c, const uint8_t* d_base, const std::vector<UnitIn>& units, const starch_options& opt,
                  Layout lay, bool planned = false, bool split_ok = false)
{
    hipEvent_t* tv = c->timers();   // owned by the context: nothing to release on a throw
    hipEvent_t e0 = tv[0], e1 = tv[1], e2 = tv[2];
    HIP_CHECK(hipEventRecord(e0, c->st));
    c->have = false;
    c->streamed = false;
    c->gathered = false;
    c->stats = starch_stats{};
    for (auto& u : units) c->stats.input_bytes += u.len;
    std::vector<SegInfo> si;
    std::vector<uint64_t> unit_of;
    uint64_t tbytes = 0, nlines = 0;
    const uint8_t* text = transform_units(c, d_base, units, si, unit_of, tbytes, nlines, planned);
    std::vector<uint64_t> bc_u, bc_n;
    if (opt.base_counts) {   // per unit (units start segments), in segment order
        std::vector<uint64_t> uu, nn;
        for (auto& u : units) {
            c->tf.base_counts(d_base + u.off, u.len, c->st, u.init_start, u.init_stop, uu, nn);
            bc_u.insert(bc_u.end(), uu.begin(), uu.end());
            bc_n.insert(bc_n.end(), nn.begin(), nn.end());
        }
        if (bc_u.size() != si.size()) throw StarchError(STARCH_ERR_INTERNAL, "base counts: segment count mismatch");
    }
    HIP_CHECK(hipEventRecord(e1, c->st));
    const uint64_t nseg = si.size();
    c->stats.n_lines = nlines;
    c->stats.n_segments = nseg;
    c->stats.text_bytes = tbytes;
    c->text_bytes = tbytes;
    c->text_dev = text;
    // segment names: one gather + one copy, read once the encoder has synced
    PendingNames pnames;
    fetch_names(c, d_base, si, pnames);
    c->segs.assign(nseg, starch_segment{});
    for (uint64_t s = 0; s < nseg; ++s) {
        c->segs[s].line_count = si[s].line_count;
        c->segs[s].text_bytes = si[s].text_len;
        c->segs[s].name_len = si[s].name_len;
        c->segs[s].unit = unit_of[s];
        if (opt.base_counts) {
            c->segs[s].base_count_unique = (int64_t)bc_u[s];
            c->segs[s].base_count_nonunique = (int64_t)bc_n[s];
        }
    }
    const uint64_t base = (lay == L_ARCHIVE) ? 4 : 0;
    if (opt.reference_compat && lay == L_ARCHIVE) {   // the reference writes only the magic (hpp:765-769)
        uint8_t* out = c->archive.as<uint8_t>(64);
        HIP_CHECK(hipMemcpyAsync(out, kMagic, 4, hipMemcpyHostToDevice, c->st));
        HIP_CHECK(hipStreamSynchronize(c->st));
        finish_names(c, pnames);
        c->archive_bytes = 4;
        c->have = true;
        return;
    }
    std::vector<bz::StreamIn> sin(nseg);
    for (uint64_t s = 0; s < nseg; ++s) {
        sin[s].text_off = si[s].text_off;
        sin[s].text_len = si[s].text_len;
        sin[s].final_run_joins = 1;
        sin[s].group = (uint32_t)s;
    }
    std::vector<bz::StreamOut> outs;
    bz::Stats bst;
    const bool gzip = opt.compression_method == STARCH_METHOD_GZIP;
    const std::vector<uint64_t> cuts = !gzip && split_ok ? lane_cuts(si, tbytes, c->dev_lanes) : std::vector<uint64_t>();
    const size_t nl = cuts.size();
    std::vector<starch_ctx*> ln(nl);
    std::vector<std::vector<bz::StreamOut>> lo(nl);   // each lane's streams (offsets from its own base)
    std::vector<bz::Stats> lst(nl);
    std::vector<uint64_t> lbase(nl, 0);                // lane i's first byte after `base`
    if (gzip) {
        c->genc.plan(text, sin, c->st, outs, &bst);
    } else if (nl) {
        std::vector<int> code(nl, 0);
        std::vector<std::string> msg(nl);
        std::vector<std::vector<bz::StreamIn>> li(nl);
        for (size_t i = 0; i < nl; ++i) {
            ln[i] = lane_ctx(c, (int)i);
            ln[i]->enc.set_mem_share(1.0 / (double)nl);
            const uint64_t s0 = cuts[i], s1 = i + 1 < nl ? cuts[i + 1] : nseg;
            li[i].assign(sin.begin() + s0, sin.begin() + s1);
            for (auto& x : li[i]) x.group -= (uint32_t)s0;
        }
        auto plan_lane = [&](size_t i) {
            try {
                Ctx g(ln[i]);
                ln[i]->enc.plan(text, li[i], opt.block_size_100k, ln[i]->st, lo[i], &lst[i]);
            } catch (const StarchError& e) {
                code[i] = e.code;
                msg[i] = e.what();
            } catch (const std::exception& e) {
                code[i] = STARCH_ERR_INTERNAL;
                msg[i] = e.what();
            }
        };
        for (size_t i = 1; i < nl; ++i) HIP_CHECK(hipStreamWaitEvent(ln[i]->st, e1, 0));   // the text is written
        for (size_t i = 1; i < nl; ++i) ln[i]->worker.start([&plan_lane, i] { plan_lane(i); });
        plan_lane(0);
        for (size_t i = 1; i < nl; ++i) ln[i]->worker.wait();
        for (size_t i = 0; i < nl; ++i)
            if (code[i]) {
                for (size_t j = 1; j < nl; ++j) (void)hipStreamSynchronize(ln[j]->st);
                throw StarchError(code[i], msg[i]);
            }
        uint64_t end = 0;
        for (size_t i = 0; i < nl; ++i) {
            lbase[i] = end;
            uint64_t b = 0;
            for (auto o : lo[i]) {
                b = std::max(b, o.out_off + o.bytes);
                o.out_off += end;
                outs.push_back(o);
            }
            end += b;
            if (i) merge_counters(lst[0], lst[i]);
        }
        bst = lst[0];
    } else {
        c->enc.set_mem_share(1.0);
        c->enc.plan(text, sin, opt.block_size_100k, c->st, outs, &bst);
    }
    finish_names(c, pnames);
    uint64_t streams_bytes = 0;
    for (auto& o : outs) streams_bytes = std::max(streams_bytes, o.out_off + o.bytes);
    for (uint64_t s = 0; s < nseg; ++s) {
        c->segs[s].stream_offset = base + outs[s].out_off;
        c->segs[s].stream_bytes = outs[s].bytes;
        c->segs[s].n_blocks = outs[s].n_blocks;
    }
    const uint64_t index_off = base + streams_bytes;
    uint64_t names_b = 0;
    for (auto& nm : c->names) names_b += 6 * nm.size();
    const bool index = lay == L_ARCHIVE && opt.emit_index;
    const uint64_t cap = align_up(index_off + 4 + (index ? 256 + 256 * nseg + 64 + names_b : 0) +
                                      (opt.note && index ? 6 * strlen(opt.note) : 0),
                                  256);
    uint8_t* out = (lay == L_ARCHIVE ? c->archive : c->part).as<uint8_t>(cap);
    if (lay == L_ARCHIVE) HIP_CHECK(hipMemcpyAsync(out, kMagic, 4, hipMemcpyHostToDevice, c->st));
    if (gzip) {
        c->genc.emit(out, cap, base, outs, c->st, &bst);
    } else if (nl) {   // (plan left the lanes' streams idle: every lane's emit goes on this one, in order)
        uint64_t s = 0;
        for (size_t i = 0; i < nl; ++i) {
            ln[i]->enc.emit(out, cap, base + lbase[i], lo[i], c->st, &lst[i]);
            for (auto& o : lo[i]) outs[s++].combined_crc = o.combined_crc;
        }
    } else {
        c->enc.emit(out, cap, base, outs, c->st, &bst);
    }
    for (uint64_t s = 0; s < nseg; ++s) c->segs[s].combined_crc = outs[s].combined_crc;
    uint64_t total = index_off;
    std::string idx;
    if (index) {
        std::vector<const char*> np(nseg);
        std::vector<uint64_t> nl(nseg);
        for (uint64_t s = 0; s < nseg; ++s) { np[s] = c->names[s].data(); nl[s] = c->names[s].size(); }
        idx = build_index(c->segs.data(), np.data(), nl.data(), nseg, index_off, opt.note, opt.block_size_100k,
                          opt.base_counts != 0, opt.compression_method);
        if (index_off + idx.size() > cap) throw StarchError(STARCH_ERR_INTERNAL, "index capacity");
        HIP_CHECK(hipMemcpyAsync(out + index_off, idx.data(), idx.size(), hipMemcpyHostToDevice, c->st));
        total += idx.size();
    }
    HIP_CHECK(hipEventRecord(e2, c->st));
    HIP_CHECK(hipStreamSynchronize(c->st));
    if (nl) {
        std::vector<bz::Encoder::Interval> iv;
        for (size_t i = 0; i < nl; ++i) ln[i]->enc.take_intervals(e1, iv);
        stage_union(iv, bst);
    } else if (!gzip) {
        c->enc.resolve_timers(&bst);
    }
    float ms_t = 0, ms_all = 0;
    HIP_CHECK(hipEventElapsedTime(&ms_t, e0, e1));
    HIP_CHECK(hipEventElapsedTime(&ms_all, e0, e2));
    if (lay == L_ARCHIVE) c->archive_bytes = total;
    else c->part_bytes = total;
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

// transform + bzip2 + archive of a whole input into ctx->archive (device)
void encode_device(starch_ctx* c, const uint8_t* d_bed, uint64_t n, const starch_options& opt)
{
    std::vector<UnitIn> u(1, UnitIn{0, n, 0, 0, 0});
    encode_units(c, d_bed, u, opt, L_ARCHIVE, false, true);
}

// Pipelined encode of pinned host bytes (the one-call host path).  The input
// is cut at chromosome boundaries (shard::plan_units) into batches; every
// batch crosses PCIe in input order on one copy stream into one device buffer,
// and the batches go round robin to "lanes": the context itself and extra
// contexts on the same device (ctx->lanes), each with its own stream, encoder
// scratch and host thread.  A lane encodes a batch as soon as its bytes are in
// HBM, and the lanes' encodes run concurrently, so one lane's host syncs and
// small end-of-round launches are filled by the other's kernels.  Every
// batch's streams are appended to its lane's collect buffer; the archive is
// then laid out in batch (= input) order, and its bytes equal encode_device's:
// units are independent (shard.cpp), the index is built over all segments at
// the end.  The planner runs to the end of the bytes without a host 0xFF scan;
// a batch whose transform meets a 0xFF (which reads as EOF, hpp:181) abandons
// the pipeline and the caller takes the one-copy path.
bool host_is_pinned(const void* p)
{
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeHost;
}

struct LaneBatch {
    int lane = 0;
    uint64_t coll_off = 0, bytes = 0;
    std::vector<starch_segment> segs;
    std::vector<std::string> names;
    starch_stats stats{};
};

starch_ctx* lane_ctx(starch_ctx* c, int i)
{
    if (i == 0) return c;
    while ((int)c->lanes.size() < i) {
        std::unique_ptr<starch_ctx> L(new starch_ctx());
        L->device = c->device;
        L->is_lane = true;
        HIP_CHECK(hipStreamCreateWithFlags(&L->own, hipStreamNonBlocking));
        L->st = L->own;
        c->lanes.push_back(std::move(L));
    }
    return c->lanes[i - 1].get();
}

// append n device bytes to a lane's collect buffer (grown keeping its bytes)
void collect_append(starch_ctx* L, uint64_t& end, const void* src, uint64_t n)
{
    if (end + n > L->collect.cap) {
        const uint64_t ncap = align_up(std::max<uint64_t>(end + n, L->collect.cap + L->collect.cap / 2) + 4096, 1 << 20);
        DevBuf nb;
        uint8_t* np = nb.as<uint8_t>(ncap);
        if (end) HIP_CHECK(hipMemcpyAsync(np, L->collect.p, end, hipMemcpyDeviceToDevice, L->st));
        HIP_CHECK(hipStreamSynchronize(L->st));
        std::swap(L->collect.p, nb.p);
        std::swap(L->collect.cap, nb.cap);
    }
    if (n) HIP_CHECK(hipMemcpyAsync(static_cast<uint8_t*>(L->collect.p) + end, src, n, hipMemcpyDeviceToDevice, L->st));
    end += n;
}

// Host output of the pipelined encode (starch_encode_host_into): a batch's
// archive offset is known once every earlier batch has finished, so each
// finished batch whose predecessors are done goes device-to-host at once, on
// its lane's stream (after the append that put it in the collect buffer).
// Appends run under mu, so collect.p is read consistently, and a collect
// reallocation syncs its stream before freeing, so a queued copy's source
// stays valid.
struct HostOut {
    uint8_t* out = nullptr;
    uint64_t cap = 0, off = 4;     // next batch's archive offset (after the magic)
    size_t next = 0;               // first batch not yet written
    bool overflow = false;
    std::mutex mu;
    std::vector<char> done;
    std::vector<starch_ctx*> lane;
    void finished(size_t k, const std::vector<LaneBatch>& res)
    {
        std::lock_guard<std::mutex> lk(mu);
        done[k] = 1;
        while (next < done.size() && done[next]) {
            const LaneBatch& r = res[next];
            if (off + r.bytes > cap) overflow = true;
            else if (r.bytes) {
                starch_ctx* L = lane[r.lane];
                HIP_CHECK(hipMemcpyAsync(out + off, static_cast<uint8_t*>(L->collect.p) + r.coll_off, r.bytes,
                                         hipMemcpyDeviceToHost, L->st));
            }
            off += r.bytes;
            ++next;
        }
    }
};

// one lane: batches `mine` (indices into `batches`) in order, each once its
// bytes are in HBM (ev[k], recorded on the shared copy stream after its H2D)
void run_lane(starch_ctx* L, const uint8_t* d_in, const std::vector<shard::Unit>& plan,
              const std::vector<std::pair<size_t, size_t>>& batches, const std::vector<hipEvent_t>& ev,
              const std::vector<size_t>& mine, const starch_options& opt, std::vector<LaneBatch>& out, int lane,
              const std::atomic<bool>& stop, HostOut* hout)
{
    uint64_t total = 0;
    for (size_t k : mine)
        for (size_t u = batches[k].first; u < batches[k].second; ++u) total += plan[u].length;
    uint64_t cend = 0;
    if (L->collect.cap < total / 3 + (1 << 20)) L->collect.as<uint8_t>(total / 3 + (1 << 20));
    for (size_t j = 0; j < mine.size() && !stop.load(); ++j) {
        const size_t k = mine[j];
        HIP_CHECK(hipStreamWaitEvent(L->st, ev[k], 0));
        const uint64_t base = plan[batches[k].first].offset;
        std::vector<UnitIn> u;
        for (size_t q = batches[k].first; q < batches[k].second; ++q)
            u.push_back(UnitIn{plan[q].offset - base, plan[q].length, plan[q].init_start, plan[q].init_stop, q});
        STRACE("lane %d batch %zu: %zu units, encode", lane, k, u.size());
        encode_units(L, d_in + base, u, opt, L_STREAMS, true);
        STRACE("lane %d batch %zu: encoded, %llu stream bytes, device %.3f ms", lane, k,
               (unsigned long long)L->part_bytes, L->stats.ms_total);
        LaneBatch& r = out[k];
        r.lane = lane;
        r.coll_off = cend;
        r.bytes = L->part_bytes;
        r.segs = L->segs;
        r.names = L->names;
        r.stats = L->stats;
        if (hout) {   // appends (and collect reallocations) under the writer's lock: it reads collect.p
            {
                std::lock_guard<std::mutex> lk(hout->mu);
                collect_append(L, cend, L->part.p, L->part_bytes);
            }
            hout->finished(k, out);
        } else {
            collect_append(L, cend, L->part.p, L->part_bytes);
        }
    }
    HIP_CHECK(hipStreamSynchronize(L->st));
}

bool encode_host_pipelined(starch_ctx* c, const uint8_t* bed, uint64_t n, const starch_options& opt,
                           const HostRegistration& reg_in, uint8_t* hout_p = nullptr, uint64_t hout_cap = 0,
                           uint64_t* hout_len = nullptr)
{
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    std::vector<shard::Unit> plan;
    shard::plan_units_upto(bed, n, 4096, plan);
    // batches of consecutive units: a small first one (the GPU starts early),
    // then an eighth of the input, halving toward the end (the encode after the
    // last copy is short)
    static const int nbatch = [] { const char* e = getenv("STARCH_PIPE_BATCHES"); return e ? std::max(1, atoi(e)) : 8; }();
    static const int nlanes = [] { const char* e = getenv("STARCH_LANES"); return e ? std::min(4, std::max(1, atoi(e))) : 2; }();
    static const int first_div = [] { const char* e = getenv("STARCH_PIPE_FIRST"); return e ? std::max(1, atoi(e)) : 24; }();
    std::vector<std::pair<size_t, size_t>> batches;   // [u0, u1)
    {
        const uint64_t target = std::max<uint64_t>(64ull << 20, n / (uint64_t)nbatch);
        uint64_t left = n;
        for (size_t k = 0; k < plan.size();) {
            uint64_t want = std::max<uint64_t>(32ull << 20, std::min<uint64_t>(target, left / 2));
            if (k == 0) want = std::max<uint64_t>(32ull << 20, std::min<uint64_t>(want, n / (uint64_t)first_div));
            size_t e = k;
            uint64_t b = 0;
            while (e < plan.size() && (b == 0 || b + plan[e].length <= want)) b += plan[e++].length;
            batches.emplace_back(k, e);
            left -= b;
            k = e;
        }
    }
    const int nl = (int)std::min<size_t>((size_t)nlanes, std::max<size_t>(1, batches.size()));
    std::vector<std::vector<size_t>> mine(nl);
    for (size_t k = 0; k < batches.size(); ++k) mine[k % nl].push_back(k);
    std::vector<starch_ctx*> lane(nl);
    for (int i = 0; i < nl; ++i) lane[i] = lane_ctx(c, i);
    std::vector<LaneBatch> res(batches.size());
    std::atomic<bool> stop{false}, saw_ff{false};
    std::unique_ptr<HostOut> hout;
    if (hout_p) {
        hout.reset(new HostOut());
        hout->out = hout_p;
        hout->cap = hout_cap;
        hout->done.assign(batches.size(), 0);
        hout->lane = lane;
    }
    std::vector<int> codes(nl, 0);
    std::vector<std::string> errs(nl);
    // every batch crosses PCIe in input order on one copy stream, into one
    // device buffer, so the first batch arrives at full link rate
    if (!c->cst) HIP_CHECK(hipStreamCreateWithFlags(&c->cst, hipStreamNonBlocking));
    uint8_t* d_in = c->input.as<uint8_t>(n + 64);
    std::vector<hipEvent_t> ev(batches.size(), nullptr);
    for (auto& e : ev) HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    try {
        for (size_t k = 0; k < batches.size(); ++k) {
            const uint64_t o = plan[batches[k].first].offset;
            const uint64_t e = batches[k].second < plan.size() ? plan[batches[k].second].offset : n;
            if (e > o) reg_in.h2d(d_in + o, bed + o, e - o, c->cst);
            HIP_CHECK(hipEventRecord(ev[k], c->cst));
        }
    } catch (...) {
        (void)hipStreamSynchronize(c->cst);
        for (auto& e : ev) (void)hipEventDestroy(e);
        throw;
    }
    auto work = [&](int i) {
        try {
            Ctx g(lane[i]);
            run_lane(lane[i], d_in, plan, batches, ev, mine[i], opt, res, i, stop, hout.get());
        } catch (const FFInBatch&) {
            saw_ff = true;
            stop = true;
        } catch (const StarchError& e) {
            codes[i] = e.code;
            errs[i] = e.what();
            stop = true;
        } catch (const std::exception& e) {
            codes[i] = STARCH_ERR_INTERNAL;
            errs[i] = e.what();
            stop = true;
        }
    };
    {
        std::vector<std::thread> th;
        for (int i = 1; i < nl; ++i) th.emplace_back(work, i);
        work(0);
        for (auto& t : th) t.join();
    }
    (void)hipStreamSynchronize(c->cst);
    for (int i = 0; i < nl; ++i) (void)hipStreamSynchronize(lane[i]->st);   // device-to-host writes queued by other lanes
    for (auto& e : ev) (void)hipEventDestroy(e);
    for (int i = 0; i < nl; ++i)
        if (codes[i]) throw StarchError(codes[i], errs[i]);
    if (saw_ff) return false;
    // archive: magic, the batches' streams in input order, index
    uint64_t end = 4;
    std::vector<starch_segment> segs;
    std::vector<std::string> names;
    starch_stats st{};
    for (auto& r : res) {
        for (size_t s = 0; s < r.segs.size(); ++s) {
            starch_segment g = r.segs[s];
            g.stream_offset += end;
            segs.push_back(g);
            names.push_back(r.names[s]);
        }
        end += r.bytes;
        const starch_stats& x = r.stats;
        st.n_lines += x.n_lines;
        st.text_bytes += x.text_bytes;
        st.n_blocks += x.n_blocks;
        st.rle_bytes += x.rle_bytes;
        st.bwt_rounds += x.bwt_rounds;
        st.periodic_blocks += x.periodic_blocks;
        st.bwt_tied += x.bwt_tied;
        st.dedup_blocks += x.dedup_blocks;
        st.ms_transform += x.ms_transform;
        st.ms_rle += x.ms_rle;
        st.ms_bwt += x.ms_bwt;
        st.ms_mtf += x.ms_mtf;
        st.ms_tables += x.ms_tables;
        st.ms_emit += x.ms_emit;
    }
    std::string idx;
    if (opt.emit_index) {
        std::vector<const char*> np(segs.size());
        std::vector<uint64_t> nlen(segs.size());
        for (size_t s = 0; s < segs.size(); ++s) { np[s] = names[s].data(); nlen[s] = names[s].size(); }
        idx = build_index(segs.data(), np.data(), nlen.data(), segs.size(), end, opt.note, opt.block_size_100k,
                          opt.base_counts != 0, opt.compression_method);
    }
    uint8_t* arch = c->archive.as<uint8_t>(align_up(end + idx.size() + 64, 256));
    HIP_CHECK(hipMemcpyAsync(arch, kMagic, 4, hipMemcpyHostToDevice, c->st));
    uint64_t o = 4;
    for (size_t k = 0; k < res.size();) {   // one copy per run of batches adjacent in a lane's collect buffer
        const int ln = res[k].lane;
        uint64_t len = res[k].bytes;
        size_t k2 = k + 1;
        while (k2 < res.size() && res[k2].lane == ln && res[k2].coll_off == res[k].coll_off + len) len += res[k2++].bytes;
        if (len)
            HIP_CHECK(hipMemcpyAsync(arch + o, static_cast<uint8_t*>(lane[ln]->collect.p) + res[k].coll_off, len,
                                     hipMemcpyDeviceToDevice, c->st));
        o += len;
        k = k2;
    }
    if (!idx.empty()) HIP_CHECK(hipMemcpyAsync(arch + end, idx.data(), idx.size(), hipMemcpyHostToDevice, c->st));
    if (hout) {   // every batch went out already (all lanes finished); magic and index from the host
        if (hout->overflow || hout->off != end || end + idx.size() > hout_cap) {
            HIP_CHECK(hipStreamSynchronize(c->st));
            *hout_len = end + idx.size();   // the size needed; the buffer's contents are undefined
            throw StarchError(STARCH_ERR_MEM, "output buffer too small");
        }
        memcpy(hout_p, kMagic, 4);
        memcpy(hout_p + end, idx.data(), idx.size());
        *hout_len = end + idx.size();
    }
    HIP_CHECK(hipStreamSynchronize(c->st));
    st.input_bytes = n;
    st.n_segments = segs.size();
    st.archive_bytes = end + idx.size();
    st.ms_total = std::chrono::duration<float, std::milli>(clk::now() - t0).count();
    c->segs.swap(segs);
    c->names.swap(names);
    c->stats = st;
    c->text_bytes = 0;
    c->text_dev = nullptr;
    c->archive_bytes = st.archive_bytes;
    c->have = true;
    c->streamed = false;
    return true;
}

// Multi-device encode of host bytes: plan units, LPT them over the contexts,
// encode every shard on its own device in its own host thread, then gather
// the finished streams into ctxs[0]'s HBM (peer copies over xGMI; a plain
// device copy when two contexts share a device) and write magic + index.
void encode_multi(starch_ctx* const* ctxs, int nctx, const uint8_t* bed, uint64_t n, const starch_options& opt)
{
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    starch_ctx* c0 = ctxs[0];
    std::vector<shard::Unit> plan;
    shard::plan_units(bed, n, 64ull * (uint64_t)nctx, plan);
    std::vector<int32_t> shard_of;
    shard::assign_lpt(plan, nctx, shard_of);
    std::vector<std::vector<UnitIn>> mine(nctx);
    std::vector<uint64_t> dev_bytes(nctx, 0);
    for (size_t k = 0; k < plan.size(); ++k) {
        const int s = shard_of[k];
        mine[s].push_back(UnitIn{dev_bytes[s], plan[k].length, plan[k].init_start, plan[k].init_stop, k});
        dev_bytes[s] += plan[k].length;
    }
    std::vector<std::string> errs(nctx);
    std::vector<int> codes(nctx, 0);
    auto work = [&](int s) {
        starch_ctx* c = ctxs[s];
        try {
            Ctx g(c);
            uint8_t* d = c->input.as<uint8_t>(dev_bytes[s] + 64);
            for (auto& u : mine[s]) {
                const uint64_t src = plan[u.id].offset;
                if (u.len) HIP_CHECK(hipMemcpyAsync(d + u.off, bed + src, u.len, hipMemcpyHostToDevice, c->st));
            }
            encode_units(c, d, mine[s], opt, L_STREAMS);
        } catch (const StarchError& e) {
            codes[s] = e.code;
            errs[s] = e.what();
        } catch (const std::exception& e) {
            codes[s] = STARCH_ERR_INTERNAL;
            errs[s] = e.what();
        }
    };
    {
        std::vector<std::thread> th;
        for (int s = 1; s < nctx; ++s) th.emplace_back(work, s);
        work(0);
        for (auto& t : th) t.join();
    }
    for (int s = 0; s < nctx; ++s)
        if (codes[s]) throw StarchError(codes[s], "shard " + std::to_string(s) + ": " + errs[s]);
    // gather: archive order = unit order
    std::vector<uint64_t> unit_of, bytes;
    std::vector<std::pair<int, uint64_t>> src;   // (shard, segment) of each gathered segment
    for (int s = 0; s < nctx; ++s)
        for (uint64_t j = 0; j < ctxs[s]->segs.size(); ++j) {
            unit_of.push_back(ctxs[s]->segs[j].unit);
            bytes.push_back(ctxs[s]->segs[j].stream_bytes);
            src.emplace_back(s, j);
        }
    const uint64_t nseg = unit_of.size();
    std::vector<uint64_t> order, offset;
    uint64_t end = 4;
    shard::layout(unit_of.data(), bytes.data(), nseg, 4, order, offset, &end);
    std::vector<starch_segment> segs(nseg);
    std::vector<std::string> names(nseg);
    for (uint64_t k = 0; k < nseg; ++k) {
        const auto& sj = src[order[k]];
        segs[k] = ctxs[sj.first]->segs[sj.second];
        segs[k].stream_offset = offset[order[k]];
        names[k] = ctxs[sj.first]->names[sj.second];
    }
    std::string idx;
    if (opt.emit_index && !opt.reference_compat) {
        std::vector<const char*> np(nseg);
        std::vector<uint64_t> nl(nseg);
        for (uint64_t s = 0; s < nseg; ++s) { np[s] = names[s].data(); nl[s] = names[s].size(); }
        idx = build_index(segs.data(), np.data(), nl.data(), nseg, end, opt.note, opt.block_size_100k,
                          opt.base_counts != 0, opt.compression_method);
    }
    Ctx g(c0);
    const uint64_t total = opt.reference_compat ? 4 : end + idx.size();
    uint8_t* out = c0->archive.as<uint8_t>(align_up(total + 64, 256));
    HIP_CHECK(hipMemcpyAsync(out, kMagic, 4, hipMemcpyHostToDevice, c0->st));
    if (!opt.reference_compat) {
        for (int s = 0; s < nctx; ++s) {
            starch_ctx* c = ctxs[s];
            if (c->device != c0->device) (void)hipDeviceEnablePeerAccess(c->device, 0);
            (void)hipGetLastError();   // already enabled / not supported: the copy still works
        }
        // one copy per run of segments that are adjacent both in the part and in the archive
        for (uint64_t k = 0; k < nseg;) {
            const auto& sj = src[order[k]];
            starch_ctx* c = ctxs[sj.first];
            const uint64_t s_off = c->segs[sj.second].stream_offset, d_off = offset[order[k]];
            uint64_t len = bytes[order[k]], k2 = k + 1;
            while (k2 < nseg) {
                const auto& sn = src[order[k2]];
                if (sn.first != sj.first || c->segs[sn.second].stream_offset != s_off + len ||
                    offset[order[k2]] != d_off + len)
                    break;
                len += bytes[order[k2]];
                ++k2;
            }
            if (len) {
                if (c->device == c0->device)
                    HIP_CHECK(hipMemcpyAsync(out + d_off, static_cast<uint8_t*>(c->part.p) + s_off, len,
                                             hipMemcpyDeviceToDevice, c0->st));
                else
                    HIP_CHECK(hipMemcpyPeerAsync(out + d_off, c0->device, static_cast<uint8_t*>(c->part.p) + s_off,
                                                 c->device, len, c0->st));
            }
            k = k2;
        }
        if (!idx.empty()) HIP_CHECK(hipMemcpyAsync(out + end, idx.data(), idx.size(), hipMemcpyHostToDevice, c0->st));
    }
    HIP_CHECK(hipStreamSynchronize(c0->st));
    starch_stats st{};
    st.input_bytes = n;
    for (int s = 0; s < nctx; ++s) {
        const starch_stats& x = ctxs[s]->stats;
        st.n_lines += x.n_lines;
        st.n_segments += x.n_segments;
        st.text_bytes += x.text_bytes;
        st.n_blocks += x.n_blocks;
        st.rle_bytes += x.rle_bytes;
        st.bwt_rounds += x.bwt_rounds;
        st.periodic_blocks += x.periodic_blocks;
        st.bwt_tied += x.bwt_tied;
        st.dedup_blocks += x.dedup_blocks;
        st.ms_transform = std::max(st.ms_transform, x.ms_transform);
        st.ms_rle = std::max(st.ms_rle, x.ms_rle);
        st.ms_bwt = std::max(st.ms_bwt, x.ms_bwt);
        st.ms_mtf = std::max(st.ms_mtf, x.ms_mtf);
        st.ms_tables = std::max(st.ms_tables, x.ms_tables);
        st.ms_emit = std::max(st.ms_emit, x.ms_emit);
    }
    st.archive_bytes = total;
    st.ms_total = std::chrono::duration<float, std::milli>(clk::now() - t0).count();
    c0->segs.swap(segs);
    c0->names.swap(names);
    c0->stats = st;
    c0->text_bytes = 0;
    c0->text_dev = nullptr;
    c0->archive_bytes = total;
    c0->have = true;
    c0->streamed = false;
}

// ---- streaming ingestion (starch_stream_*) ---------------------------------
// The input arrives in pieces of any size.  Bytes not yet encoded are held in
// pinned host memory from a segment boundary on, together with the sscanf
// values current before them (shard.cpp: a unit boundary is any line start
// where the chr token changes, and a unit encoded on its own with those
// values gives exactly the streams of the whole input).  When at least a batch
// of input is held, the planner finds the last segment boundary among the
// complete lines; the prefix before it goes to the session's encoder thread
// (H2D, transform, bzip2 on the GPU, streams D2H into the ready bytes) while
// the held tail -- the last chromosome run, which may continue in the next
// piece -- moves to the other pinned buffer and the caller keeps feeding.
// end() encodes the rest and appends the index.

void stream_reserve(starch_ctx* c, int i, uint64_t need)
{
    auto& m = c->sm;
    if (need <= m.cap[i]) return;
    const uint64_t cap = align_up(std::max<uint64_t>(need, 2 * m.cap[i]), 1ull << 20);
    void* p = nullptr;
    HIP_CHECK(hipHostMalloc(&p, cap, hipHostMallocDefault));
    const bool keep = i == m.cur && m.held_n;
    if (keep) memcpy(p, m.buf[i], m.held_n);
    if (m.buf[i]) (void)hipHostFree(m.buf[i]);
    m.buf[i] = static_cast<uint8_t*>(p);
    m.cap[i] = cap;
    // the device mirror keeps the held bytes too (their H2D is ordered before on cst)
    DevBuf nb;
    uint8_t* d = nb.as<uint8_t>(cap + 64);
    if (keep) HIP_CHECK(hipMemcpyAsync(d, m.dbuf[i].p, m.held_n, hipMemcpyDeviceToDevice, c->cst));
    HIP_CHECK(hipStreamSynchronize(c->cst));
    std::swap(m.dbuf[i].p, nb.p);
    std::swap(m.dbuf[i].cap, nb.cap);
}

// pin buffer i (not the current one: nothing held) for `need` bytes, with its
// device mirror; the session's prepin thread runs this while the first batch
// is read
void stream_prepin_one(starch_ctx* c, int i, uint64_t need)
{
    auto& m = c->sm;
    if (need <= m.cap[i]) return;
    const uint64_t cap = align_up(need, 1ull << 20);
    void* p = nullptr;
    HIP_CHECK(hipHostMalloc(&p, cap, hipHostMallocDefault));
    if (m.buf[i]) (void)hipHostFree(m.buf[i]);
    m.buf[i] = static_cast<uint8_t*>(p);
    m.cap[i] = cap;
    DevBuf nb;
    (void)nb.as<uint8_t>(cap + 64);
    std::swap(m.dbuf[i].p, nb.p);
    std::swap(m.dbuf[i].cap, nb.cap);
}

void stream_prepin_join(starch_ctx* c)
{
    if (c->sm.prepin.joinable()) c->sm.prepin.join();
}

// Streaming inside a chromosome (bzip2): a batch may end inside a chromosome
// (open) and the next one then starts with the last line of it (ctx bytes of
// context).  The chromosome's stream is encoded in pieces: every batch
// encodes the complete bzip2 blocks of its text and carries the text after
// the last block boundary (a block starts a fresh RLE1 run, so the rest
// encodes the same in front of the next batch's text), the bits of the last
// partial byte, the combined CRC and the block count to the next piece; the
// header goes with the first piece, the trailer with the last one.  The
// context line is transformed on its own as well, and that output (the line
// as a segment's first) is dropped from the batch's first segment.
void stream_flush(starch_ctx::Streaming& m);

void stream_encode_pieces(starch_ctx* c, const uint8_t* d, uint64_t n, int64_t is, int64_t ip, uint64_t ctx,
                          bool open)
{
    auto& m = c->sm;
    auto& os = m.os;
    hipEvent_t* tv = c->timers();   // owned by the context: nothing to release on a throw
    hipEvent_t e0 = tv[0], e1 = tv[1], e2 = tv[2];
    HIP_CHECK(hipEventRecord(e0, c->st));
    c->stats = starch_stats{};
    c->stats.input_bytes = n - ctx;
    uint64_t o_ctx = 0;
    if (ctx) {
        TransformResult tc;
        c->tf.run(d, ctx, c->st, tc, is, ip);
        if (tc.n_lines != 1 || tc.n_segments != 1) throw StarchError(STARCH_ERR_INTERNAL, "stream: context line");
        o_ctx = tc.text_bytes;
    }
    TransformResult tr;
    c->tf.run(d, n, c->st, tr, is, ip);
    std::vector<SegInfo> si(tr.n_segments);
    if (tr.n_segments)
        HIP_CHECK(hipMemcpyAsync(si.data(), c->tf.seg_info_dev, tr.n_segments * sizeof(SegInfo), hipMemcpyDeviceToHost,
                                 c->st));
    HIP_CHECK(hipStreamSynchronize(c->st));
    if (ctx) {
        if (si.empty() || si[0].line_count < 1 || si[0].text_len < o_ctx)
            throw StarchError(STARCH_ERR_INTERNAL, "stream: context segment");
        si[0].text_off += o_ctx;
        si[0].text_len -= o_ctx;
        si[0].line_count -= 1;
        si[0].first_line += 1;
    }
    HIP_CHECK(hipEventRecord(e1, c->st));
    const uint64_t nseg = si.size();
    const bool cont = os.active;
    if (cont != (ctx > 0) || nseg == 0) throw StarchError(STARCH_ERR_INTERNAL, "stream: piece state");
    PendingNames pn;
    fetch_names(c, d, si, pn);
    // the open stream's rest, then the batch's text from segment 0 on
    const uint8_t* T = c->tf.text;
    const uint64_t new0 = si[0].text_len;
    if (cont && os.rest_len) {
        const uint64_t R = os.rest_len, t0 = si[0].text_off, span = tr.text_bytes - t0;
        uint8_t* Tb = c->text_all.as<uint8_t>(R + span + 64);
        HIP_CHECK(hipMemcpyAsync(Tb, os.rest.p, R, hipMemcpyDeviceToDevice, c->st));
        if (span) HIP_CHECK(hipMemcpyAsync(Tb + R, c->tf.text + t0, span, hipMemcpyDeviceToDevice, c->st));
        for (auto& x : si) x.text_off = x.text_off - t0 + R;
        si[0].text_off = 0;
        si[0].text_len += R;
        T = Tb;
    }
    std::vector<bz::StreamIn> sin(nseg);
    for (uint64_t s = 0; s < nseg; ++s) {
        sin[s].text_off = si[s].text_off;
        sin[s].text_len = si[s].text_len;
        sin[s].final_run_joins = 1;
        sin[s].group = (uint32_t)s;
    }
    if (cont) {
        sin[0].cont = 1;
        sin[0].phase = os.phase;
        sin[0].comb_in = os.comb;
    }
    if (open) {
        sin[nseg - 1].open = 1;
        sin[nseg - 1].final_run_joins = 0;
    }
    std::vector<bz::StreamOut> outs;
    bz::Stats bst;
    c->enc.plan(T, sin, m.opt.block_size_100k, c->st, outs, &bst);
    finish_names(c, pn);
    if (cont && c->names[0] != os.name) throw StarchError(STARCH_ERR_INTERNAL, "stream: continued chromosome");
    uint64_t total = 0;
    for (auto& o : outs) total = std::max(total, o.out_off + o.bytes);
    const uint64_t cap = align_up(total + 64, 256);
    uint8_t* out = c->part.as<uint8_t>(cap);
    c->enc.emit(out, cap, 0, outs, c->st, &bst);
    uint8_t* part = static_cast<uint8_t*>(m.back[0].get(total + 64));   // pinned: D2H at full PCIe rate
    if (total) HIP_CHECK(hipMemcpyAsync(part, out, total, hipMemcpyDeviceToHost, c->st));
    if (open) {   // the text after the last complete block waits for the next batch
        const uint64_t r0 = c->enc.open_rest(), r1 = sin[nseg - 1].text_off + sin[nseg - 1].text_len;
        os.rest_len = r1 - r0;
        if (os.rest.cap < os.rest_len + 64) HIP_CHECK(hipStreamSynchronize(c->st));   // T may hold the old rest
        uint8_t* rp = os.rest.as<uint8_t>(os.rest_len + 64);
        if (os.rest_len) HIP_CHECK(hipMemcpyAsync(rp, T + r0, os.rest_len, hipMemcpyDeviceToDevice, c->st));
    }
    HIP_CHECK(hipEventRecord(e2, c->st));
    HIP_CHECK(hipStreamSynchronize(c->st));
    c->enc.resolve_timers(&bst);
    float ms_t = 0, ms_all = 0;
    HIP_CHECK(hipEventElapsedTime(&ms_t, e0, e1));
    HIP_CHECK(hipEventElapsedTime(&ms_all, e0, e2));
    STRACE("stream batch %llu: %llu bytes in %llu segments (%s%s), device %.3f ms", (unsigned long long)m.batches,
           (unsigned long long)(n - ctx), (unsigned long long)nseg, cont ? "continues a chromosome" : "",
           open ? (cont ? ", open" : "open") : "", ms_all);
    std::lock_guard<std::mutex> lk(m.mu);
    for (uint64_t s = 0; s < nseg; ++s) {
        const bz::StreamOut& o = outs[s];
        const bool is_cont = s == 0 && cont, is_open = s + 1 == nseg && open;
        const uint8_t* b = part + o.out_off;
        const uint64_t bits = ((o.frame >> 8) & 7u) + ((o.frame & 1u) ? 32u : 0u) + o.block_bits +
                              ((o.frame & 2u) ? 80u : 0u);
        const uint64_t full = is_open ? bits / 8 : o.bytes;   // an open piece keeps its last partial byte
        const size_t at = m.ready.size();
        m.ready.insert(m.ready.end(), b, b + full);
        if (is_cont && full) m.ready[at] |= os.carry;   // the previous piece's bits of this byte
        uint8_t carry = 0;
        if (is_open && (bits & 7u)) carry = (uint8_t)(b[full] | ((is_cont && full == 0) ? os.carry : 0u));
        const uint64_t off = m.stream_end;
        m.stream_end += full;
        if (!is_cont) {               // a stream starts here
            os.clear();
            if (is_open) {
                os.active = true;
                os.name = c->names[s];
                os.off = off;
            }
        }
        if (is_cont || is_open) {     // a piece of a stream encoded in pieces
            os.bytes += full;
            os.n_blocks += o.n_blocks;
            os.comb = o.combined_crc;
            os.lines += si[s].line_count;
            os.text_bytes += s == 0 ? new0 : si[s].text_len;
            if (is_open) {
                os.phase = (uint32_t)(bits & 7u);
                os.carry = carry;
                continue;
            }
        }
        starch_segment g{};
        g.line_count = is_cont ? os.lines : si[s].line_count;
        g.text_bytes = is_cont ? os.text_bytes : si[s].text_len;
        g.name_len = c->names[s].size();
        g.stream_offset = is_cont ? os.off : off;
        g.stream_bytes = is_cont ? os.bytes : o.bytes;
        g.n_blocks = is_cont ? os.n_blocks : o.n_blocks;
        g.combined_crc = o.combined_crc;
        g.unit = m.batches;
        m.segs.push_back(g);
        m.names.push_back(c->names[s]);
        if (is_cont) os.clear();
    }
    if (!open) os.rest_len = 0;
    ++m.batches;
    ++m.seq_commit;                   // (pieces start with every earlier batch appended)
    starch_stats& t = m.stats;
    t.n_lines += tr.n_lines - (ctx ? 1 : 0);
    t.text_bytes += tr.text_bytes - o_ctx;
    t.n_blocks += bst.n_blocks;
    t.rle_bytes += bst.rle_bytes;
    t.bwt_rounds += bst.bwt_rounds;
    t.periodic_blocks += bst.periodic_blocks;
    t.bwt_tied += bst.bwt_tied;
    t.dedup_blocks += bst.dedup_blocks;
    t.ms_transform += ms_t;
    t.ms_rle += bst.rle;
    t.ms_bwt += bst.bwt;
    t.ms_mtf += bst.mtf;
    t.ms_tables += bst.tables;
    t.ms_emit += bst.emit;
    t.ms_total += ms_all;
    stream_flush(m);                  // batches after it that finished first
}

void add_stats(starch_stats& t, const starch_stats& x)
{
    t.n_lines += x.n_lines;
    t.text_bytes += x.text_bytes;
    t.n_blocks += x.n_blocks;
    t.rle_bytes += x.rle_bytes;
    t.bwt_rounds += x.bwt_rounds;
    t.periodic_blocks += x.periodic_blocks;
    t.bwt_tied += x.bwt_tied;
    t.dedup_blocks += x.dedup_blocks;
    t.ms_transform += x.ms_transform;
    t.ms_rle += x.ms_rle;
    t.ms_bwt += x.ms_bwt;
    t.ms_mtf += x.ms_mtf;
    t.ms_tables += x.ms_tables;
    t.ms_emit += x.ms_emit;
    t.ms_total += x.ms_total;
}

// append the next batch in hand-over order to the ready bytes (m.mu held)
void stream_append(starch_ctx::Streaming& m, const uint8_t* b, uint64_t nb, const std::vector<starch_segment>& segs,
                   const std::vector<std::string>& names, const starch_stats& x)
{
    m.ready.insert(m.ready.end(), b, b + nb);
    for (size_t s = 0; s < segs.size(); ++s) {
        starch_segment g = segs[s];
        g.stream_offset += m.stream_end;
        g.unit = m.batches;
        m.segs.push_back(g);
        m.names.push_back(names[s]);
    }
    m.stream_end += nb;
    ++m.batches;
    ++m.seq_commit;
    add_stats(m.stats, x);
    stream_flush(m);
}

// the parked batches that are next in hand-over order (m.mu held)
void stream_flush(starch_ctx::Streaming& m)
{
    for (auto it = m.done.find(m.seq_commit); it != m.done.end(); it = m.done.find(m.seq_commit)) {
        starch_ctx::Streaming::Done d = std::move(it->second);
        m.done.erase(it);
        stream_append(m, d.bytes.data(), d.bytes.size(), d.segs, d.names, d.stats);
    }
}

// lane `lane`: encode the job's batch (segment boundary to segment boundary,
// or to the end) and append its streams in hand-over order
void stream_encode(starch_ctx* c, int lane, const starch_ctx::Streaming::Job& j)
{
    auto& m = c->sm;
    starch_ctx* L = lane ? c->lanes[lane - 1].get() : c;
    if (m.opt.reference_compat) {     // the reference writes only the magic (hpp:765-769)
        std::lock_guard<std::mutex> lk(m.mu);
        if (j.seq == m.seq_commit) stream_append(m, nullptr, 0, {}, {}, starch_stats{});
        else m.done[j.seq] = starch_ctx::Streaming::Done{};
        return;
    }
    const uint8_t* d = static_cast<const uint8_t*>(m.dbuf[j.bufi].p);
    // the batch's H2D (copy stream) must be done before any kernel of the
    // lane reads it -- the piece path (context line + open stream) included
    HIP_CHECK(hipStreamWaitEvent(L->st, m.buf_ev[j.bufi], 0));
    if (j.ctx || j.open || j.cont) {   // handed over with no other batch in flight, to lane 0
        if (lane) throw StarchError(STARCH_ERR_INTERNAL, "stream: piece batch on an extra lane");
        stream_encode_pieces(c, d, j.n, j.is, j.ip, j.ctx, j.open);
        return;
    }
    STRACE("stream batch %llu (lane %d): %llu bytes, encode", (unsigned long long)j.seq, lane, (unsigned long long)j.n);
    std::vector<UnitIn> u(1, UnitIn{0, j.n, j.is, j.ip, 0});
    encode_units(L, d, u, m.opt, L_STREAMS);
    STRACE("stream batch %llu: encoded, device %.3f ms", (unsigned long long)j.seq, L->stats.ms_total);
    uint8_t* part = static_cast<uint8_t*>(m.back[lane].get(L->part_bytes + 64));   // pinned: D2H at full PCIe rate
    if (L->part_bytes) HIP_CHECK(hipMemcpyAsync(part, L->part.p, L->part_bytes, hipMemcpyDeviceToHost, L->st));
    HIP_CHECK(hipStreamSynchronize(L->st));
    STRACE("stream batch %llu: streams read back", (unsigned long long)j.seq);
    std::unique_lock<std::mutex> lk(m.mu);
    if (j.seq == m.seq_commit) {
        stream_append(m, part, L->part_bytes, L->segs, L->names, L->stats);
    } else {                          // an earlier batch is still encoding on the other lane
        lk.unlock();
        starch_ctx::Streaming::Done dn;
        dn.bytes.assign(part, part + L->part_bytes);
        dn.segs = L->segs;
        dn.names = L->names;
        dn.stats = L->stats;
        lk.lock();
        if (j.seq == m.seq_commit) stream_append(m, dn.bytes.data(), dn.bytes.size(), dn.segs, dn.names, dn.stats);
        else m.done[j.seq] = std::move(dn);
    }
}

void stream_worker(starch_ctx* c, int lane)
{
    auto& m = c->sm;
    (void)hipSetDevice(c->device);
    for (;;) {
        starch_ctx::Streaming::Job j;
        {
            std::unique_lock<std::mutex> lk(m.mu);
            m.cv.wait(lk, [&] { return m.lj[lane].pending || m.stop; });
            if (!m.lj[lane].pending) return;
            j = m.lj[lane];
            m.lj[lane].pending = false;
            m.lj[lane].busy = true;
        }
        int code = 0;
        std::string msg;
        try {
            stream_encode(c, lane, j);
        } catch (const StarchError& e) {
            code = e.code;
            msg = e.what();
        } catch (const std::exception& e) {
            code = STARCH_ERR_INTERNAL;
            msg = e.what();
        }
        {
            std::lock_guard<std::mutex> lk(m.mu);
            m.lj[lane].busy = false;
            m.buf_busy[j.bufi] = false;
            if (code && !m.err) { m.err = code; m.err_msg = msg; }
        }
        m.cv.notify_all();
    }
}

bool lane_idle(const starch_ctx::Streaming& m, int i) { return !m.lj[i].pending && !m.lj[i].busy; }

// wait until every lane is idle; rethrow a lane's error
void stream_wait(starch_ctx* c)
{
    auto& m = c->sm;
    std::unique_lock<std::mutex> lk(m.mu);
    m.cv.wait(lk, [&] {
        for (int i = 0; i < starch_ctx::Streaming::NLANE; ++i)
            if (!lane_idle(m, i)) return false;
        return true;
    });
    if (m.err) throw StarchError(m.err, m.err_msg);
}

// a buffer other than buf[cur] that no lane holds (waits for one)
int stream_free_buf(starch_ctx* c)
{
    auto& m = c->sm;
    std::unique_lock<std::mutex> lk(m.mu);
    int o = -1;
    m.cv.wait(lk, [&] {
        if (m.err) return true;
        for (int i = 0; i < starch_ctx::Streaming::NBUF; ++i)
            if (i != m.cur && !m.buf_busy[i]) { o = i; return true; }
        return false;
    });
    if (m.err) throw StarchError(m.err, m.err_msg);
    return o;
}

// hand buf[cur][0, n) to a lane: its first m.ctx_len bytes are context
// (already counted), open: it ends inside a chromosome.  A batch cut inside a
// chromosome, and the one after it, depend on each other's state (the open
// bzip2 stream): they go to lane 0 with no other batch in flight; any other
// batch to the first idle lane
void stream_submit(starch_ctx* c, uint64_t n, bool open = false)
{
    auto& m = c->sm;
    const bool serial = m.ctx_len > 0 || open || m.last_open;
    HIP_CHECK(hipEventRecord(m.buf_ev[m.cur], c->cst));
    {
        std::unique_lock<std::mutex> lk(m.mu);
        int lane = -1;
        m.cv.wait(lk, [&] {
            if (m.err) return true;
            if (serial) {
                for (int i = 0; i < starch_ctx::Streaming::NLANE; ++i)
                    if (!lane_idle(m, i)) return false;
                lane = 0;
                return true;
            }
            for (int i = 0; i < starch_ctx::Streaming::NLANE; ++i)
                if (lane_idle(m, i)) { lane = i; return true; }
            return false;
        });
        if (m.err) throw StarchError(m.err, m.err_msg);
        auto& j = m.lj[lane];
        j.pending = true;
        j.bufi = m.cur;
        j.n = n;
        j.ctx = m.ctx_len;
        j.open = open;
        j.cont = m.last_open;
        j.is = m.init_start;
        j.ip = m.init_stop;
        j.seq = m.seq_next++;
        m.buf_busy[m.cur] = true;
        m.last_open = open;
        m.stats.input_bytes += n - m.ctx_len;
    }
    m.cv.notify_all();
}

// hand everything before the last segment boundary among the complete lines
// to the encoder thread; the tail moves to the other buffer
void stream_cut(starch_ctx* c)
{
    auto& m = c->sm;
    uint8_t* h = m.buf[m.cur];
    const void* nl = memrchr(h, '\n', m.held_n);
    std::vector<shard::Unit> u;
    if (nl) {
        const uint64_t lim = (uint64_t)(static_cast<const uint8_t*>(nl) - h) + 1;
        shard::plan_units_upto(h, lim, 4096, u, m.init_start, m.init_stop);   // commit cut the bytes at any 0xFF
    }
    if (u.size() < 2) {   // no chromosome boundary among the complete lines
        // bzip2 streams encode in pieces: a whole batch of one chromosome is
        // cut at its last complete line (STARCH_STREAM_HOLD=1: held whole)
        static const bool hold = [] { const char* e = getenv("STARCH_STREAM_HOLD"); return e && !strcmp(e, "1"); }();
        const bool pieces = !hold && m.opt.compression_method == STARCH_METHOD_BZIP2 && !m.opt.base_counts &&
                            !m.opt.reference_compat;
        uint64_t ls = 0, cut = 0;
        if (pieces && nl && m.held_n >= m.batch) {
            cut = (uint64_t)(static_cast<const uint8_t*>(nl) - h) + 1;
            ls = cut - 1;
            while (ls > 0 && h[ls - 1] != '\n') --ls;   // the last complete line [ls, cut): the next context
        }
        if (!pieces || ls <= m.ctx_len || ls == 0) {   // the held run continues
            m.try_at = m.held_n + m.batch / 2;
            return;
        }
        int64_t st = m.init_start, sp = m.init_stop;
        shard::values_before(h, 0, ls, &st, &sp);      // sscanf values current before the context line
        const uint64_t tail = m.held_n - ls;
        STRACE("stream cut inside a chromosome at %llu of %llu held", (unsigned long long)cut,
               (unsigned long long)m.held_n);
        stream_prepin_join(c);
        const int o = stream_free_buf(c);
        stream_reserve(c, o, std::max<uint64_t>(tail + m.batch + (m.batch >> 2), 1ull << 20));
        m.pool.copy(m.buf[o], h + ls, tail);
        HIP_CHECK(hipMemcpyAsync(m.dbuf[o].p, static_cast<uint8_t*>(m.dbuf[m.cur].p) + ls, tail,
                                 hipMemcpyDeviceToDevice, c->cst));
        stream_submit(c, cut, true);
        m.cur = o;
        m.held_n = tail;
        m.ctx_len = cut - ls;
        m.init_start = st;
        m.init_stop = sp;
        m.try_at = std::max(m.batch, tail + m.batch / 2);
        return;
    }
    const uint64_t cut = u.back().offset, tail = m.held_n - cut;
    stream_prepin_join(c);
    STRACE("stream cut at %llu of %llu held: wait for a free buffer", (unsigned long long)cut, (unsigned long long)m.held_n);
    const int o = stream_free_buf(c);
    STRACE("stream cut: buffer %d free", o);
    stream_reserve(c, o, std::max<uint64_t>(tail + m.batch + (m.batch >> 2), 1ull << 20));
    m.pool.copy(m.buf[o], h + cut, tail);
    if (tail)   // the tail's device bytes move with it (ordered after their H2D on cst)
        HIP_CHECK(hipMemcpyAsync(m.dbuf[o].p, static_cast<uint8_t*>(m.dbuf[m.cur].p) + cut, tail,
                                 hipMemcpyDeviceToDevice, c->cst));
    stream_submit(c, cut);
    m.cur = o;
    m.held_n = tail;
    m.ctx_len = 0;
    m.init_start = u.back().init_start;
    m.init_stop = u.back().init_stop;
    m.try_at = std::max(m.batch, tail + m.batch / 2);
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
        case STARCH_ERR_DATA: return "malformed or corrupt compressed data";
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
    c->stream_shutdown();
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->st);
    if (c->cst) (void)hipStreamDestroy(c->cst);
    if (c->own) (void)hipStreamDestroy(c->own);
    delete c;
}

int starch_set_stream(starch_ctx* c, void* s)
{
    if (!c) return STARCH_ERR_ARG;
    c->st = static_cast<hipStream_t>(s);   // NULL = the HIP null stream (include/starch_amd.h)
    return STARCH_OK;
}

int starch_set_lanes(starch_ctx* c, int lanes)
{
    if (!c || lanes < 0 || lanes > 8) return STARCH_ERR_ARG;
    GUARD(c)
    c->dev_lanes = lanes;
    if (lanes == 1)   // the extra lanes' encoders give their HBM back (one encoder now holds every block)
        for (auto& l : c->lanes) {
            HIP_CHECK(hipStreamSynchronize(l->st));
            l->enc.release_device();
        }
    return STARCH_OK;
    END_GUARD(c)
}

int starch_use_own_stream(starch_ctx* c)
{
    if (!c) return STARCH_ERR_ARG;
    c->st = c->own;
    return STARCH_OK;
}

void starch_options_init(starch_options* o)
{
    if (!o) return;
    o->block_size_100k = 9;
    o->emit_index = 1;
    o->reference_compat = 0;
    o->note = nullptr;
    o->base_counts = 0;
    o->compression_method = STARCH_METHOD_BZIP2;
}

int starch_encode_device(starch_ctx* c, const void* d_bed, uint64_t n, const starch_options* opt)
{
    GUARD(c)
    starch_options o;
    starch_options_init(&o);
    if (opt) o = *opt;
    if (o.block_size_100k < 1 || o.block_size_100k > 9 ||
        (o.compression_method != STARCH_METHOD_BZIP2 && o.compression_method != STARCH_METHOD_GZIP)) return STARCH_ERR_ARG;
    if (n && !d_bed) return STARCH_ERR_ARG;
    encode_device(c, static_cast<const uint8_t*>(d_bed), n, o);
    return STARCH_OK;
    END_GUARD(c)
}

int starch_encode_host(starch_ctx* c, const void* bed, uint64_t n, const starch_options* opt)
{
    GUARD(c)
    if (n && !bed) return STARCH_ERR_ARG;
    starch_options o;
    starch_options_init(&o);
    if (opt) o = *opt;
    if (o.block_size_100k < 1 || o.block_size_100k > 9 ||
        (o.compression_method != STARCH_METHOD_BZIP2 && o.compression_method != STARCH_METHOD_GZIP)) return STARCH_ERR_ARG;
    // large pinned inputs: PCIe copy of the next batch overlaps the encode
    // (STARCH_PIPELINE=0 turns it off; pageable memory has no async copy)
    static const bool pipe_off = [] { const char* e = getenv("STARCH_PIPELINE"); return e && !strcmp(e, "0"); }();
    HostRegistration reg(pipe_off || o.reference_compat ? nullptr : bed, n, 256ull << 20);
    if (!pipe_off && !o.reference_compat && n >= (256ull << 20) && (reg.ok() || host_is_pinned(bed)) &&
        encode_host_pipelined(c, static_cast<const uint8_t*>(bed), n, o, reg))
        return STARCH_OK;
    uint8_t* d = c->input.as<uint8_t>(n + 64);
    reg.h2d(d, bed, n, c->st);
    HIP_CHECK(hipStreamSynchronize(c->st));
    encode_device(c, d, n, o);
    return STARCH_OK;
    END_GUARD(c)
}

static int units_in(const starch_unit* units, const uint64_t* ids, uint64_t nunits, std::vector<UnitIn>& u)
{
    if (nunits && !units) return STARCH_ERR_ARG;
    u.resize(nunits);
    for (uint64_t k = 0; k < nunits; ++k)
        u[k] = UnitIn{units[k].offset, units[k].length, units[k].init_start, units[k].init_stop, ids ? ids[k] : k};
    for (uint64_t k = 1; k < nunits; ++k)
        if (u[k].id <= u[k - 1].id) return STARCH_ERR_ARG;   // units in input order
    return STARCH_OK;
}

int starch_encode_host_into(starch_ctx* c, const void* bed, uint64_t n, const starch_options* opt, void* out,
                            uint64_t cap, uint64_t* out_len)
{
    GUARD(c)
    if ((n && !bed) || !out || !out_len) return STARCH_ERR_ARG;
    starch_options o;
    starch_options_init(&o);
    if (opt) o = *opt;
    if (o.block_size_100k < 1 || o.block_size_100k > 9 ||
        (o.compression_method != STARCH_METHOD_BZIP2 && o.compression_method != STARCH_METHOD_GZIP)) return STARCH_ERR_ARG;
    static const bool pipe_off = [] { const char* e = getenv("STARCH_PIPELINE"); return e && !strcmp(e, "0"); }();
    HostRegistration reg(pipe_off || o.reference_compat ? nullptr : bed, n, 256ull << 20);
    if (!pipe_off && !o.reference_compat && n >= (256ull << 20) && (reg.ok() || host_is_pinned(bed)) &&
        encode_host_pipelined(c, static_cast<const uint8_t*>(bed), n, o, reg, static_cast<uint8_t*>(out), cap, out_len))
        return STARCH_OK;
    uint8_t* d = c->input.as<uint8_t>(n + 64);
    reg.h2d(d, bed, n, c->st);
    HIP_CHECK(hipStreamSynchronize(c->st));
    encode_device(c, d, n, o);
    if (cap < c->archive_bytes) { *out_len = c->archive_bytes; return STARCH_ERR_MEM; }
    if (c->archive_bytes) HIP_CHECK(hipMemcpyAsync(out, c->archive.p, c->archive_bytes, hipMemcpyDeviceToHost, c->st));
    HIP_CHECK(hipStreamSynchronize(c->st));
    *out_len = c->archive_bytes;
    return STARCH_OK;
    END_GUARD(c)
}

int starch_encode_units_device(starch_ctx* c, const void* d_base, const starch_unit* units, const uint64_t* unit_ids,
                               uint64_t nunits, const starch_options* opt)
{
    GUARD(c)
    starch_options o;
    starch_options_init(&o);
    if (opt) o = *opt;
    if (o.block_size_100k < 1 || o.block_size_100k > 9 ||
        (o.compression_method != STARCH_METHOD_BZIP2 && o.compression_method != STARCH_METHOD_GZIP) || (nunits && !d_base)) return STARCH_ERR_ARG;
    std::vector<UnitIn> u;
    int rc = units_in(units, unit_ids, nunits, u);
    if (rc) return rc;
    encode_units(c, static_cast<const uint8_t*>(d_base), u, o, L_STREAMS, false, true);
    return STARCH_OK;
    END_GUARD(c)
}

int starch_encode_units_host(starch_ctx* c, const void* bed, const starch_unit* units, const uint64_t* unit_ids,
                             uint64_t nunits, const starch_options* opt)
{
    GUARD(c)
    starch_options o;
    starch_options_init(&o);
    if (opt) o = *opt;
    if (o.block_size_100k < 1 || o.block_size_100k > 9 ||
        (o.compression_method != STARCH_METHOD_BZIP2 && o.compression_method != STARCH_METHOD_GZIP) || (nunits && !bed))
        return STARCH_ERR_ARG;
    std::vector<UnitIn> u;
    int rc = units_in(units, unit_ids, nunits, u);
    if (rc) return rc;
    uint64_t total = 0;
    for (auto& x : u) total += x.len;
    uint8_t* d = c->input.as<uint8_t>(total + 64);
    uint64_t pos = 0;
    const uint8_t* h = static_cast<const uint8_t*>(bed);
    for (auto& x : u) {   // packed copies; coalesce units adjacent on the host
        const uint64_t src = x.off;
        x.off = pos;
        if (x.len) HIP_CHECK(hipMemcpyAsync(d + pos, h + src, x.len, hipMemcpyHostToDevice, c->st));
        pos += x.len;
    }
    encode_units(c, d, u, o, L_STREAMS);
    return STARCH_OK;
    END_GUARD(c)
}

int starch_streams_device(starch_ctx* c, const void** d_ptr, uint64_t* n)
{
    if (!c || !d_ptr || !n) return STARCH_ERR_ARG;
    if (!c->have || c->gathered) return STARCH_ERR_STATE;
    *d_ptr = c->part.p;
    *n = c->part_bytes;
    return STARCH_OK;
}

int starch_streams_copy(starch_ctx* c, void* dst, uint64_t cap)
{
    GUARD(c)
    if (!c->have || c->gathered) return STARCH_ERR_STATE;
    if (cap < c->part_bytes || (c->part_bytes && !dst)) return STARCH_ERR_MEM;
    if (c->part_bytes) HIP_CHECK(hipMemcpyAsync(dst, c->part.p, c->part_bytes, hipMemcpyDeviceToHost, c->st));
    HIP_CHECK(hipStreamSynchronize(c->st));
    return STARCH_OK;
    END_GUARD(c)
}

int starch_encode_multi_host(starch_ctx* const* ctxs, int nctx, const void* bed, uint64_t n, const starch_options* opt)
{
    if (!ctxs || nctx < 1 || (n && !bed)) return STARCH_ERR_ARG;
    for (int i = 0; i < nctx; ++i) {
        if (!ctxs[i]) return STARCH_ERR_ARG;
        for (int j = 0; j < i; ++j)
            if (ctxs[j] == ctxs[i]) return STARCH_ERR_ARG;   // one context per shard
    }
    starch_ctx* c = ctxs[0];
    GUARD(c)
    starch_options o;
    starch_options_init(&o);
    if (opt) o = *opt;
    if (o.block_size_100k < 1 || o.block_size_100k > 9 ||
        (o.compression_method != STARCH_METHOD_BZIP2 && o.compression_method != STARCH_METHOD_GZIP)) return STARCH_ERR_ARG;
    if (nctx == 1) {
        uint8_t* d = c->input.as<uint8_t>(n + 64);
        if (n) HIP_CHECK(hipMemcpyAsync(d, bed, n, hipMemcpyHostToDevice, c->st));
        encode_device(c, d, n, o);
    } else {
        encode_multi(ctxs, nctx, static_cast<const uint8_t*>(bed), n, o);
    }
    return STARCH_OK;
    END_GUARD(c)
}

int starch_plan_units(const void* bed, uint64_t n, uint64_t max_units, starch_unit* out, uint64_t* nunits)
{
    return starch_plan_units_from(bed, n, max_units, 0, 0, out, nunits);
}

int starch_plan_units_from(const void* bed, uint64_t n, uint64_t max_units, int64_t init_start, int64_t init_stop,
                           starch_unit* out, uint64_t* nunits)
{
    if (!nunits || !out || max_units < 1 || (n && !bed)) return STARCH_ERR_ARG;
    try {
        std::vector<shard::Unit> u;
        shard::plan_units(static_cast<const uint8_t*>(bed), n, max_units, u, init_start, init_stop);
        for (size_t k = 0; k < u.size(); ++k)
            out[k] = starch_unit{u[k].offset, u[k].length, u[k].init_start, u[k].init_stop};
        *nunits = u.size();
    } catch (const std::exception&) {
        return STARCH_ERR_MEM;
    }
    return STARCH_OK;
}

int starch_assign_shards(const starch_unit* units, uint64_t nunits, int nshards, int32_t* shard_of)
{
    if ((nunits && (!units || !shard_of)) || nshards < 1) return STARCH_ERR_ARG;
    std::vector<shard::Unit> u(nunits);
    for (uint64_t k = 0; k < nunits; ++k)
        u[k] = shard::Unit{units[k].offset, units[k].length, units[k].init_start, units[k].init_stop};
    std::vector<int32_t> s;
    shard::assign_lpt(u, nshards, s);
    if (nunits) memcpy(shard_of, s.data(), nunits * sizeof(int32_t));
    return STARCH_OK;
}

int starch_archive_layout(const uint64_t* unit_of, const uint64_t* bytes, uint64_t nseg, uint64_t base,
                          uint64_t* order, uint64_t* offset, uint64_t* end)
{
    if (!end || (nseg && (!unit_of || !bytes || !order || !offset))) return STARCH_ERR_ARG;
    std::vector<uint64_t> o, f;
    shard::layout(unit_of, bytes, nseg, base, o, f, end);
    if (nseg) {
        memcpy(order, o.data(), nseg * sizeof(uint64_t));
        memcpy(offset, f.data(), nseg * sizeof(uint64_t));
    }
    return STARCH_OK;
}

int starch_archive_size(starch_ctx* c, uint64_t* n)
{
    if (!c || !n) return STARCH_ERR_ARG;
    if (!c->have || c->streamed) return STARCH_ERR_STATE;
    *n = c->archive_bytes;
    return STARCH_OK;
}

int starch_archive_device(starch_ctx* c, const void** p)
{
    if (!c || !p) return STARCH_ERR_ARG;
    if (!c->have || c->streamed) return STARCH_ERR_STATE;
    *p = c->archive.p;
    return STARCH_OK;
}

int starch_archive_copy(starch_ctx* c, void* dst, uint64_t cap)
{
    GUARD(c)
    if (!c->have || c->streamed) return STARCH_ERR_STATE;
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

// transform stage only on device-resident BED bytes (segments: stream_offset =
// offset of the segment's text in the text buffer)
static void transform_only(starch_ctx* c, const uint8_t* d, uint64_t n, int64_t init_start = 0, int64_t init_stop = 0)
{
    hipEvent_t* tv = c->timers();
    hipEvent_t e0 = tv[0], e1 = tv[1];
    HIP_CHECK(hipEventRecord(e0, c->st));
    TransformResult tr;
    c->tf.run(d, n, c->st, tr, init_start, init_stop);
    HIP_CHECK(hipEventRecord(e1, c->st));
    std::vector<SegInfo> si(tr.n_segments);
    if (tr.n_segments)
        HIP_CHECK(hipMemcpyAsync(si.data(), c->tf.seg_info_dev, tr.n_segments * sizeof(SegInfo),
                                 hipMemcpyDeviceToHost, c->st));
    HIP_CHECK(hipStreamSynchronize(c->st));
    c->segs.assign(tr.n_segments, starch_segment{});
    PendingNames pnames;
    fetch_names(c, d, si, pnames);
    for (uint64_t s = 0; s < tr.n_segments; ++s) {
        c->segs[s].line_count = si[s].line_count;
        c->segs[s].text_bytes = si[s].text_len;
        c->segs[s].stream_offset = si[s].text_off;   // transform-only: offset into the text
        c->segs[s].name_len = si[s].name_len;
    }
    finish_names(c, pnames);
    float ms = 0;
    HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
    c->stats = starch_stats{};
    c->stats.input_bytes = n;
    c->stats.n_lines = tr.n_lines;
    c->stats.n_segments = tr.n_segments;
    c->stats.text_bytes = tr.text_bytes;
    c->stats.ms_transform = ms;
    c->stats.ms_total = ms;
    c->text_bytes = tr.text_bytes;
    c->text_dev = c->tf.text;
    c->archive_bytes = 0;
    c->have = true;
}

int starch_transform_host(starch_ctx* c, const void* bed, uint64_t n)
{
    return starch_transform_host_init(c, bed, n, 0, 0);
}

int starch_transform_host_init(starch_ctx* c, const void* bed, uint64_t n, int64_t init_start, int64_t init_stop)
{
    GUARD(c)
    if (n && !bed) return STARCH_ERR_ARG;
    uint8_t* d = c->input.as<uint8_t>(n + 64);
    {
        HostRegistration reg(bed, n, 64ull << 20);   // (a mapped file: DMA instead of staging)
        reg.h2d(d, bed, n, c->st);
        HIP_CHECK(hipStreamSynchronize(c->st));
    }
    transform_only(c, d, n, init_start, init_stop);
    return STARCH_OK;
    END_GUARD(c)
}

int starch_host_register(const void* p, uint64_t n)
{
    const uintptr_t pg = 4096, b = reinterpret_cast<uintptr_t>(p);
    const uintptr_t l = (b + pg - 1) & ~(pg - 1), h = (b + n) & ~(pg - 1);
    if (!p || h <= l) return STARCH_ERR_ARG;
    PinRegistry& R = pin_registry();
    std::lock_guard<std::mutex> lk(R.mu);
    if (R.overlaps(l, h)) return STARCH_ERR_ARG;            // (already registered, or in use by a call)
    bool ok = hipHostRegister(reinterpret_cast<void*>(l), h - l, hipHostRegisterPortable) == hipSuccess;
    if (!ok) {
        (void)hipGetLastError();   // a read-only mapping (a mapped input file): registered for reads
        ok = hipHostRegister(reinterpret_cast<void*>(l), h - l, hipHostRegisterReadOnly | hipHostRegisterPortable) == hipSuccess;
    }
    if (!ok) {
        (void)hipGetLastError();
        return STARCH_ERR_DEVICE;
    }
    R.m[l] = PinRegistry::Range{h, 0, false};               // the library DMAs from [l, h) only
    return STARCH_OK;
}

int starch_host_unregister(const void* p)
{
    const uintptr_t pg = 4096, l = (reinterpret_cast<uintptr_t>(p) + pg - 1) & ~(pg - 1);
    if (!p) return STARCH_ERR_ARG;
    PinRegistry& R = pin_registry();
    std::lock_guard<std::mutex> lk(R.mu);
    auto it = R.m.find(l);
    if (it == R.m.end() || it->second.temp) return STARCH_ERR_ARG;
    R.m.erase(it);
    if (hipHostUnregister(reinterpret_cast<void*>(l)) != hipSuccess) {
        (void)hipGetLastError();
        return STARCH_ERR_DEVICE;
    }
    return STARCH_OK;
}

int starch_transform_device(starch_ctx* c, const void* d_bed, uint64_t n)
{
    GUARD(c)
    if (n && !d_bed) return STARCH_ERR_ARG;
    transform_only(c, static_cast<const uint8_t*>(d_bed), n);
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
    if (c->text_bytes) HIP_CHECK(hipMemcpyAsync(dst, c->text_dev, c->text_bytes, hipMemcpyDeviceToHost, c->st));
    HIP_CHECK(hipStreamSynchronize(c->st));
    return STARCH_OK;
    END_GUARD(c)
}

int starch_text_read(starch_ctx* c, uint64_t off, void* dst, uint64_t n)
{
    GUARD(c)
    if (!c->have) return STARCH_ERR_STATE;
    if (off > c->text_bytes || n > c->text_bytes - off || (n && !dst)) return STARCH_ERR_ARG;
    if (n) HIP_CHECK(hipMemcpyAsync(dst, c->text_dev + off, n, hipMemcpyDeviceToHost, c->st));
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
    c->bz_nblocks = nstreams ? outs[0].n_blocks : 0;
    c->bz_crc = nstreams ? outs[0].combined_crc : 0;
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

int starch_bz2_stream_info(starch_ctx* c, uint32_t* n_blocks, uint32_t* combined_crc)
{
    if (!c || !n_blocks || !combined_crc) return STARCH_ERR_ARG;
    *n_blocks = c->bz_nblocks;
    *combined_crc = c->bz_crc;
    return STARCH_OK;
}

int starch_stream_begin(starch_ctx* c, const starch_options* opt, uint64_t batch_bytes)
{
    GUARD(c)
    starch_options o;
    starch_options_init(&o);
    if (opt) o = *opt;
    if (o.block_size_100k < 1 || o.block_size_100k > 9 ||
        (o.compression_method != STARCH_METHOD_BZIP2 && o.compression_method != STARCH_METHOD_GZIP)) return STARCH_ERR_ARG;
    c->stream_shutdown();                       // a session left open is abandoned
    auto& m = c->sm;
    if (!c->cst) HIP_CHECK(hipStreamCreateWithFlags(&c->cst, hipStreamNonBlocking));
    for (auto& e : m.buf_ev)
        if (!e) HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    for (int i = 1; i < starch_ctx::Streaming::NLANE; ++i) lane_ctx(c, i);   // (created here, not in a worker)
    HIP_CHECK(hipStreamSynchronize(c->cst));
    m.active = true;
    m.eof = false;
    m.note = o.note ? o.note : "";
    m.opt = o;
    m.opt.note = o.note ? m.note.c_str() : nullptr;
    m.cur = 0;
    m.held_n = 0;
    m.ctx_len = 0;
    m.os.clear();                                // a session left open may have left a piece behind
    m.os.rest_len = 0;
    m.batch = batch_bytes ? batch_bytes : (256ull << 20);
    m.try_at = m.batch;
    m.batches = 0;
    m.init_start = m.init_stop = 0;
    for (auto& j : m.lj) j = starch_ctx::Streaming::Job{};
    for (auto& b : m.buf_busy) b = false;
    m.last_open = false;
    m.seq_next = m.seq_commit = 0;
    m.done.clear();
    m.err = 0;
    m.err_msg.clear();
    m.ready.assign(kMagic, kMagic + 4);
    m.ready_off = 0;
    m.stream_end = 4;
    m.segs.clear();
    m.names.clear();
    m.stats = starch_stats{};
    c->have = false;
    c->streamed = false;
    // the pinned buffers sized once for a batch plus a long held run (kept
    // across sessions: pinning is paid on the context's first session only):
    // the first now, the others on the prepin thread while the first fills
    // STARCH_PIN=eager (default): all three now; bg: the others on the prepin
    // thread; lazy: the others at their first use (stream_cut)
    static const int pin_mode = [] {
        const char* e = getenv("STARCH_PIN");
        return e && !strcmp(e, "bg") ? 1 : e && !strcmp(e, "lazy") ? 2 : 0;
    }();
    stream_reserve(c, 0, pin_mode ? m.batch + m.batch / 2 : 2 * m.batch);
    bool more = false;
    for (int i = 1; i < starch_ctx::Streaming::NBUF; ++i) more |= m.cap[i] < 2 * m.batch;
    if (more && pin_mode == 0)
        for (int i = 1; i < starch_ctx::Streaming::NBUF; ++i) stream_reserve(c, i, 2 * m.batch);
    else if (more && pin_mode == 1)
        m.prepin = std::thread([c]() {
            (void)hipSetDevice(c->device);
            try {
                for (int i = 1; i < starch_ctx::Streaming::NBUF; ++i) stream_prepin_one(c, i, 2 * c->sm.batch);
            } catch (const StarchError& e) {   // the next stream_reserve of that buffer retries and reports
                STRACE("prepin failed: %s", e.what());
            }
        });
    for (int i = 0; i < starch_ctx::Streaming::NLANE; ++i) m.workers[i] = std::thread(stream_worker, c, i);
    return STARCH_OK;
    END_GUARD(c)
}

int starch_stream_window(starch_ctx* c, uint64_t min_bytes, void** ptr, uint64_t* cap)
{
    GUARD(c)
    auto& m = c->sm;
    if (!m.active) return STARCH_ERR_STATE;
    if (!ptr || !cap) return STARCH_ERR_ARG;
    {
        std::lock_guard<std::mutex> lk(m.mu);
        if (m.err) throw StarchError(m.err, m.err_msg);
    }
    stream_reserve(c, m.cur, m.held_n + std::max<uint64_t>(min_bytes, 1));
    *ptr = m.buf[m.cur] + m.held_n;
    *cap = m.cap[m.cur] - m.held_n;
    return STARCH_OK;
    END_GUARD(c)
}

// commit n window bytes of which the first k precede any 0xFF (0xFF reads as
// EOF, hpp:181); ff_known: k was found while copying (starch_stream_feed)
static int stream_commit_k(starch_ctx* c, uint64_t n, uint64_t k, bool ff_known)
{
    GUARD(c)
    auto& m = c->sm;
    if (!m.active) return STARCH_ERR_STATE;
    if (m.held_n + n > m.cap[m.cur]) return STARCH_ERR_ARG;
    if (m.eof || n == 0) return STARCH_OK;
    if (!ff_known) k = shard::input_limit(m.buf[m.cur] + m.held_n, n);
    if (k < n) m.eof = true;
    if (k && !m.opt.reference_compat)
        HIP_CHECK(hipMemcpyAsync(static_cast<uint8_t*>(m.dbuf[m.cur].p) + m.held_n, m.buf[m.cur] + m.held_n, k,
                                 hipMemcpyHostToDevice, c->cst));
    m.held_n += k;
    if (m.held_n >= m.try_at) stream_cut(c);
    return STARCH_OK;
    END_GUARD(c)
}

int starch_stream_commit(starch_ctx* c, uint64_t n) { return stream_commit_k(c, n, 0, false); }

int starch_stream_feed(starch_ctx* c, const void* bed, uint64_t n)
{
    if (!c) return STARCH_ERR_ARG;
    if (n && !bed) return STARCH_ERR_ARG;
    if (c->sm.eof || n == 0) return c->sm.active ? STARCH_OK : STARCH_ERR_STATE;
    void* w = nullptr;
    uint64_t cap = 0;
    int rc = starch_stream_window(c, n, &w, &cap);
    if (rc) return rc;
    const double t0 = tracing() ? trace_t0() : 0.0;
    const uint64_t k = c->sm.pool.copy_find_ff(static_cast<uint8_t*>(w), static_cast<const uint8_t*>(bed), n);
    const double t1 = tracing() ? trace_t0() : 0.0;
    rc = stream_commit_k(c, n, k, true);
    if (tracing()) {
        c->sm.t_copy += t1 - t0;
        c->sm.t_commit += trace_t0() - t1;
        c->sm.fed += n;
    }
    return rc;
}

int starch_stream_end(starch_ctx* c)
{
    GUARD(c)
    auto& m = c->sm;
    if (!m.active) return STARCH_ERR_STATE;
    try {
        stream_prepin_join(c);
        // the rest goes to a lane as soon as one is free (the other may still
        // be encoding); an open stream's last piece waits for its predecessor
        if (m.held_n > m.ctx_len || m.last_open) stream_submit(c, m.held_n);
        stream_wait(c);
    } catch (...) {
        c->stream_shutdown();
        throw;
    }
    c->stream_shutdown();
    STRACE("stream end: fed %.1f MB, copy %.1f ms (%.1f GB/s), commit+cut %.1f ms", m.fed / 1e6, m.t_copy,
           m.t_copy > 0 ? m.fed / m.t_copy / 1e6 : 0.0, m.t_commit);
    m.t_copy = m.t_commit = 0;
    m.fed = 0;
    m.held_n = 0;
    m.ctx_len = 0;
    if (m.opt.emit_index && !m.opt.reference_compat) {
        std::vector<const char*> np(m.segs.size());
        std::vector<uint64_t> nl(m.segs.size());
        for (size_t s = 0; s < m.segs.size(); ++s) { np[s] = m.names[s].data(); nl[s] = m.names[s].size(); }
        const std::string idx = build_index(m.segs.data(), np.data(), nl.data(), m.segs.size(), m.stream_end,
                                            m.opt.note, m.opt.block_size_100k, m.opt.base_counts != 0,
                                            m.opt.compression_method);
        m.ready.insert(m.ready.end(), idx.begin(), idx.end());
        m.stats.archive_bytes = m.stream_end + idx.size();
    } else {
        m.stats.archive_bytes = m.opt.reference_compat ? 4 : m.stream_end;
    }
    m.stats.n_segments = m.segs.size();
    c->segs = m.segs;
    c->names = m.names;
    c->stats = m.stats;
    c->archive_bytes = m.stats.archive_bytes;
    c->have = true;
    c->streamed = true;
    return STARCH_OK;
    END_GUARD(c)
}

int starch_stream_available(starch_ctx* c, uint64_t* n)
{
    if (!c || !n) return STARCH_ERR_ARG;
    std::lock_guard<std::mutex> lk(c->sm.mu);
    *n = c->sm.ready.size() - c->sm.ready_off;
    return STARCH_OK;
}

int starch_stream_read(starch_ctx* c, void* dst, uint64_t cap, uint64_t* len)
{
    if (!c || !len || (cap && !dst)) return STARCH_ERR_ARG;
    auto& m = c->sm;
    std::lock_guard<std::mutex> lk(m.mu);
    const uint64_t k = std::min<uint64_t>(cap, m.ready.size() - m.ready_off);
    if (k) memcpy(dst, m.ready.data() + m.ready_off, k);
    m.ready_off += k;
    if (m.ready_off == m.ready.size()) {
        m.ready.clear();
        m.ready_off = 0;
    } else if (m.ready_off > (64ull << 20) && 2 * m.ready_off > m.ready.size()) {
        m.ready.erase(m.ready.begin(), m.ready.begin() + (std::ptrdiff_t)m.ready_off);
        m.ready_off = 0;
    }
    *len = k;
    return STARCH_OK;
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

int starch_build_index_opt(const starch_segment* segs, const char* const* names, const uint64_t* name_lens,
                           uint64_t nseg, uint64_t index_offset, const starch_options* opt, char* dst, uint64_t cap,
                           uint64_t* len)
{
    if (!len || !opt || (nseg && (!segs || !names || !name_lens))) return STARCH_ERR_ARG;
    std::string s = build_index(segs, names, name_lens, nseg, index_offset, opt->note, opt->block_size_100k,
                                opt->base_counts != 0, opt->compression_method);
    *len = s.size();
    if (!dst) return STARCH_OK;
    if (cap < s.size()) return STARCH_ERR_MEM;
    memcpy(dst, s.data(), s.size());
    return STARCH_OK;
}

}  // extern "C"

namespace {

// Reader of this library's archive index (build_index above): the footer's
// index offset, then per stream its chromosome (JSON string, \u00XX escapes
// byte-wise), offset and size.  Only what unstarch needs; anything else is
// skipped.  Throws on a layout build_index does not write.
struct IndexEntry { std::string chr; uint64_t offset, size; };

std::vector<IndexEntry> read_index(const uint8_t* a, uint64_t n, uint64_t* index_off)
{
    auto bad = [](const char* m) { throw StarchError(STARCH_ERR_DATA, std::string("archive: ") + m); };
    if (n < 4 + 32 || memcmp(a, kMagic, 4) != 0) bad("no magic / footer");
    const char* f = reinterpret_cast<const char*>(a + n - 32);
    uint64_t off = 0;
    for (int i = 0; i < 20; ++i) {
        if (f[i] < '0' || f[i] > '9') bad("footer");
        off = off * 10 + (uint64_t)(f[i] - '0');
    }
    if (f[31] != '\n' || off < 4 || off > n - 32) bad("footer");
    *index_off = off;
    const std::string j(reinterpret_cast<const char*>(a + off), n - 32 - off);
    std::vector<IndexEntry> out;
    size_t p = j.find("\"streams\":[");
    if (p == std::string::npos) bad("index without streams");
    p += 11;
    auto num = [&](const char* key, size_t from, size_t to) -> uint64_t {
        const std::string k = std::string("\"") + key + "\":";
        size_t q = j.find(k, from);
        if (q == std::string::npos || q > to) bad("index field missing");
        q += k.size();
        uint64_t v = 0;
        if (q >= j.size() || j[q] < '0' || j[q] > '9') bad("index number");
        while (q < j.size() && j[q] >= '0' && j[q] <= '9') v = v * 10 + (uint64_t)(j[q++] - '0');
        return v;
    };
    while (p < j.size() && j[p] == '{') {
        const size_t e = j.find('}', p);   // entries hold no nested objects
        if (e == std::string::npos) bad("index entry");
        size_t q = j.find("\"chromosome\":\"", p);
        if (q == std::string::npos || q > e) bad("index chromosome");
        q += 14;
        std::string chr;
        for (;;) {
            if (q >= e) bad("index string");
            const char ch = j[q];
            if (ch == '"') break;
            if (ch != '\\') { chr += ch; ++q; continue; }
            const char x = j[q + 1];
            if (x == 'u') {
                unsigned v = 0;
                for (int k = 2; k < 6; ++k) {
                    const char h = j[q + k];
                    v = v * 16 + (unsigned)(h >= '0' && h <= '9' ? h - '0' : h >= 'a' && h <= 'f' ? h - 'a' + 10
                                             : h >= 'A' && h <= 'F' ? h - 'A' + 10 : 0);
                }
                chr += (char)v;
                q += 6;
            } else {
                chr += x == 'n' ? '\n' : x == 't' ? '\t' : x == 'r' ? '\r' : x == 'b' ? '\b' : x == 'f' ? '\f' : x;
                q += 2;
            }
        }
        out.push_back(IndexEntry{chr, num("offset", p, e), num("size", p, e)});
        p = e + 1;
        if (p < j.size() && j[p] == ',') ++p;
    }
    return out;
}

}  // namespace

extern "C" {

int starch_bz2_decompress_device(starch_ctx* c, const void* d_in, uint64_t n)
{
    GUARD(c)
    if (n && !d_in) return STARCH_ERR_ARG;
    c->have_out = false;
    uint8_t* d = c->dec_in.as<uint8_t>(n + 256);   // aligned copy with read-ahead padding
    if (n) HIP_CHECK(hipMemcpyAsync(d, d_in, n, hipMemcpyDeviceToDevice, c->st));
    HIP_CHECK(hipMemsetAsync(d + n, 0, 256, c->st));
    c->out_bytes = c->dec.decode(d, n, nullptr, c->st, c->dec_out, c->dstreams);
    c->out_dev = static_cast<const uint8_t*>(c->dec_out.p);
    c->have_out = true;
    return STARCH_OK;
    END_GUARD(c)
}

int starch_bz2_decompress_host(starch_ctx* c, const void* in, uint64_t n)
{
    GUARD(c)
    if (n && !in) return STARCH_ERR_ARG;
    c->have_out = false;
    uint8_t* d = c->dec_in.as<uint8_t>(n + 256);
    if (n) HIP_CHECK(hipMemcpyAsync(d, in, n, hipMemcpyHostToDevice, c->st));
    HIP_CHECK(hipMemsetAsync(d + n, 0, 256, c->st));
    c->out_bytes = c->dec.decode(d, n, static_cast<const uint8_t*>(in), c->st, c->dec_out, c->dstreams);
    c->out_dev = static_cast<const uint8_t*>(c->dec_out.p);
    c->have_out = true;
    return STARCH_OK;
    END_GUARD(c)
}

int starch_bz2_stream_count(starch_ctx* c, uint64_t* n)
{
    if (!c || !n) return STARCH_ERR_ARG;
    if (!c->have_out) return STARCH_ERR_STATE;
    *n = c->dstreams.size();
    return STARCH_OK;
}

int starch_bz2_streams(starch_ctx* c, starch_dec_stream* out, uint64_t cap)
{
    if (!c || (cap && !out)) return STARCH_ERR_ARG;
    if (!c->have_out) return STARCH_ERR_STATE;
    if (cap < c->dstreams.size()) return STARCH_ERR_MEM;
    for (size_t k = 0; k < c->dstreams.size(); ++k) {
        const bz::DecStream& s = c->dstreams[k];
        out[k] = starch_dec_stream{s.in_beg, s.in_end, s.out_off, s.out_len, s.level, s.n_blocks, s.stored_crc};
    }
    return STARCH_OK;
}

int starch_untransform_host(starch_ctx* c, const void* text, uint64_t n, const char* chr, uint64_t chr_len)
{
    GUARD(c)
    if ((n && !text) || (chr_len && !chr)) return STARCH_ERR_ARG;
    c->have_out = false;
    uint8_t* d = c->dec_out.as<uint8_t>(n + 64);
    if (n) HIP_CHECK(hipMemcpyAsync(d, text, n, hipMemcpyHostToDevice, c->st));
    std::vector<ut::Untransform::Seg> segs;
    if (n) segs.push_back(ut::Untransform::Seg{0, n, std::string(chr ? chr : "", chr_len)});
    c->out_bytes = c->untf.run(c->tf, d, n, segs, c->st, c->ut_out);
    c->out_dev = static_cast<const uint8_t*>(c->ut_out.p);
    c->have_out = true;
    return STARCH_OK;
    END_GUARD(c)
}

int starch_unstarch_host(starch_ctx* c, const void* archive, uint64_t n)
{
    GUARD(c)
    if (!archive) return STARCH_ERR_ARG;
    c->have_out = false;
    const uint8_t* a = static_cast<const uint8_t*>(archive);
    uint64_t index_off = 0;
    const std::vector<IndexEntry> idx = read_index(a, n, &index_off);
    // the streams region [4, index_off) is the concatenated bzip2 streams, in index order
    const uint64_t m = index_off - 4;
    uint8_t* d = c->dec_in.as<uint8_t>(m + 256);
    if (m) HIP_CHECK(hipMemcpyAsync(d, a + 4, m, hipMemcpyHostToDevice, c->st));
    HIP_CHECK(hipMemsetAsync(d + m, 0, 256, c->st));
    const uint64_t tbytes = c->dec.decode(d, m, a + 4, c->st, c->dec_out, c->dstreams);
    if (c->dstreams.size() != idx.size()) throw StarchError(STARCH_ERR_DATA, "archive: index and streams disagree");
    std::vector<ut::Untransform::Seg> segs;
    for (size_t k = 0; k < idx.size(); ++k) {
        const bz::DecStream& s = c->dstreams[k];
        if (s.in_beg + 4 != idx[k].offset || s.in_end - s.in_beg != idx[k].size)
            throw StarchError(STARCH_ERR_DATA, "archive: stream " + std::to_string(k) + " is not where the index says");
        segs.push_back(ut::Untransform::Seg{s.out_off, s.out_len, idx[k].chr});
    }
    c->out_bytes = c->untf.run(c->tf, static_cast<const uint8_t*>(c->dec_out.p), tbytes, segs, c->st, c->ut_out);
    c->out_dev = static_cast<const uint8_t*>(c->ut_out.p);
    c->have_out = true;
    return STARCH_OK;
    END_GUARD(c)
}

int starch_output_size(starch_ctx* c, uint64_t* n)
{
    if (!c || !n) return STARCH_ERR_ARG;
    if (!c->have_out) return STARCH_ERR_STATE;
    *n = c->out_bytes;
    return STARCH_OK;
}

int starch_output_device(starch_ctx* c, const void** d_ptr)
{
    if (!c || !d_ptr) return STARCH_ERR_ARG;
    if (!c->have_out) return STARCH_ERR_STATE;
    *d_ptr = c->out_dev;
    return STARCH_OK;
}

int starch_output_copy(starch_ctx* c, void* dst, uint64_t cap)
{
    GUARD(c)
    if (!c->have_out) return STARCH_ERR_STATE;
    if (cap < c->out_bytes || (c->out_bytes && !dst)) return STARCH_ERR_MEM;
    if (c->out_bytes) HIP_CHECK(hipMemcpyAsync(dst, c->out_dev, c->out_bytes, hipMemcpyDeviceToHost, c->st));
    HIP_CHECK(hipStreamSynchronize(c->st));
    return STARCH_OK;
    END_GUARD(c)
}

}  // extern "C"
