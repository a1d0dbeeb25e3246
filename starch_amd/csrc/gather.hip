// starch_amd/csrc/gather.hip -- the one collective of the multi-GPU path
// (SURVEY §5, §8e): every rank holds the finished bzip2 streams of its share
// of the chromosome units (starch_encode_units_*); rank 0 gathers them into
// the archive, in input (unit) order, and writes magic + index around them.
//
// The reference has no distributed layer: its unit of independence is the
// per-chromosome hand-off process_tf_buffer (include/starch3api.hpp:393-407),
// so the streams shard with no data-path exchange.  The exchange is:
//   1. all-gather of (segment count, name bytes) per rank        16 B / rank
//   2. all-gather of the segment records + chromosome names      80 B / seg
//   3. grouped point-to-point: each rank sends its runs of streams that are
//      adjacent both in its buffer and in the archive; rank 0 receives each
//      run straight into its place in the archive (no staging, no host copy).
// Every rank computes the same layout from the gathered records
// (shard::layout), so senders and the receiver agree on the runs.
//
// Transports: RCCL over xGMI (device memory, one communicator per process,
// librccl loaded on first use -- the same soname torch-ROCm loads, so a
// process holding both shares one RCCL), and a host-callback transport whose
// four primitives are supplied by the caller (the gloo CPU tests drive the
// same gather code through it).
#include <arpa/inet.h>
#include <dlfcn.h>
#include <errno.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <string.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <string>
#include <thread>
#include <vector>

#include <rccl/rccl.h>

#include "ctx.hpp"
#include "shard.hpp"

struct starch_comm {
    int device = 0, rank = 0, world = 1;
    ncclComm_t comm = nullptr;
    DevBuf s0, s1;                 // all-gather send / receive scratch
};

namespace {

// ---- RCCL, loaded on first use ---------------------------------------------
struct Rccl {
    bool tried = false, ok = false;
    std::string why;
    std::string path;   // the file the symbols came from (dladdr)
    ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
    ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*CommGetAsyncError)(ncclComm_t, ncclResult_t*) = nullptr;
    ncclResult_t (*AllGather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*GroupStart)() = nullptr;
    ncclResult_t (*GroupEnd)() = nullptr;
    const char* (*GetErrorString)(ncclResult_t) = nullptr;
};

std::mutex g_rccl_mu;
Rccl g_rccl;

const Rccl& rccl()
{
    std::lock_guard<std::mutex> lk(g_rccl_mu);
    Rccl& r = g_rccl;
    if (r.tried) {
        if (!r.ok) throw StarchError(STARCH_ERR_DEVICE, "RCCL unavailable: " + r.why);
        return r;
    }
    r.tried = true;
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
    if (!h) {
        r.why = dlerror();
        throw StarchError(STARCH_ERR_DEVICE, "RCCL unavailable: " + r.why);
    }
    bool all = true;
    auto sym = [&](auto& fn, const char* name) {
        fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
        if (!fn) { all = false; g_rccl.why += std::string(" missing ") + name; }
    };
    sym(r.GetUniqueId, "ncclGetUniqueId");
    sym(r.CommInitRank, "ncclCommInitRank");
    sym(r.CommDestroy, "ncclCommDestroy");
    sym(r.CommGetAsyncError, "ncclCommGetAsyncError");
    sym(r.AllGather, "ncclAllGather");
    sym(r.Send, "ncclSend");
    sym(r.Recv, "ncclRecv");
    sym(r.GroupStart, "ncclGroupStart");
    sym(r.GroupEnd, "ncclGroupEnd");
    sym(r.GetErrorString, "ncclGetErrorString");
    r.ok = all;
    if (!all) throw StarchError(STARCH_ERR_DEVICE, "RCCL unavailable:" + r.why);
    // which librccl answered: a process that already holds torch-ROCm's RCCL
    // (SONAME librccl.so.1) gets that same object back from dlopen
    Dl_info di{};
    if (dladdr(reinterpret_cast<void*>(r.GetUniqueId), &di) && di.dli_fname) r.path = di.dli_fname;
    return r;
}

void nccl_check(ncclResult_t e, const char* what)
{
    if (e != ncclSuccess)
        throw StarchError(STARCH_ERR_DEVICE, std::string("RCCL ") + what + ": " + rccl().GetErrorString(e));
}

// ---- the gather, over any transport -----------------------------------------
struct Transport {
    int rank = 0, world = 1;
    virtual ~Transport() = default;
    virtual uint8_t* scratch(int slot, uint64_t n) = 0;               // transport memory, reused
    virtual uint8_t* output(uint64_t n) = 0;                          // rank 0's archive
    virtual void put(void* dst, const void* host, uint64_t n) = 0;    // host -> transport memory
    virtual void get(void* host, const void* src, uint64_t n) = 0;    // transport memory -> host, completed
    virtual void copy(void* dst, const void* src, uint64_t n) = 0;    // within transport memory
    virtual void all_gather(const void* send, void* recv, uint64_t bytes) = 0;   // recv: world x bytes
    virtual void group_begin() = 0;
    virtual void send(const void* p, uint64_t n, int peer) = 0;
    virtual void recv(void* p, uint64_t n, int peer) = 0;
    virtual void group_end() = 0;                                     // the group's sends/recvs are issued
    virtual void finish() = 0;                                        // everything issued has completed
};

constexpr int kCols = 10;   // u64 fields exchanged per segment (rec_of / seg_of)

void rec_of(const starch_segment& s, uint64_t* r)
{
    r[0] = s.unit;
    r[1] = s.stream_offset;
    r[2] = s.stream_bytes;
    r[3] = s.line_count;
    r[4] = s.text_bytes;
    r[5] = s.n_blocks;
    r[6] = s.combined_crc;
    r[7] = s.name_len;
    r[8] = (uint64_t)s.base_count_unique;
    r[9] = (uint64_t)s.base_count_nonunique;
}

starch_segment seg_of(const uint64_t* r)
{
    starch_segment s{};
    s.unit = r[0];
    s.stream_offset = r[1];
    s.stream_bytes = r[2];
    s.line_count = r[3];
    s.text_bytes = r[4];
    s.n_blocks = (uint32_t)r[5];
    s.combined_crc = (uint32_t)r[6];
    s.name_len = r[7];
    s.base_count_unique = (int64_t)r[8];
    s.base_count_nonunique = (int64_t)r[9];
    return s;
}

struct Gathered {
    std::vector<starch_segment> segs;   // archive order, stream_offset = archive offset (rank 0)
    std::vector<std::string> names;
    uint64_t bytes = 0;                 // archive bytes (rank 0), 0 elsewhere
};

// segs[k].stream_offset are offsets into `streams` (this rank's buffer, in
// transport memory); segs[k].unit = the global unit index (archive order).
void gather(Transport& t, const std::vector<starch_segment>& segs, const std::vector<std::string>& names,
            const uint8_t* streams, const starch_options& opt, Gathered& out)
{
    const int W = t.world;
    // 1. segment count and name bytes of every rank
    uint64_t nb = 0;
    for (auto& n : names) nb += n.size();
    const uint64_t hdr[2] = {segs.size(), nb};
    uint8_t* s0 = t.scratch(0, 16);
    uint8_t* s1 = t.scratch(1, 16 * (uint64_t)W);
    t.put(s0, hdr, 16);
    t.all_gather(s0, s1, 16);
    std::vector<uint64_t> cnt(2 * (size_t)W);
    t.get(cnt.data(), s1, 16 * (uint64_t)W);
    uint64_t maxn = 1, maxb = 1;
    for (int r = 0; r < W; ++r) {
        maxn = std::max(maxn, cnt[2 * r]);
        maxb = std::max(maxb, cnt[2 * r + 1]);
    }
    // 2. records + names, padded to the largest rank
    const uint64_t per = (maxn * kCols * 8 + maxb + 7) / 8 * 8;
    std::vector<uint8_t> mine(per, 0);
    for (size_t k = 0; k < segs.size(); ++k) rec_of(segs[k], reinterpret_cast<uint64_t*>(mine.data()) + k * kCols);
    uint64_t pos = maxn * kCols * 8;
    for (auto& n : names) {
        if (!n.empty()) memcpy(mine.data() + pos, n.data(), n.size());
        pos += n.size();
    }
    s0 = t.scratch(0, per);
    s1 = t.scratch(1, per * (uint64_t)W);
    t.put(s0, mine.data(), per);
    t.all_gather(s0, s1, per);
    std::vector<uint8_t> all(per * (size_t)W);
    t.get(all.data(), s1, per * (uint64_t)W);

    // global list in (rank, local order); the layout is stable by unit
    struct G { int rank; starch_segment s; std::string name; };
    std::vector<G> g;
    for (int r = 0; r < W; ++r) {
        const uint8_t* base = all.data() + per * (size_t)r;
        const uint64_t* rec = reinterpret_cast<const uint64_t*>(base);
        uint64_t np = maxn * kCols * 8;
        if (cnt[2 * r] > maxn || cnt[2 * r + 1] > maxb) throw StarchError(STARCH_ERR_INTERNAL, "gather: bad header");
        for (uint64_t k = 0; k < cnt[2 * r]; ++k) {
            G x{r, seg_of(rec + k * kCols), std::string()};
            if (np + x.s.name_len > maxn * kCols * 8 + cnt[2 * r + 1])
                throw StarchError(STARCH_ERR_INTERNAL, "gather: bad name length");
            x.name.assign(reinterpret_cast<const char*>(base + np), x.s.name_len);
            np += x.s.name_len;
            g.push_back(std::move(x));
        }
    }
    const uint64_t nseg = g.size();
    std::vector<uint64_t> unit_of(nseg), bytes(nseg), order, offset;
    for (uint64_t k = 0; k < nseg; ++k) { unit_of[k] = g[k].s.unit; bytes[k] = g[k].s.stream_bytes; }
    uint64_t end = 4;
    shard::layout(unit_of.data(), bytes.data(), nseg, 4, order, offset, &end);
    // runs: (rank, source offset, archive offset, length), adjacent on both sides
    struct Run { int rank; uint64_t src, dst, len; };
    std::vector<Run> runs;
    for (uint64_t k = 0; k < nseg; ++k) {
        const G& x = g[order[k]];
        if (!runs.empty() && runs.back().rank == x.rank && runs.back().src + runs.back().len == x.s.stream_offset &&
            runs.back().dst + runs.back().len == offset[order[k]])
            runs.back().len += x.s.stream_bytes;
        else
            runs.push_back(Run{x.rank, x.s.stream_offset, offset[order[k]], x.s.stream_bytes});
    }

    std::string idx;
    uint8_t* arch = nullptr;
    out.segs.clear();
    out.names.clear();
    out.bytes = 0;
    if (t.rank == 0) {
        for (uint64_t k = 0; k < nseg; ++k) {
            starch_segment s = g[order[k]].s;
            s.stream_offset = offset[order[k]];
            out.segs.push_back(s);
            out.names.push_back(g[order[k]].name);
        }
        const bool compat = opt.reference_compat != 0;
        if (opt.emit_index && !compat) {
            std::vector<const char*> np(nseg);
            std::vector<uint64_t> nl(nseg);
            for (uint64_t k = 0; k < nseg; ++k) { np[k] = out.names[k].data(); nl[k] = out.names[k].size(); }
            idx = archive::build_index(out.segs.data(), np.data(), nl.data(), nseg, end, opt.note, opt.block_size_100k,
                                       opt.base_counts != 0, opt.compression_method);
        }
        out.bytes = compat ? 4 : end + idx.size();
        arch = t.output(out.bytes);
        t.put(arch, archive::kMagic, 4);
        if (compat) runs.clear();   // the reference writes only the magic (hpp:765-769)
        for (auto& r : runs)
            if (r.rank == 0 && r.len) t.copy(arch + r.dst, streams + r.src, r.len);
    } else if (opt.reference_compat) {
        runs.clear();
    }
    // 3. grouped point-to-point: every stream byte crosses xGMI once
    t.group_begin();
    for (auto& r : runs) {
        if (!r.len || r.rank == 0) continue;
        if (t.rank == 0) t.recv(arch + r.dst, r.len, r.rank);
        else if (r.rank == t.rank) t.send(streams + r.src, r.len, 0);
    }
    t.group_end();
    if (t.rank == 0 && !idx.empty()) t.put(arch + end, idx.data(), idx.size());
    t.finish();
}

// RCCL transport: device memory on the context's stream
struct RcclTransport : Transport {
    starch_comm* cm;
    starch_ctx* c;
    RcclTransport(starch_comm* m, starch_ctx* x) : cm(m), c(x) { rank = m->rank; world = m->world; }
    uint8_t* scratch(int slot, uint64_t n) override { return (slot ? cm->s1 : cm->s0).as<uint8_t>(n + 64); }
    uint8_t* output(uint64_t n) override { return c->archive.as<uint8_t>((n + 64 + 255) / 256 * 256); }
    void put(void* d, const void* h, uint64_t n) override
    {
        if (n) HIP_CHECK(hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, c->st));
    }
    void get(void* h, const void* d, uint64_t n) override
    {
        if (n) HIP_CHECK(hipMemcpyAsync(h, d, n, hipMemcpyDeviceToHost, c->st));
        HIP_CHECK(hipStreamSynchronize(c->st));
    }
    void copy(void* d, const void* s, uint64_t n) override
    {
        if (n) HIP_CHECK(hipMemcpyAsync(d, s, n, hipMemcpyDeviceToDevice, c->st));
    }
    void all_gather(const void* s, void* r, uint64_t n) override
    {
        nccl_check(rccl().AllGather(s, r, n, ncclUint8, cm->comm, c->st), "all-gather");
    }
    void group_begin() override { nccl_check(rccl().GroupStart(), "group start"); }
    void send(const void* p, uint64_t n, int peer) override
    {
        nccl_check(rccl().Send(p, n, ncclUint8, peer, cm->comm, c->st), "send");
    }
    void recv(void* p, uint64_t n, int peer) override
    {
        nccl_check(rccl().Recv(p, n, ncclUint8, peer, cm->comm, c->st), "recv");
    }
    void group_end() override { nccl_check(rccl().GroupEnd(), "group end"); }
    void finish() override
    {
        HIP_CHECK(hipStreamSynchronize(c->st));
        ncclResult_t a = ncclSuccess;
        nccl_check(rccl().CommGetAsyncError(cm->comm, &a), "async error query");
        nccl_check(a, "async");
    }
};

// host-callback transport: host memory, the caller's primitives
struct HostTransport : Transport {
    const starch_host_comm* h;
    std::vector<uint8_t> b0, b1, out;
    explicit HostTransport(const starch_host_comm* x) : h(x) { rank = x->rank; world = x->world; }
    uint8_t* scratch(int slot, uint64_t n) override
    {
        auto& b = slot ? b1 : b0;
        if (b.size() < n) b.resize(n);
        return b.data();
    }
    uint8_t* output(uint64_t n) override
    {
        out.assign(n, 0);
        return out.data();
    }
    void put(void* d, const void* s, uint64_t n) override { if (n) memcpy(d, s, n); }
    void get(void* d, const void* s, uint64_t n) override { if (n) memcpy(d, s, n); }
    void copy(void* d, const void* s, uint64_t n) override { if (n) memmove(d, s, n); }
    static void ok(int rc, const char* what)
    {
        if (rc) throw StarchError(STARCH_ERR_DEVICE, std::string("host transport ") + what + " failed");
    }
    void all_gather(const void* s, void* r, uint64_t n) override { ok(h->all_gather(h->user, s, r, n), "all_gather"); }
    void group_begin() override {}
    void send(const void* p, uint64_t n, int peer) override { ok(h->send(h->user, p, n, peer), "send"); }
    void recv(void* p, uint64_t n, int peer) override { ok(h->recv(h->user, p, n, peer), "recv"); }
    void group_end() override { ok(h->group_end(h->user), "group_end"); }
    void finish() override {}
};

// ---- TCP bootstrap of the RCCL unique id (no torch, no MPI) ------------------
bool send_all(int fd, const void* p, size_t n)
{
    const char* c = static_cast<const char*>(p);
    while (n) {
        ssize_t k = ::send(fd, c, n, MSG_NOSIGNAL);
        if (k < 0 && errno == EINTR) continue;
        if (k <= 0) return false;
        c += k;
        n -= (size_t)k;
    }
    return true;
}

bool recv_all(int fd, void* p, size_t n, int timeout_ms)
{
    char* c = static_cast<char*>(p);
    while (n) {
        pollfd pf{fd, POLLIN, 0};
        int pr = poll(&pf, 1, timeout_ms);
        if (pr < 0 && errno == EINTR) continue;
        if (pr <= 0) return false;
        ssize_t k = ::recv(fd, c, n, 0);
        if (k < 0 && errno == EINTR) continue;
        if (k <= 0) return false;
        c += k;
        n -= (size_t)k;
    }
    return true;
}

constexpr uint32_t kHello = 0x53544348;   // "STCH"

// rank 0 listens on port and hands `id` to world-1 peers; others connect to
// host:port (retrying until the deadline) and receive it
void tcp_bootstrap(int rank, int world, const char* host, int port, ncclUniqueId* id, int timeout_s)
{
    const auto deadline = std::chrono::steady_clock::now() + std::chrono::seconds(timeout_s);
    auto left_ms = [&]() {
        auto d = std::chrono::duration_cast<std::chrono::milliseconds>(deadline - std::chrono::steady_clock::now());
        return (int)std::max<long long>(0, d.count());
    };
    if (rank == 0) {
        int ls = socket(AF_INET, SOCK_STREAM, 0);
        if (ls < 0) throw StarchError(STARCH_ERR_DEVICE, "bootstrap: socket");
        int one = 1;
        setsockopt(ls, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
        sockaddr_in a{};
        a.sin_family = AF_INET;
        a.sin_port = htons((uint16_t)port);
        a.sin_addr.s_addr = htonl(INADDR_ANY);
        if (bind(ls, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0 || listen(ls, world) != 0) {
            close(ls);
            throw StarchError(STARCH_ERR_DEVICE, "bootstrap: cannot listen on port " + std::to_string(port));
        }
        std::vector<bool> seen(world, false);
        for (int got = 1; got < world;) {
            pollfd pf{ls, POLLIN, 0};
            int pr = poll(&pf, 1, left_ms());
            if (pr < 0 && errno == EINTR) continue;
            if (pr <= 0) { close(ls); throw StarchError(STARCH_ERR_DEVICE, "bootstrap: peers did not connect"); }
            int fd = accept(ls, nullptr, nullptr);
            if (fd < 0) continue;
            uint32_t hello[2] = {0, 0};
            if (recv_all(fd, hello, sizeof(hello), left_ms()) && hello[0] == kHello && (int)hello[1] > 0 &&
                (int)hello[1] < world && !seen[hello[1]] && send_all(fd, id, sizeof(*id))) {
                seen[hello[1]] = true;
                ++got;
            }
            close(fd);
        }
        close(ls);
        return;
    }
    for (;;) {
        addrinfo hints{}, *res = nullptr;
        hints.ai_family = AF_INET;
        hints.ai_socktype = SOCK_STREAM;
        const std::string ps = std::to_string(port);
        if (getaddrinfo(host, ps.c_str(), &hints, &res) == 0 && res) {
            int fd = socket(AF_INET, SOCK_STREAM, 0);
            bool done = false;
            if (fd >= 0 && connect(fd, res->ai_addr, res->ai_addrlen) == 0) {
                const uint32_t hello[2] = {kHello, (uint32_t)rank};
                done = send_all(fd, hello, sizeof(hello)) && recv_all(fd, id, sizeof(*id), left_ms());
            }
            if (fd >= 0) close(fd);
            freeaddrinfo(res);
            if (done) return;
        }
        if (left_ms() == 0) throw StarchError(STARCH_ERR_DEVICE, "bootstrap: could not reach rank 0");
        std::this_thread::sleep_for(std::chrono::milliseconds(50));
    }
}

struct DevGuard {
    int prev = -1;
    explicit DevGuard(int d) { (void)hipGetDevice(&prev); (void)hipSetDevice(d); }
    ~DevGuard() { if (prev >= 0) (void)hipSetDevice(prev); }
};

thread_local std::string g_comm_err;

int comm_fail(const std::exception& e, int code)
{
    g_comm_err = e.what();
    return code;
}

}  // namespace

extern "C" {

const char* starch_comm_last_error(void) { return g_comm_err.c_str(); }

int starch_comm_id(void* id)
{
    if (!id) return STARCH_ERR_ARG;
    try {
        ncclUniqueId u;
        nccl_check(rccl().GetUniqueId(&u), "unique id");
        memcpy(id, &u, sizeof(u));
        return STARCH_OK;
    } catch (const StarchError& e) {
        return comm_fail(e, e.code);
    }
}

int starch_comm_create(int device, int rank, int world, const void* id, starch_comm** out)
{
    if (!out || !id || world < 1 || rank < 0 || rank >= world) return STARCH_ERR_ARG;
    *out = nullptr;
    try {
        DevGuard g(device);
        ncclUniqueId u;
        memcpy(&u, id, sizeof(u));
        starch_comm* m = new starch_comm();
        m->device = device;
        m->rank = rank;
        m->world = world;
        ncclResult_t e = rccl().CommInitRank(&m->comm, world, u, rank);
        if (e != ncclSuccess) {
            delete m;
            nccl_check(e, "communicator init");
        }
        *out = m;
        return STARCH_OK;
    } catch (const StarchError& e) {
        return comm_fail(e, e.code);
    } catch (const std::exception& e) {
        return comm_fail(e, STARCH_ERR_INTERNAL);
    }
}

int starch_comm_create_tcp(int device, int rank, int world, const char* host, int port, starch_comm** out)
{
    if (!out || world < 1 || rank < 0 || rank >= world || port <= 0 || port > 65535 || (rank && !host))
        return STARCH_ERR_ARG;
    try {
        ncclUniqueId u;
        memset(&u, 0, sizeof(u));
        if (rank == 0) nccl_check(rccl().GetUniqueId(&u), "unique id");
        if (world > 1) tcp_bootstrap(rank, world, host, port, &u, 600);
        return starch_comm_create(device, rank, world, &u, out);
    } catch (const StarchError& e) {
        return comm_fail(e, e.code);
    } catch (const std::exception& e) {
        return comm_fail(e, STARCH_ERR_INTERNAL);
    }
}

const char* starch_rccl_library(void)
{
    try {
        return rccl().path.c_str();
    } catch (const std::exception&) {
        return "";
    }
}

void starch_comm_destroy(starch_comm* m)
{
    if (!m) return;
    {
        DevGuard g(m->device);
        if (m->comm) (void)rccl().CommDestroy(m->comm);
        m->s0.release();
        m->s1.release();
    }
    delete m;
}

int starch_gather_archive(starch_ctx* c, starch_comm* m, const starch_options* opt)
{
    if (!c || !m) return STARCH_ERR_ARG;
    if (m->device != c->device) return STARCH_ERR_ARG;
    // a second gather would read archive offsets as offsets into the shard streams
    if (!c->have || c->streamed || c->gathered) return STARCH_ERR_STATE;
    starch_options o;
    starch_options_init(&o);
    if (opt) o = *opt;
    try {
        DevGuard g(c->device);
        RcclTransport t(m, c);
        Gathered r;
        gather(t, c->segs, c->names, static_cast<const uint8_t*>(c->part.p), o, r);
        if (m->rank == 0) {
            c->segs.swap(r.segs);
            c->names.swap(r.names);
            c->archive_bytes = r.bytes;
            c->gathered = true;
        } else {
            c->archive_bytes = 0;   // rank 0 holds the archive; this rank keeps its own segments
        }
        c->stats.archive_bytes = c->archive_bytes;
        return STARCH_OK;
    } catch (const StarchError& e) {
        c->err = e.what();
        return e.code;
    } catch (const std::exception& e) {
        c->err = e.what();
        return STARCH_ERR_INTERNAL;
    }
}

int starch_gather_host(const starch_host_comm* comm, const starch_segment* segs, const char* const* names,
                       const uint64_t* name_lens, uint64_t nseg, const void* streams, const starch_options* opt,
                       void** archive, uint64_t* len)
{
    if (!comm || !archive || !len || !comm->all_gather || !comm->send || !comm->recv || !comm->group_end ||
        comm->world < 1 || comm->rank < 0 || comm->rank >= comm->world ||
        (nseg && (!segs || !names || !name_lens)))
        return STARCH_ERR_ARG;
    *archive = nullptr;
    *len = 0;
    starch_options o;
    starch_options_init(&o);
    if (opt) o = *opt;
    try {
        std::vector<starch_segment> s(segs, segs + nseg);
        std::vector<std::string> n(nseg);
        for (uint64_t k = 0; k < nseg; ++k) {
            n[k].assign(names[k], name_lens[k]);
            s[k].name_len = name_lens[k];
        }
        HostTransport t(comm);
        Gathered r;
        gather(t, s, n, static_cast<const uint8_t*>(streams), o, r);
        if (comm->rank == 0) {
            void* p = malloc(std::max<uint64_t>(1, r.bytes));
            if (!p) return STARCH_ERR_MEM;
            if (r.bytes) memcpy(p, t.out.data(), r.bytes);
            *archive = p;
            *len = r.bytes;
        }
        return STARCH_OK;
    } catch (const StarchError& e) {
        return comm_fail(e, e.code);
    } catch (const std::exception& e) {
        return comm_fail(e, STARCH_ERR_INTERNAL);
    }
}

void starch_free(void* p) { free(p); }

}  // extern "C"
