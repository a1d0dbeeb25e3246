// tools/starch3_cli.cpp -- the `starch3` command line on MI355X.
//
// Keeps the reference CLI surface (src/starch3.cpp:72-167): getopt_long with
// "n:bghv?", long options --note/--bzip2/--gzip/--help/--version, an optional
// input filename (extra names warned and ignored, cpp:147-157), stdin checked
// for a redirect (hpp:890-905), and the same exit codes: 61 (ENODATA) no input
// / missing file, 38 (ENOSYS) gzip under --reference-compat, 1 two methods, 22
// (EINVAL) codec init.  The archive goes to stdout: magic ca5cad1a, one bzip2
// stream (-g: one gzip member) per chromosome,
// JSON index + footer.  Build-only flags: --level N, --no-index,
// --reference-compat (stdout exactly as the reference: the 4 magic bytes),
// --device N, --gpus N (shard chromosomes over devices 0..N-1 in one process),
// --devices LIST (explicit device list, e.g. 0,1 or 0,0 for virtual shards),
// --stats, --batch-mb N (streamed batches: 256 MiB, 32 MiB from a pipe), --slurp,
// --distributed.
//
// --distributed: one process per GPU (e.g. `torchrun --no-python
// --nproc-per-node 8 starch3 --distributed in.bed > out`): RANK / WORLD_SIZE /
// LOCAL_RANK / MASTER_ADDR from the environment, the RCCL id handed out by
// rank 0 over TCP on STARCH_COMM_PORT (default MASTER_PORT + 1).  Every rank
// maps the input file, plans the chromosome units, encodes its LPT share on
// its GPU, and the library's RCCL gather (starch_gather_archive) assembles the
// archive on rank 0, which writes it to stdout.
//
// A pipe on stdin (`sort-bed ... | starch3`, `cat f | starch3`, hpp:158-199's
// documented use): a reader thread starts at once, before the device opens,
// with the pipe's buffer raised (F_SETPIPE_SZ) so each read(2) takes up to
// that much; it fills a small pool of reused 32 MiB buffers that the main
// thread hands to the session (starch_stream_feed: a multi-threaded copy into
// the pinned buffers) as they fill, so reading overlaps the device open, the
// session set-up and the encode.  STARCH_CLI_PIPE=0: read(2) into the pinned
// window after set-up, as for any other stream.
//
// One device (the default): streaming ingestion -- the input
// is read(2) in 64 MiB pieces straight into the session's pinned buffer
// (starch_stream_window / _commit); every finished chromosome run goes to the
// library's encoder thread (H2D + GPU encode) while reading continues into the
// other buffer, and finished streams are written to stdout as they come, so
// host memory holds only the unfinished chromosome run.  --slurp (and --gpus/--devices) read the
// whole input first and encode it in one call.
#include <errno.h>
#include <getopt.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <chrono>
#include <condition_variable>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../include/starch_amd.h"

static const char* kName = "starch3";
static const char* kVersion = "0.1 (mi355x)";

static void usage(FILE* f)
{
    fprintf(f,
            "%s\n  version: %s\n\n"
            "  Compress sorted BED data to a Starch archive (bzip2 streams per chromosome) on AMD MI355X.\n\n"
            "  Usage:  %s [options] < input > output\n"
            "     or:  %s [options] input > output\n\n"
            "  --note=\"text\"        note stored in the archive index\n"
            "  --bzip2 | -b          bzip2 streams (default)\n"
            "  --gzip | -g           gzip members (one per chromosome; the reference: unsupported, exit 38)\n"
            "  --level N             bzip2 block size 1..9 (default 9)\n"
            "  --no-index            streams only, no JSON index/footer\n"
            "  --reference-compat    write exactly what the reference writes (magic bytes only)\n"
            "  --device N            GPU ordinal (default 0)\n"
            "  --gpus N              shard chromosomes over GPUs 0..N-1 (archive identical to one GPU)\n"
            "  --devices LIST        comma-separated GPU ordinals to shard over (may repeat)\n"
            "  --stats               print per-stage timings to stderr\n"
            "  --batch-mb N          streamed encode: encode once N MiB are held (default 256)\n"
            "  --slurp               read the whole input, then encode it in one call\n"
            "  --base-counts         per-chromosome unique / non-unique base counts in the index\n"
            "  --distributed         one process per GPU (RANK/WORLD_SIZE/LOCAL_RANK/MASTER_ADDR from the env;\n"
            "                        input must be a file); rank 0 writes the archive\n"
            "  --help | -h           this message\n"
            "  --version | -v        version\n",
            kName, kVersion, kName, kName);
}

static int env_int(const char* k, int dflt)
{
    const char* v = getenv(k);
    return v && *v ? atoi(v) : dflt;
}

// seconds from the start to the first input byte read (device open, session
// set-up: pinned buffers, lanes); -1 when the input was not streamed
static double g_setup_s = -1.0;
static double g_create_s = -1.0;   // ... of which: device contexts open (starch_create)
static double g_open_s = -1.0, g_fault_s = -1.0;   // mapped path: the device open and the page faulting alone
static double g_begin_s = -1.0;    // session begun (starch_stream_begin)
static double g_end_s = -1.0;      // last archive byte written
static double g_premain_s = -1.0;
static double g_encode_s = -1.0;   // mapped file: encode returned (archive in host memory)  // process start -> main() (loader, library constructors)

// seconds since this process started (/proc/self/stat starttime, clock ticks
// since boot, against CLOCK_BOOTTIME); -1 if unavailable
static double since_process_start()
{
    FILE* f = fopen("/proc/self/stat", "r");
    if (!f) return -1.0;
    char buf[1024];
    const size_t k = fread(buf, 1, sizeof(buf) - 1, f);
    fclose(f);
    buf[k] = 0;
    const char* p = strrchr(buf, ')');
    if (!p) return -1.0;
    unsigned long long start = 0;
    int field = 2;
    for (const char* q = p + 1; *q; ++q)
        if (*q == ' ' && ++field == 22) { start = strtoull(q + 1, nullptr, 10); break; }
    struct timespec ts;
    clock_gettime(CLOCK_BOOTTIME, &ts);
    const double hz = (double)sysconf(_SC_CLK_TCK);
    return ts.tv_sec + ts.tv_nsec * 1e-9 - (double)start / hz;
}

// the archive reached stdout: flushed, and no write failed on the way (ENOSPC,
// EPIPE, ...); otherwise the process must not exit 0 with a truncated archive
// stdin as a pipe: read(2) on a thread of its own into pooled buffers (see the
// header comment); the consumer takes filled buffers in order and gives them
// back once fed
struct PipeReader {
    static constexpr size_t kChunk = 32ull << 20;
    static constexpr int kPool = 8;          // buffers in flight (256 MiB)
    int fd = -1;
    std::thread th;
    std::mutex mu;
    std::condition_variable cv;
    std::deque<std::pair<char*, size_t>> full;
    std::vector<char*> free_;
    bool eof = false;
    int err = 0;
    size_t pipe_sz = 0;
    void start(int f)
    {
        fd = f;
        for (int i = 0; i < kPool; ++i) free_.push_back(static_cast<char*>(malloc(kChunk)));
        for (char* b : free_)
            if (!b) { err = ENOMEM; return; }
        th = std::thread([this]() { run(); });
    }
    void run()
    {
        // the largest pipe buffer allowed (/proc/sys/fs/pipe-max-size, 1 MiB by default)
        for (size_t sz = 64ull << 20; sz >= (64u << 10); sz >>= 1) {
            const int r = fcntl(fd, F_SETPIPE_SZ, (int)sz);
            if (r >= 0) { pipe_sz = (size_t)r; break; }
        }
        for (;;) {
            char* b;
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&]() { return !free_.empty(); });
                b = free_.back();
                free_.pop_back();
            }
            size_t got = 0;
            int e = 0;
            bool end = false;
            while (got < kChunk) {
                const ssize_t r = read(fd, b + got, kChunk - got);
                if (r < 0 && errno == EINTR) continue;
                if (r < 0) { e = errno ? errno : EIO; break; }
                if (r == 0) { end = true; break; }
                got += (size_t)r;
            }
            std::lock_guard<std::mutex> lk(mu);
            if (got) full.emplace_back(b, got);
            else free_.push_back(b);
            if (e) err = e;
            if (e || end) eof = true;
            cv.notify_all();
            if (e || end) return;
        }
    }
    // the next filled buffer, or {nullptr, 0} at the end of input
    std::pair<char*, size_t> next()
    {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&]() { return !full.empty() || eof; });
        if (full.empty()) return {nullptr, 0};
        auto x = full.front();
        full.pop_front();
        return x;
    }
    void give_back(char* b)
    {
        std::lock_guard<std::mutex> lk(mu);
        free_.push_back(b);
        cv.notify_all();
    }
    ~PipeReader()
    {
        if (th.joinable()) th.detach();   // (an early error exit: the process ends with it)
    }
    void join()
    {
        if (th.joinable()) th.join();
        for (char* b : free_) free(b);
        for (auto& x : full) free(x.first);
        free_.clear();
        full.clear();
    }
};

static bool stdout_ok()
{
    if (fflush(stdout) != 0 || ferror(stdout)) {
        fprintf(stderr, "Error: writing the archive failed (%s)\n", strerror(errno ? errno : EIO));
        fflush(stderr);
        return false;
    }
    return true;
}

static void print_stats(starch_ctx* ctx, std::chrono::steady_clock::time_point t0, uint64_t input_bytes)
{
    const double wall = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    starch_stats s;
    starch_get_stats(ctx, &s);
    const double run = g_setup_s >= 0 ? wall - g_setup_s : wall;
    fprintf(stderr,
            "{\"input_bytes\": %llu, \"lines\": %llu, \"segments\": %llu, \"text_bytes\": %llu, "
            "\"archive_bytes\": %llu, \"blocks\": %llu, \"ms_total\": %.3f, \"ms_transform\": %.3f, "
            "\"ms_rle\": %.3f, \"ms_bwt\": %.3f, \"ms_mtf\": %.3f, \"ms_tables\": %.3f, \"ms_emit\": %.3f, "
            "\"wall_s\": %.3f, \"e2e_mb_s\": %.1f, \"setup_s\": %.3f, \"create_s\": %.3f, \"begin_s\": %.3f, "
            "\"end_s\": %.3f, \"premain_s\": %.3f, \"encode_s\": %.3f, \"open_s\": %.3f, \"fault_s\": %.3f, "
            "\"after_setup_mb_s\": %.1f}\n",
            (unsigned long long)input_bytes, (unsigned long long)s.n_lines, (unsigned long long)s.n_segments,
            (unsigned long long)s.text_bytes, (unsigned long long)s.archive_bytes, (unsigned long long)s.n_blocks,
            s.ms_total, s.ms_transform, s.ms_rle, s.ms_bwt, s.ms_mtf, s.ms_tables, s.ms_emit, wall,
            wall > 0 ? input_bytes / wall / 1e6 : 0.0, g_setup_s, g_create_s, g_begin_s, g_end_s, g_premain_s, g_encode_s, g_open_s, g_fault_s,
            run > 0 ? input_bytes / run / 1e6 : 0.0);
}

// One rank of a multi-process run: map the file, plan units, LPT
// them over the ranks, encode this rank's share on LOCAL_RANK's GPU, gather
// over RCCL; rank 0 writes the archive.
static int run_distributed(const std::string& input, FILE* in, const starch_options& opt, int stats,
                           std::chrono::steady_clock::time_point t0)
{
    const int rank = env_int("RANK", 0), world = env_int("WORLD_SIZE", 1), local = env_int("LOCAL_RANK", rank);
    const char* host = getenv("MASTER_ADDR") ? getenv("MASTER_ADDR") : "127.0.0.1";
    const int port = env_int("STARCH_COMM_PORT", env_int("MASTER_PORT", 29500) + 1);
    if (input.empty()) {
        fprintf(stderr, "Error: --distributed needs an input file (every rank maps it)\n");
        return ENODATA;
    }
    if (in != stdin) fclose(in);
    // stdout is the archive: anything the communication library prints (RCCL
    // writes its version banner to stdout) goes to stderr instead
    fflush(stdout);
    const int out_fd = dup(STDOUT_FILENO);
    dup2(STDERR_FILENO, STDOUT_FILENO);
    const int fd = open(input.c_str(), O_RDONLY);
    struct stat sb;
    if (fd < 0 || fstat(fd, &sb) != 0) {
        fprintf(stderr, "Error: Input file handle could not be created\n");
        return ENODATA;
    }
    const uint64_t n = (uint64_t)sb.st_size;
    const uint8_t* bed = nullptr;
    if (n) {
        void* m = mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0);
        if (m == MAP_FAILED) {
            fprintf(stderr, "Error: cannot map %s\n", input.c_str());
            close(fd);
            return ENODATA;
        }
        bed = static_cast<const uint8_t*>(m);
    }
    std::vector<starch_unit> units(64ull * (uint64_t)world);
    uint64_t nu = 0;
    int rc = starch_plan_units(bed, n, units.size(), units.data(), &nu);
    units.resize(nu);
    std::vector<int32_t> shard_of(nu);
    if (rc == STARCH_OK) rc = starch_assign_shards(units.data(), nu, world, shard_of.data());
    std::vector<starch_unit> mine;
    std::vector<uint64_t> ids;
    for (uint64_t k = 0; k < nu; ++k)
        if (shard_of[k] == rank) { mine.push_back(units[k]); ids.push_back(k); }
    starch_ctx* ctx = nullptr;
    starch_comm* comm = nullptr;
    if (rc == STARCH_OK && (rc = starch_create(local, &ctx)) != STARCH_OK)
        fprintf(stderr, "Error: could not open MI355X device %d (%s)\n", local, starch_strerror(rc));
    if (rc == STARCH_OK && (rc = starch_comm_create_tcp(local, rank, world, host, port, &comm)) != STARCH_OK)
        fprintf(stderr, "Error: rank %d: communicator (%s)\n", rank, starch_comm_last_error());
    if (rc == STARCH_OK) rc = starch_encode_units_host(ctx, bed, mine.data(), ids.data(), mine.size(), &opt);
    if (rc == STARCH_OK) rc = starch_gather_archive(ctx, comm, &opt);
    if (rc == STARCH_OK && rank == 0) {
        uint64_t an = 0;
        starch_archive_size(ctx, &an);
        std::vector<char> out(an);
        rc = starch_archive_copy(ctx, out.data(), an);
        for (uint64_t w = 0; rc == STARCH_OK && w < an;) {
            const ssize_t k = write(out_fd, out.data() + w, an - w);
            if (k < 0 && errno == EINTR) continue;
            if (k <= 0) { rc = STARCH_ERR_INTERNAL; break; }
            w += (uint64_t)k;
        }
    }
    if (rc != STARCH_OK && ctx) fprintf(stderr, "Error: rank %d: %s (%s)\n", rank, starch_strerror(rc), starch_last_error(ctx));
    if (rc == STARCH_OK && stats) print_stats(ctx, t0, n);
    if (comm) starch_comm_destroy(comm);
    if (ctx) starch_destroy(ctx);
    if (bed) munmap(const_cast<uint8_t*>(bed), n);
    close(fd);
    close(out_fd);
    return rc == STARCH_OK ? 0 : (rc == STARCH_ERR_MEM ? ENOMEM : EINVAL);
}

int main(int argc, char** argv)
{
    g_premain_s = since_process_start();
    std::string note, input;
    int methods = 0, gzip = 0, level = 9, emit_index = 1, compat = 0, device = 0, stats = 0, slurp = 0, bases = 0;
    int distributed = 0;
    uint64_t batch_mb = 0;          // 0: 256 MiB, or 32 MiB for a pipe (see below)
    std::vector<int> devices;
    static struct option longs[] = {
        {"note", required_argument, nullptr, 'n'}, {"bzip2", no_argument, nullptr, 'b'},
        {"gzip", no_argument, nullptr, 'g'},       {"help", no_argument, nullptr, 'h'},
        {"version", no_argument, nullptr, 'v'},    {"level", required_argument, nullptr, 'L'},
        {"no-index", no_argument, nullptr, 'I'},   {"reference-compat", no_argument, nullptr, 'R'},
        {"device", required_argument, nullptr, 'D'}, {"stats", no_argument, nullptr, 'S'},
        {"gpus", required_argument, nullptr, 'G'},   {"devices", required_argument, nullptr, 'E'},
        {"batch-mb", required_argument, nullptr, 'M'}, {"slurp", no_argument, nullptr, 'U'},
        {"base-counts", no_argument, nullptr, 'B'}, {"distributed", no_argument, nullptr, 'P'},
        {nullptr, 0, nullptr, 0}};
    opterr = 0;
    int c, li;
    while ((c = getopt_long(argc, argv, "n:bghv?", longs, &li)) != -1) {
        switch (c) {
            case 'n': note = optarg; break;
            case 'b': ++methods; gzip = 0; break;
            case 'g': ++methods; gzip = 1; break;
            case 'h': usage(stdout); return 0;
            case 'v': printf("%s\n  version: %s\n", kName, kVersion); return 0;
            case '?': usage(stdout); return 0;
            case 'L': level = atoi(optarg); break;
            case 'I': emit_index = 0; break;
            case 'R': compat = 1; break;
            case 'D': device = atoi(optarg); break;
            case 'S': stats = 1; break;
            case 'M': batch_mb = strtoull(optarg, nullptr, 10); break;
            case 'U': slurp = 1; break;
            case 'B': bases = 1; break;
            case 'P': distributed = 1; break;
            case 'G': {
                devices.clear();
                for (int i = 0, k = atoi(optarg); i < k; ++i) devices.push_back(i);
                break;
            }
            case 'E': {
                devices.clear();
                for (const char* p = optarg; *p;) {
                    devices.push_back(atoi(p));
                    while (*p && *p != ',') ++p;
                    if (*p == ',') ++p;
                }
                break;
            }
            default: break;
        }
    }
    for (; optind < argc; ++optind) {
        if (input.empty()) {
            struct stat sb;
            if (stat(argv[optind], &sb) != 0) {
                fprintf(stderr, "Error: Input file does not exist (%s)\n", argv[optind]);
                return ENODATA;
            }
            input = argv[optind];
        } else {
            fprintf(stderr, "Warning: Ignoring additional input file [%s]\n", argv[optind]);
        }
    }
    if (methods > 1) {
        fprintf(stderr, "Error: Only one compression method may be set\n");
        usage(stderr);
        return EXIT_FAILURE;
    }
    if (level < 1 || level > 9) {
        fprintf(stderr, "Error: --level must be 1..9\n");
        return EINVAL;
    }
    struct stat st;
    if (input.empty() && fstat(STDIN_FILENO, &st) == 0 && S_ISCHR(st.st_mode)) {
        fprintf(stderr, "Error: No input is specified; please redirect or pipe in formatted data, or specify filename\n");
        usage(stderr);
        return ENODATA;
    }
    FILE* in = input.empty() ? stdin : fopen(input.c_str(), "rb");
    if (!in) {
        fprintf(stderr, "Error: Input file handle could not be created\n");
        return ENODATA;
    }
    static const unsigned char magic[4] = {0xca, 0x5c, 0xad, 0x1a};
    if (gzip && compat) {   // the reference writes the magic, then fails (hpp:765-769, 777-779)
        fwrite(magic, 1, 4, stdout);
        fprintf(stderr, "Error: This method is unsupported at this time\n");
        return ENOSYS;
    }
    const auto t0 = std::chrono::steady_clock::now();
    starch_options opt;
    starch_options_init(&opt);
    opt.block_size_100k = level;
    opt.emit_index = emit_index;
    opt.reference_compat = compat;
    opt.note = note.empty() ? nullptr : note.c_str();
    opt.base_counts = bases;
    opt.compression_method = gzip ? STARCH_METHOD_GZIP : STARCH_METHOD_BZIP2;
    if (distributed) return run_distributed(input, in, opt, stats, t0);
    if (devices.empty()) devices.push_back(device);
    std::vector<starch_ctx*> ctxs(devices.size(), nullptr);
    int rc = STARCH_OK;
    // A regular file of >= 256 MiB (a path, or stdin redirected from one) on
    // one device is mapped whole (see below); its pages are faulted in by 16
    // threads while the device opens on another (the HIP runtime's start-up
    // took 0.1-0.4 s)
    struct stat ms;
    const char* map_env = getenv("STARCH_CLI_MAP");
    const bool map_file = devices.size() == 1 && !slurp && !(map_env && !strcmp(map_env, "0")) &&
                          fstat(fileno(in), &ms) == 0 && S_ISREG(ms.st_mode) && ms.st_size >= (256ll << 20) &&
                          lseek(fileno(in), 0, SEEK_CUR) == 0;
    void* map = MAP_FAILED;
    std::unique_ptr<char[]> outp;   // the mapped path's archive buffer
    uint64_t out_cap = 0;
    std::thread opener;
    int open_rc = STARCH_OK;
    if (map_file)
        opener = std::thread([&]() {
            open_rc = starch_create(devices[0], &ctxs[0]);
            g_open_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        });
    if (map_file) {
        const uint64_t n = (uint64_t)ms.st_size;
        map = mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fileno(in), 0);
        if (map != MAP_FAILED) {
            (void)madvise(map, n, MADV_WILLNEED);
            // the output buffer is not initialised: only the pages the archive
            // lands on are ever touched (zero-filling a 1.2 GB std::vector took
            // ~0.25 s); its first n/8 (BED text compresses ~9x) are written
            // once here, beside the input's faults, so the finished batches'
            // device-to-host copies do not fault them in one by one
            // (STARCH_CLI_OUT_PREFAULT=0: not)
            out_cap = n / 2 + (16ull << 20);
            outp.reset(new char[out_cap]);
            const char* pe = getenv("STARCH_CLI_OUT_PREFAULT");
            const uint64_t pre = (pe && !strcmp(pe, "0")) ? 0 : std::min<uint64_t>(out_cap, n / 8);
            const int nt = std::max(1, std::min(16, (int)std::thread::hardware_concurrency()));
            std::vector<std::thread> th;
            const uint64_t per = ((n + nt - 1) / nt + 4095) & ~4095ull;
            const uint64_t oper = ((pre + nt - 1) / nt + 4095) & ~4095ull;
            std::vector<unsigned> sink(nt, 0);
            for (int t = 0; t < nt; ++t)
                th.emplace_back([&, t]() {
                    const volatile unsigned char* p = static_cast<const unsigned char*>(map);
                    unsigned acc = 0;
                    for (uint64_t o = (uint64_t)t * per; o < n && o < (uint64_t)(t + 1) * per; o += 4096) acc += p[o];
                    sink[t] = acc;
                    volatile char* q = outp.get();
                    for (uint64_t o = (uint64_t)t * oper; o < pre && o < (uint64_t)(t + 1) * oper; o += 4096) q[o] = 0;
                });
            for (auto& x : th) x.join();
            g_fault_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        }
        opener.join();
        rc = open_rc;
        if (rc != STARCH_OK) {
            fprintf(stderr, "Error: could not open MI355X device %d (%s)\n", devices[0], starch_strerror(rc));
            return EINVAL;
        }
    }
    // stdin from a pipe: start reading before the device opens
    PipeReader pipe;
    bool piped = false;
    {
        struct stat ps;
        const char* pe = getenv("STARCH_CLI_PIPE");
        piped = !map_file && devices.size() == 1 && !slurp && !(pe && !strcmp(pe, "0")) &&
                fstat(fileno(in), &ps) == 0 && (S_ISFIFO(ps.st_mode) || S_ISSOCK(ps.st_mode));
        if (piped) {
            pipe.start(fileno(in));
            if (pipe.err) {
                fprintf(stderr, "Error: out of memory for the input buffers\n");
                return ENOMEM;
            }
        }
    }
    for (size_t i = 0; i < devices.size() && !map_file; ++i) {
        rc = starch_create(devices[i], &ctxs[i]);
        if (rc != STARCH_OK) {
            fprintf(stderr, "Error: could not open MI355X device %d (%s)\n", devices[i], starch_strerror(rc));
            for (size_t j = 0; j < i; ++j) starch_destroy(ctxs[j]);
            return EINVAL;
        }
    }
    g_create_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    starch_ctx* ctx = ctxs[0];
    // The mapped file is encoded by the pipelined host path, which registers
    // the mapping with the runtime for the call (no bounce copy, no pinned
    // buffers to allocate or release) while finished chromosome batches come
    // back into the output buffer.  STARCH_CLI_MAP=0: the streamed session
    // below.
    if (map_file) {
        const uint64_t n = (uint64_t)ms.st_size;
        void* m = map;
        if (m != MAP_FAILED) {
            g_setup_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            g_begin_s = g_setup_s;
            uint64_t cap = out_cap, len = 0;
            rc = starch_encode_host_into(ctx, m, n, &opt, outp.get(), cap, &len);
            if (rc == STARCH_ERR_MEM && len > cap) {   // larger than guessed: the archive is still in the context
                outp.reset(new char[len]);
                rc = starch_archive_copy(ctx, outp.get(), len);
            }
            char* out = outp.get();
            munmap(m, n);
            if (in != stdin) fclose(in);
            g_encode_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            if (rc == STARCH_OK) {
                for (uint64_t w = 0; w < len;) {
                    const size_t k = fwrite(out + w, 1, len - w, stdout);
                    if (k == 0) { rc = STARCH_ERR_INTERNAL; break; }
                    w += k;
                }
            }
            g_end_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            if (rc != STARCH_OK) {
                fprintf(stderr, "Error: encode failed (%s: %s)\n", starch_strerror(rc), starch_last_error(ctx));
                return rc == STARCH_ERR_MEM ? ENOMEM : EINVAL;
            }
            if (!stdout_ok()) _exit(EIO);
            if (stats) {
                starch_stats s;
                starch_get_stats(ctx, &s);
                print_stats(ctx, t0, s.input_bytes);
            }
            fflush(stderr);
            _exit(0);
        }
    }
    if (ctxs.size() == 1 && !slurp) {
        // streamed: read(2) straight into the session's pinned buffer while the
        // encoder thread works on the previous batch; drain finished streams
        const uint64_t kPiece = 128ull << 20;
        std::vector<char> out(1u << 20);
        auto drain = [&]() {
            uint64_t k = 0;
            do {
                if (starch_stream_read(ctx, out.data(), out.size(), &k) != STARCH_OK) break;
                if (k) fwrite(out.data(), 1, k, stdout);
            } while (k == out.size());
        };
        const int fd = fileno(in);
        // a regular file (a path, or stdin redirected from one) is read by
        // several threads at once with pread(2) up to the size it had at the
        // start: one read(2) stream from the page cache runs at a few GB/s,
        // below what the encoder takes.  Past that size (a growing file, or
        // one whose st_size says 0, as in /proc) read(2) goes on to EOF.
        struct stat fs;
        const bool regular = fstat(fd, &fs) == 0 && S_ISREG(fs.st_mode) && fs.st_size > 0;
        const off_t start = regular ? lseek(fd, 0, SEEK_CUR) : (off_t)-1;
        bool par = regular && start >= 0;
        uint64_t off = par ? (uint64_t)start : 0;
        const uint64_t fsize = par ? (uint64_t)fs.st_size : 0;
        const int nthr = std::max(1, std::min(16, (int)std::thread::hardware_concurrency()));
        bool read_err = false;
        // a pipe delivers a few GB/s at most: small batches keep the pinned
        // buffers small (pinning them, and unpinning at exit, cost ~0.15 s per
        // GB; cfg2 through `cat | starch3`: 256 / 128 / 64 / 32 MiB batches
        // 1.19 / 1.08-1.20 / 0.82-0.93 / 0.78 s whole process)
        if (!batch_mb) batch_mb = piped ? 32 : 256;
        rc = starch_stream_begin(ctx, &opt, batch_mb << 20);
        g_begin_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        drain();
        g_setup_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        while (piped && rc == STARCH_OK) {       // the pipe reader's buffers, in order
            const auto x = pipe.next();
            if (!x.first) break;
            rc = starch_stream_feed(ctx, x.first, x.second);
            pipe.give_back(x.first);
            drain();
        }
        if (piped) {
            if (rc != STARCH_OK) {   // (the reader may be blocked on a full pool: let it finish the pipe)
                for (auto x = pipe.next(); x.first; x = pipe.next()) pipe.give_back(x.first);
            }
            pipe.join();
            if (pipe.err) read_err = true, errno = pipe.err;
        }
        while (!piped && rc == STARCH_OK) {
            void* w = nullptr;
            uint64_t cap = 0;
            rc = starch_stream_window(ctx, kPiece, &w, &cap);
            if (rc != STARCH_OK) break;
            uint64_t want = cap < kPiece ? cap : kPiece;
            uint64_t got = 0;
            if (par) {
                want = std::min<uint64_t>(want, fsize > off ? fsize - off : 0);
                if (want == 0) {          // the size taken at the start is read: on with read(2)
                    par = false;
                    if (lseek(fd, (off_t)off, SEEK_SET) < 0) { read_err = true; break; }
                    continue;
                }
                const uint64_t sub = (want + nthr - 1) / nthr;
                std::vector<uint64_t> n_read(nthr, 0);
                std::vector<int> failed(nthr, 0);
                std::vector<std::thread> th;
                for (int t = 0; t < nthr; ++t)
                    th.emplace_back([&, t]() {
                        const uint64_t b = (uint64_t)t * sub, e = std::min<uint64_t>(want, b + sub);
                        uint64_t q = b;
                        while (q < e) {
                            const ssize_t r = pread(fd, static_cast<char*>(w) + q, e - q, (off_t)(off + q));
                            if (r < 0 && errno == EINTR) continue;
                            if (r < 0) failed[t] = 1;
                            if (r <= 0) break;
                            q += (uint64_t)r;
                        }
                        n_read[t] = q - b;
                    });
                for (auto& x : th) x.join();
                for (int t = 0; t < nthr; ++t) read_err |= failed[t] != 0;
                if (read_err) break;
                for (int t = 0; t < nthr; ++t) {   // the bytes read contiguously from the piece's start
                    got += n_read[t];
                    if (n_read[t] < std::min<uint64_t>(want, (uint64_t)(t + 1) * sub) - std::min<uint64_t>(want, (uint64_t)t * sub)) break;
                }
                off += got;
                if (got < want) {         // shorter than its size said: read(2) decides where EOF is
                    par = false;
                    if (lseek(fd, (off_t)off, SEEK_SET) < 0) { read_err = true; break; }
                    if (got == 0) continue;
                }
            } else {
                const ssize_t k = read(fd, w, want);
                if (k < 0 && errno == EINTR) continue;
                if (k < 0) { read_err = true; break; }
                if (k == 0) break;
                got = (uint64_t)k;
            }
            rc = starch_stream_commit(ctx, got);
            drain();
        }
        if (read_err && rc == STARCH_OK) {
            fprintf(stderr, "Error: reading the input failed (%s)\n", strerror(errno));
            if (in != stdin) fclose(in);
            for (auto* c2 : ctxs) starch_destroy(c2);
            return EIO;
        }
        if (in != stdin) fclose(in);
        if (rc == STARCH_OK) rc = starch_stream_end(ctx);
        drain();
        g_end_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    } else {
        std::vector<char> data;
        {
            std::vector<char> buf(1 << 24);
            size_t k;
            while ((k = fread(buf.data(), 1, buf.size(), in)) > 0) data.insert(data.end(), buf.begin(), buf.begin() + k);
            if (in != stdin) fclose(in);
        }
        rc = ctxs.size() > 1 ? starch_encode_multi_host(ctxs.data(), (int)ctxs.size(), data.data(), data.size(), &opt)
                             : starch_encode_host(ctx, data.data(), data.size(), &opt);
        if (rc == STARCH_OK) {
            uint64_t n = 0;
            starch_archive_size(ctx, &n);
            std::vector<char> out(n);
            starch_archive_copy(ctx, out.data(), n);
            fwrite(out.data(), 1, n, stdout);
        }
    }
    if (rc != STARCH_OK) {
        fprintf(stderr, "Error: encode failed (%s: %s)\n", starch_strerror(rc), starch_last_error(ctx));
        for (auto* c : ctxs) starch_destroy(c);
        return rc == STARCH_ERR_MEM ? ENOMEM : EINVAL;
    }
    if (!stdout_ok()) {
        if (getenv("STARCH_CLI_TEARDOWN")) for (auto* c : ctxs) starch_destroy(c);
        _exit(EIO);
    }
    if (stats) {
        starch_stats s;
        starch_get_stats(ctx, &s);
        print_stats(ctx, t0, s.input_bytes);
    }
    // The archive is out: the contexts' pinned buffers, device memory and
    // streams go back to the driver with the process instead of one by one
    // (STARCH_CLI_TEARDOWN=1: destroy them first)
    const char* td = getenv("STARCH_CLI_TEARDOWN");
    if (td && !strcmp(td, "1")) {
        const auto d0 = std::chrono::steady_clock::now();
        for (auto* c : ctxs) starch_destroy(c);
        if (stats)
            fprintf(stderr, "teardown %.1f ms\n",
                    std::chrono::duration<double>(std::chrono::steady_clock::now() - d0).count() * 1e3);
        return 0;
    }
    fflush(stderr);
    _exit(0);
}
