/*
 * include/starch3_amd.hpp -- the reference's C++ surface, class
 * starch3::Starch (include/starch3api.hpp:21-149 of alexpreynolds/starch3),
 * header-only over the C ABI of libstarch_amd.so (include/starch_amd.h).
 *
 * Same names, argument meaning and exit behaviour as the reference for the
 * configuration and I/O members (hpp:724-817, 890-919):
 *   set_note/get_note, set_compression_method/get_compression_method
 *   (k_bzip2 / k_gzip / k_compression_method_undefined, hpp:23-27),
 *   set_input_fn (exit ENODATA on a missing file, hpp:747-754),
 *   initialize_in_stream (stdin or the file, hpp:728-736),
 *   initialize_out_stream (stdout + the 4 magic bytes, hpp:765-769),
 *   initialize_out_compression_stream (gzip / undefined: exit ENOSYS,
 *   hpp:771-785), test_stdin_availability (tty stdin without a file: exit
 *   ENODATA, hpp:890-905), initialize_header_magic_bytes (ca5cad1a, hpp:907-910).
 * The reference's four pthreads (produce_line / consume_line / update_chr /
 * consume_tf_buffer, hpp:158-391) are replaced by compress_in_stream(): the
 * whole input goes to the GPU(s) at once -- transform, per-chromosome bzip2
 * -9 streams, archive -- and everything after the magic is written to the out
 * stream.
 *
 * The per-chromosome hand-off keeps the reference's shape: the types bed_t,
 * transform_state_t and shared_buffer_t (hpp:37-88), the bz_stream lifecycle
 * initialize_bz_stream_ptr / setup_bz_stream_callbacks / delete_bz_stream_ptr
 * and the block-close callbacks (hpp:126-129, 819-888), and
 *   static void process_tf_buffer(shared_buffer_t* sb)      (hpp:393-407)
 * which here FEEDS the patched-libbz2 ABI (include/starch_bzlib.h, on the
 * GPU): sb->tf_buffer[0, tf_buffer_size) goes through BZ2_bzCompress(BZ_FINISH)
 * of starch3::self's bz_stream, the stream is written to the out stream, and
 * the stream's block_close_functor (bz:bzlib.c:470) records the chromosome
 * (tf_state->current_chr, ->line_count) for the index; then, as in the
 * reference, the transformation state and tf_buffer are reset.  One bzip2
 * stream per chromosome: the bz_stream is re-initialised after each.
 * transform_and_flush_in_stream() drives it like consume_tf_buffer would
 * (GPU transform, one process_tf_buffer per chromosome); finish_tf_buffers()
 * writes the index.  As in the reference (cpp:10, hpp:921) the program defines
 * `starch3::Starch* starch3::self` and points it at its Starch.
 *
 * Link with -lstarch_amd.  Compiles as C++11.
 */
#ifndef STARCH3_AMD_HPP_
#define STARCH3_AMD_HPP_

#include <pthread.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <cinttypes>
#include <cstdio>
#include <cstdlib>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "starch_amd.h"
#include "starch_bzlib.h"

namespace starch3
{
class Starch
{
public:
    typedef enum compression_method {
        k_bzip2 = 0,
        k_gzip,
        k_compression_method_undefined
    } compression_method_t;

    // ---- the reference's pipeline types (hpp:37-88), same fields ---------------
    typedef struct bed {
        char* chr;
        size_t chr_capacity;
        char* start_str;
        size_t start_str_capacity;
        int64_t start;
        char* stop_str;
        size_t stop_str_capacity;
        int64_t stop;
        char* rem;
        size_t rem_capacity;
        int token;
    } bed_t;

    typedef struct transform_state {
        int64_t line_count;
        char* last_chr;
        int64_t last_start;
        int64_t last_stop;
        int64_t last_coord_diff;
        char* current_chr;
        int64_t current_start;
        int64_t current_stop;
        int64_t current_coord_diff;
        int64_t base_count_unique;
        int64_t base_count_nonunique;
    } transform_state_t;

    typedef struct shared_buffer {
        pthread_mutex_t lock;
        pthread_cond_t new_line_is_available;
        pthread_cond_t new_line_is_empty;
        pthread_cond_t new_chromosome_is_available;
        pthread_cond_t new_tf_buffer_is_available;
        char* in_line;
        size_t in_line_capacity;
        int next_in;
        int next_out;
        bool is_new_line_available;
        bool is_new_chromosome_available;
        bool is_new_tf_buffer_available;
        bool is_eof;
        FILE* in_stream;
        bed_t* bed;
        transform_state_t* tf_state;
        char* tf_line;
        size_t tf_line_capacity;
        char* tf_buffer;
        size_t tf_buffer_capacity;
        size_t tf_buffer_size;
    } shared_buffer_t;

    static const int tf_buffer_initial_length = 1024;   // hpp:152

    shared_buffer_t buffer;

    Starch()
        : _bz_stream_ptr(NULL), _bz_stream_used(false), _in_stream(NULL), _out_stream(NULL), _block_size(9),
          _reference_compat(false), _emit_index(true), _base_counts(false), _stream_end(4)
    {
        set_note(std::string());
        set_compression_method(k_compression_method_undefined);   // hpp:912-916
        initialize_header_magic_bytes();
        _devices.push_back(0);
        std::memset(&buffer, 0, sizeof(buffer));
        std::memset(&_tf_state, 0, sizeof(_tf_state));
        buffer.tf_state = &_tf_state;
    }
    ~Starch()
    {
        hook_drain(true);
        hook_stop();
        delete_bz_stream_ptr();
        delete_out_compression_stream();
        text_pool_clear();
        std::free(buffer.tf_buffer);
        std::free(_tf_state.current_chr);
        std::free(_tf_state.last_chr);
    }

    // ---- the bz_stream lifecycle (hpp:819-888) over the GPU-backed ABI ---------
    void initialize_bz_stream_ptr(void)
    {
        _bz_stream_ptr = new bz_stream;
        std::memset(_bz_stream_ptr, 0, sizeof(*_bz_stream_ptr));
        _bz_stream_ptr->bzalloc = NULL;
        _bz_stream_ptr->bzfree = NULL;
        _bz_stream_ptr->opaque = NULL;
        switch (BZ2_bzCompressInit(_bz_stream_ptr, _block_size, 0, 30)) {   // hpp:835-837
        case BZ_CONFIG_ERROR:
            std::fprintf(stderr, "Error: bzip2 initialization failed - library was miscompiled\n");
            std::exit(EINVAL);
        case BZ_PARAM_ERROR:
            std::fprintf(stderr, "Error: bzip2 initialization failed - incorrect parameters\n");
            std::exit(EINVAL);
        case BZ_MEM_ERROR:
            std::fprintf(stderr, "Error: bzip2 initialization failed - insufficient memory\n");
            std::exit(EINVAL);
        default:
            break;
        }
        _bz_stream_used = false;
    }
    // the reference installs &h, the address of its by-value parameter
    // (hpp:860, dangling); the handler here is the instance itself
    void setup_bz_stream_callbacks(starch3::Starch* h)
    {
        if (!_bz_stream_ptr) return;
        _bz_stream_ptr->handler = h;
        _bz_stream_ptr->block_close_functor = bzip2_block_close_static_callback;
    }
    void delete_bz_stream_ptr(void)
    {
        if (!_bz_stream_ptr) return;
        if (BZ2_bzCompressEnd(_bz_stream_ptr) == BZ_PARAM_ERROR) {   // hpp:868-872
            std::fprintf(stderr, "Error: Could not release internals of bz_stream pointer\n");
            std::exit(EINVAL);
        }
        delete _bz_stream_ptr;
        _bz_stream_ptr = NULL;
    }
    static void bzip2_block_close_static_callback(void* s)   // hpp:882-884
    {
        reinterpret_cast<starch3::Starch*>(s)->bzip2_block_close_callback();
    }
    // BZ_STREAM_END of a chromosome's stream: its index entry
    void bzip2_block_close_callback(void)
    {
        starch_segment sg;
        std::memset(&sg, 0, sizeof(sg));
        unsigned nb = 0, crc = 0;
        starch_bzstream_info(_bz_stream_ptr, &nb, &crc);
        sg.line_count = (uint64_t)_closing_lines;
        sg.text_bytes = _closing_text;
        sg.stream_offset = _stream_end;
        sg.stream_bytes = (uint64_t)_bz_stream_ptr->total_out_hi32 << 32 | _bz_stream_ptr->total_out_lo32;
        sg.name_len = _closing_chr.size();
        sg.n_blocks = nb;
        sg.combined_crc = crc;
        sg.unit = _closed.size();
        _stream_end += sg.stream_bytes;
        _closed.push_back(Closed(_closing_chr, sg));
    }

    // ---- I/O (hpp:724-769) ------------------------------------------------
    FILE* get_in_stream(void) { return _in_stream; }
    void set_in_stream(FILE* is) { _in_stream = is; }
    void initialize_in_stream(void)
    {
        FILE* in_fp = get_input_fn().empty() ? stdin : std::fopen(get_input_fn().c_str(), "r");
        if (!in_fp) {
            std::fprintf(stderr, "Error: Input file handle could not be created\n");
            std::exit(ENODATA);
        }
        set_in_stream(in_fp);
    }
    std::string get_input_fn(void) { return _input_fn; }
    void set_input_fn(std::string s)
    {
        struct stat buf;
        if (stat(s.c_str(), &buf) == 0) {
            _input_fn = s;
        } else {
            std::fprintf(stderr, "Error: Input file does not exist (%s)\n", s.c_str());
            std::exit(ENODATA);
        }
    }
    void set_out_stream(FILE* wo_stream) { _out_stream = wo_stream; }
    FILE* get_out_stream(void) { return _out_stream; }
    void initialize_out_stream(void)
    {
        set_out_stream(stdout);
        std::fwrite(_header_magic_bytes, sizeof(unsigned char), 4, _out_stream);
    }

    // ---- compression method (hpp:771-817) ----------------------------------
    void initialize_out_compression_stream(void)
    {
        switch (get_compression_method()) {
        case k_bzip2:
            // the device contexts open on a thread of their own (HIP start-up,
            // ~0.1-0.2 s) while the caller goes on to read its input; the
            // first call that needs them waits (open_devices)
            if (_ctx.empty() && !_opener.joinable()) _opener = std::thread([this]() { _open_rc = open_devices_now(); });
            break;
        case k_gzip:
            std::fprintf(stderr, "Error: This method is unsupported at this time\n");
            std::exit(ENOSYS);
        case k_compression_method_undefined:
            std::fprintf(stderr, "Error: This method is undefined\n");
            std::exit(ENOSYS);
        }
    }
    void delete_out_compression_stream(void)
    {
        if (_opener.joinable()) _opener.join();
        if (_ctx_aux) starch_destroy(_ctx_aux);
        _ctx_aux = NULL;
        for (size_t i = 0; i < _ctx.size(); ++i) starch_destroy(_ctx[i]);
        _ctx.clear();
    }
    std::string get_note(void) { return _note; }
    void set_note(std::string s) { _note = s; }
    compression_method_t get_compression_method(void) { return _compression_method; }
    void set_compression_method(compression_method_t t) { _compression_method = t; }

    void test_stdin_availability(void)   // hpp:890-905
    {
        struct stat stats;
        if (fstat(STDIN_FILENO, &stats) == -1) {
            int errsv = errno;
            std::fprintf(stderr, "Error: fstat() call failed (%s)",
                         (errsv == EBADF ? "EBADF" : (errsv == EIO ? "EIO" : "EOVERFLOW")));
            std::exit(errsv);
        }
        if (S_ISCHR(stats.st_mode) && !S_ISREG(stats.st_mode) && get_input_fn().empty()) {
            std::fprintf(stderr,
                         "Error: No input is specified; please redirect or pipe in formatted data, or specify filename\n");
            std::exit(ENODATA);
        }
    }
    void initialize_header_magic_bytes(void)
    {
        const unsigned char mb[] = {0xca, 0x5c, 0xad, 0x1a};   // ca5cad1a
        std::memcpy(_header_magic_bytes, mb, sizeof(_header_magic_bytes));
    }
    const unsigned char* get_header_magic_bytes(void) const { return _header_magic_bytes; }

    // ---- MI355X settings ----------------------------------------------------
    void set_devices(const std::vector<int>& d) { _devices = d.empty() ? std::vector<int>(1, 0) : d; }
    void set_block_size(int bs100k) { _block_size = bs100k; }
    void set_reference_compat(bool on) { _reference_compat = on; }
    void set_emit_index(bool on) { _emit_index = on; }
    // per-segment base_count_unique / base_count_nonunique (hpp:61-62) in the index
    void set_base_counts(bool on) { _base_counts = on; }
    starch_ctx* context(void)
    {
        if (_opener.joinable()) _opener.join();
        return _ctx.empty() ? NULL : _ctx[0];
    }

    // ---- the hot path -------------------------------------------------------
    // In-memory: BED bytes -> the whole archive (magic included).  Returns a
    // STARCH_* status.
    int compress(const void* bed, size_t n, std::vector<unsigned char>* archive)
    {
        int rc = open_devices();
        if (rc) return rc;
        starch_options o = options();
        rc = _ctx.size() > 1 ? starch_encode_multi_host(&_ctx[0], (int)_ctx.size(), bed, n, &o)
                             : starch_encode_host(_ctx[0], bed, n, &o);
        if (rc) return rc;
        uint64_t sz = 0;
        if ((rc = starch_archive_size(_ctx[0], &sz))) return rc;
        archive->resize(sz);
        return sz ? starch_archive_copy(_ctx[0], &(*archive)[0], sz) : STARCH_OK;
    }

    // Read the in stream to EOF and write everything after the magic (which
    // initialize_out_stream wrote) to the out stream.  One device: the
    // streaming session (starch_stream_*) -- the input is read in 16 MiB
    // pieces straight into the session's pinned window and the archive bytes
    // are written as they finish, so memory stays at about two batches
    // (hpp:158-199 reads line by line).  Several devices: batches of whole
    // chromosome runs (for_each_run_batch), each batch's runs sharded over the
    // devices (LPT), encoded concurrently and their streams written in input
    // order; the index of all of them at the end.  Host memory: one batch (or
    // the longest chromosome run, which one device must encode whole).
    int compress_in_stream(void)
    {
        int rc;
        if (_devices.size() == 1) {
            bool done = false;
            if ((rc = compress_mapped(done)) || done) return rc;
        }
        if ((rc = open_devices())) return rc;
        if (_ctx.size() > 1) return compress_in_stream_multi();
        starch_ctx* c = _ctx[0];
        starch_options o = options();
        if ((rc = starch_stream_begin(c, &o, 0))) return rc;
        std::vector<unsigned char> out(1 << 24);
        uint64_t skip = 4;   // the magic, already written
        auto drain = [&]() -> int {
            for (;;) {
                uint64_t got = 0;
                const int r = starch_stream_read(c, &out[0], out.size(), &got);
                if (r || !got) return r;
                const uint64_t off = skip < got ? skip : got;
                skip -= off;
                if (got > off) std::fwrite(&out[off], 1, got - off, _out_stream);
            }
        };
        for (;;) {
            void* w = NULL;
            uint64_t cap = 0;
            if ((rc = starch_stream_window(c, 1 << 24, &w, &cap))) return rc;
            const size_t k = std::fread(w, 1, cap < (1u << 24) ? (size_t)cap : (size_t)(1u << 24), _in_stream);
            if (k == 0) break;
            if ((rc = starch_stream_commit(c, k)) || (rc = drain())) return rc;
        }
        if ((rc = starch_stream_end(c)) || (rc = drain())) return rc;
        std::fflush(_out_stream);
        return STARCH_OK;
    }

    // smallest file the mapped paths take (tests: STARCH_HPP_MAP_MIN bytes)
    static uint64_t map_min(uint64_t dflt)
    {
        const char* e = std::getenv("STARCH_HPP_MAP_MIN");
        return e && std::atoll(e) > 0 ? (uint64_t)std::atoll(e) : dflt;
    }

    // compress_in_stream for a regular file of >= 256 MiB that ends at its
    // st_size, on one device: the file is mapped and its pages faulted in by
    // 16 threads while the device opens (initialize_out_compression_stream
    // started it), then one starch_encode_host_into -- the library registers
    // the mapping for the call and DMAs chromosome batches from it while
    // finished ones come back -- and the archive after the magic to the out
    // stream.  done = false: not taken (pipe, small or growing file,
    // STARCH_HPP_MAP=0).
    int compress_mapped(bool& done)
    {
        done = false;
        const char* e = std::getenv("STARCH_HPP_MAP");
        if (!_in_stream || (e && !std::strcmp(e, "0"))) return STARCH_OK;
        const int fd = fileno(_in_stream);
        struct stat st;
        const off_t cur = lseek(fd, 0, SEEK_CUR);
        if (fd < 0 || fstat(fd, &st) != 0 || !S_ISREG(st.st_mode) || cur < 0 ||
            (uint64_t)st.st_size < (uint64_t)cur + map_min(256ull << 20))
            return STARCH_OK;
        unsigned char x;
        if (pread(fd, &x, 1, st.st_size) != 0) return STARCH_OK;
        const uint64_t pg = (uint64_t)sysconf(_SC_PAGESIZE), mo = (uint64_t)cur & ~(pg - 1);
        const uint64_t len = (uint64_t)st.st_size - mo, n = (uint64_t)st.st_size - (uint64_t)cur;
        void* m = mmap(NULL, len, PROT_READ, MAP_PRIVATE, fd, (off_t)mo);
        if (m == MAP_FAILED) return STARCH_OK;
        done = true;
        // the archive buffer, not zero-filled: only the archive's pages are
        // touched, and its first n/8 (BED text compresses ~9x) are written
        // here beside the input's faults, while the device may still be
        // opening, so the finished batches' device-to-host copies do not
        // fault them in one by one
        uint64_t cap = n / 2 + (16ull << 20), got = 0;
        std::unique_ptr<char[]> out(new char[cap]);
        {
            (void)madvise(m, len, MADV_WILLNEED);
            const int nt = 16;
            const uint64_t per = ((len + nt - 1) / nt + pg - 1) & ~(pg - 1);
            const uint64_t pre = std::min<uint64_t>(cap, n / 8), oper = ((pre + nt - 1) / nt + pg - 1) & ~(pg - 1);
            std::vector<std::thread> th;
            std::vector<unsigned> sink(nt, 0);
            for (int t = 0; t < nt; ++t)
                th.push_back(std::thread([&, t]() {
                    const volatile unsigned char* p = static_cast<const unsigned char*>(m);
                    unsigned acc = 0;
                    for (uint64_t o = (uint64_t)t * per; o < len && o < (uint64_t)(t + 1) * per; o += pg) acc += p[o];
                    sink[t] = acc;
                    volatile char* q = out.get();
                    for (uint64_t o = (uint64_t)t * oper; o < pre && o < (uint64_t)(t + 1) * oper; o += pg) q[o] = 0;
                }));
            for (size_t t = 0; t < th.size(); ++t) th[t].join();
        }
        int rc = open_devices();
        if (!rc) {
            starch_ctx* c = _ctx[0];
            const starch_options o = options();
            const unsigned char* bed = static_cast<const unsigned char*>(m) + ((uint64_t)cur - mo);
            rc = starch_encode_host_into(c, bed, n, &o, out.get(), cap, &got);
            if (rc == STARCH_ERR_MEM && got > cap) {      // larger than guessed: the archive is still in the context
                out.reset(new char[got]);
                rc = starch_archive_copy(c, out.get(), got);
            }
            if (!rc && got > 4) std::fwrite(out.get() + 4, 1, got - 4, _out_stream);   // (the magic is out already)
        }
        munmap(m, len);
        (void)lseek(fd, st.st_size, SEEK_SET);
        std::fflush(_out_stream);
        return rc;
    }

    // The in stream in batches of whole chromosome runs (units of
    // starch_plan_units_from): 16 MiB pieces are read until at least `batch`
    // bytes are held; every run but the last (which may go on) is handed to
    // f(bytes, units, count); the last run carries over with the sscanf values
    // current before it (hpp:306-307).  A run longer than a batch is held
    // whole.  At EOF, or at a 0xFF (which reads as EOF, hpp:181), every run
    // goes.  Returns the first nonzero status of f.
    struct FileReader;
    template <class F>
    int for_each_run_batch(uint64_t batch, F f)
    {
        const char* eb = std::getenv("STARCH_HPP_BATCH");   // tests: small batches
        if (eb && std::atoll(eb) > 0) batch = (uint64_t)std::atoll(eb);
        FileReader rd(_in_stream);
        {
            bool done = false;
            const int rc = mapped_batches(rd, batch, f, done);
            if (rc || done) return rc;
        }
        InBuf buf;
        std::vector<starch_unit> units(4096);
        int64_t is = 0, ip = 0;
        bool eof = false;
        uint64_t want = batch;
        uint64_t scanned = 0;      // bytes of buf known to hold no newline after the last complete line
        for (;;) {
            while (!eof && buf.size() < want) {
                const size_t o = buf.size();
                const size_t piece = rd.regular() ? (size_t)std::max<uint64_t>(want - o, 1u << 24) : (size_t)(1u << 24);
                buf.resize(o + piece);
                const size_t k = rd.read(&buf[o], piece);
                buf.resize(o + k);
                if (k == 0) eof = true;
            }
            uint64_t lim = buf.size();
            if (!eof) {            // complete lines only
                while (lim > scanned && buf[lim - 1] != '\n') --lim;
                if (lim == scanned && (scanned == 0 || buf[scanned - 1] != '\n')) lim = 0;
            }
            uint64_t nu = 0;
            int rc = lim ? starch_plan_units_from(&buf[0], lim, units.size(), is, ip, &units[0], &nu) : STARCH_OK;
            if (rc) return rc;
            uint64_t covered = 0;
            for (uint64_t k = 0; k < nu; ++k) covered = units[k].offset + units[k].length;
            if (covered < lim) eof = true;        // a 0xFF: the input ends there
            const uint64_t take = eof ? nu : (nu ? nu - 1 : 0);
            if (take == 0 && !eof) {              // one run so far: read on
                scanned = lim;
                want = buf.size() + batch;
                continue;
            }
            if (take && (rc = f(&buf[0], &units[0], take))) return rc;
            if (eof) return STARCH_OK;
            const starch_unit& last = units[nu - 1];
            is = last.init_start;
            ip = last.init_stop;
            buf.erase_front(last.offset);
            scanned = 0;
            want = batch;
        }
    }

    // for_each_run_batch over a regular file of >= 64 MiB that ends at its
    // st_size: the file is mapped, its runs planned in one pass (the library's
    // 0xFF scan runs on 16 threads and faults the mapping in) and handed to f
    // in batches straight from the mapping -- no read copies, and the library
    // DMAs each batch from the page cache.  done = false: not taken (pipe,
    // small or growing file, STARCH_HPP_MAP=0), the caller reads instead.
    template <class F>
    int mapped_batches(FileReader& rd, uint64_t batch, F& f, bool& done)
    {
        done = false;
        const char* e = std::getenv("STARCH_HPP_MAP");
        if (!rd.regular() || (e && !std::strcmp(e, "0"))) return STARCH_OK;
        struct stat st;
        if (fstat(rd.fd, &st) != 0 || (uint64_t)st.st_size < rd.off + map_min(64ull << 20)) return STARCH_OK;
        unsigned char x;
        if (pread(rd.fd, &x, 1, st.st_size) != 0) return STARCH_OK;   // more than st_size: read it instead
        const uint64_t pg = (uint64_t)sysconf(_SC_PAGESIZE), mo = rd.off & ~(pg - 1);
        const uint64_t len = (uint64_t)st.st_size - mo, n = (uint64_t)st.st_size - rd.off;
        void* m = mmap(NULL, len, PROT_READ, MAP_PRIVATE, rd.fd, (off_t)mo);
        if (m == MAP_FAILED) return STARCH_OK;
        const unsigned char* base = static_cast<const unsigned char*>(m) + (rd.off - mo);
        std::vector<starch_unit> units(1u << 16);
        uint64_t nu = 0;
        int rc = starch_plan_units_from(base, n, units.size(), 0, 0, &units[0], &nu);
        // the whole mapping page-locked once (~12 ms per GB of page-cached
        // file), so every batch's copy runs by DMA (one device: the
        // multi-device batches copy from it as pageable memory)
        const bool reg = !rc && _devices.size() == 1 && starch_host_register(m, (len + pg - 1) & ~(pg - 1)) == STARCH_OK;
        for (uint64_t k = 0; !rc && k < nu;) {   // batches of whole runs, >= batch bytes each
            uint64_t j = k, b = 0;
            while (j < nu && (j == k || b < batch)) b += units[j++].length;
            rc = f(base, &units[k], j - k);
            k = j;
        }
        if (reg) (void)starch_host_unregister(m);
        munmap(m, len);
        rd.off = (uint64_t)st.st_size;   // (a 0xFF ends the input there: nothing after it is read)
        done = true;
        return rc;
    }

    // the in stream's bytes, read with 16 pread(2) threads when it is a
    // regular file (one fread stream from the page cache runs at a few GB/s),
    // else with fread
    struct FileReader {
        FILE* f;
        int fd;
        bool reg;
        uint64_t off;
        explicit FileReader(FILE* in) : f(in), fd(-1), reg(false), off(0)
        {
            struct stat st;
            fd = in ? fileno(in) : -1;
            if (fd >= 0 && fstat(fd, &st) == 0 && S_ISREG(st.st_mode) && st.st_size > 0) {
                const off_t o = lseek(fd, 0, SEEK_CUR);
                if (o >= 0) {
                    reg = true;
                    off = (uint64_t)o;
                }
            }
        }
        ~FileReader()
        {
            if (reg) (void)lseek(fd, (off_t)off, SEEK_SET);   // the FILE's position where reading stopped
        }
        bool regular() const { return reg; }
        size_t read(unsigned char* dst, size_t n)
        {
            if (!reg) return std::fread(dst, 1, n, f);
            const int nt = 16;
            const size_t per = (n + nt - 1) / nt;
            std::vector<size_t> got(nt, 0);
            std::vector<std::thread> th;
            for (int t = 0; t < nt; ++t)
                th.push_back(std::thread([&, t]() {
                    const size_t b = (size_t)t * per, e = std::min(n, b + per);
                    size_t q = b;
                    while (q < e) {
                        const ssize_t r = pread(fd, dst + q, e - q, (off_t)(off + q));
                        if (r < 0 && errno == EINTR) continue;
                        if (r <= 0) break;
                        q += (size_t)r;
                    }
                    got[t] = q > b ? q - b : 0;
                }));
            for (size_t t = 0; t < th.size(); ++t) th[t].join();
            size_t k = 0;                          // the bytes read contiguously from the start
            for (int t = 0; t < nt; ++t) {
                k += got[t];
                const size_t b = (size_t)t * per;
                if (b >= n || got[t] < std::min(n, b + per) - b) break;
            }
            off += k;
            return k;
        }
    };

    // a growable byte buffer that is not zero-filled (std::vector::resize
    // zero-fills every 16 MiB piece before it is read into)
    struct InBuf {
        std::unique_ptr<unsigned char[]> p;
        size_t n, cap;
        InBuf() : n(0), cap(0) {}
        size_t size() const { return n; }
        unsigned char& operator[](size_t i) { return p[i]; }
        void resize(size_t k)
        {
            if (k > cap) {
                const size_t c = k + k / 2;
                std::unique_ptr<unsigned char[]> q(new unsigned char[c]);
                if (n) std::memcpy(q.get(), p.get(), std::min(n, k));
                p.swap(q);
                cap = c;
            }
            n = k;
        }
        void erase_front(size_t k)
        {
            if (k >= n) { n = 0; return; }
            std::memmove(p.get(), p.get() + k, n - k);
            n -= k;
        }
    };

    int compress_in_stream_multi(void)
    {
        const starch_options o = options();
        if (o.reference_compat) {      // the reference's stdout is the magic alone: read, write nothing
            std::vector<unsigned char> sink(1u << 24);
            while (std::fread(&sink[0], 1, sink.size(), _in_stream) > 0) {}
            std::fflush(_out_stream);
            return STARCH_OK;
        }
        const int nd = (int)_ctx.size();
        std::vector<starch_segment> all;
        std::vector<std::string> all_names;
        uint64_t end = 4, next_unit = 0;
        int rc = for_each_run_batch(1ull << 30, [&](const unsigned char* bed, const starch_unit* u, uint64_t n) -> int {
            std::vector<int32_t> shard(n);
            int r = starch_assign_shards(u, n, nd, &shard[0]);
            if (r) return r;
            std::vector<std::vector<starch_unit> > mine(nd);
            std::vector<std::vector<uint64_t> > ids(nd);
            for (uint64_t k = 0; k < n; ++k) {
                mine[shard[k]].push_back(u[k]);
                ids[shard[k]].push_back(next_unit + k);
            }
            std::vector<int> codes(nd, 0);
            std::vector<std::thread> th;
            for (int d = 0; d < nd; ++d)
                th.push_back(std::thread([&, d]() {
                    starch_options od = o;
                    od.emit_index = 0;
                    codes[d] = mine[d].empty() ? STARCH_OK
                                               : starch_encode_units_host(_ctx[d], bed, &mine[d][0], &ids[d][0],
                                                                          mine[d].size(), &od);
                }));
            for (size_t t = 0; t < th.size(); ++t) th[t].join();
            for (int d = 0; d < nd; ++d) if (codes[d]) return codes[d];
            // every device's segments and streams, then the batch's layout in unit order
            std::vector<starch_segment> segs;
            std::vector<std::string> names;
            std::vector<std::vector<unsigned char> > streams(nd);
            std::vector<int> dev_of;
            for (int d = 0; d < nd; ++d) {
                if (mine[d].empty()) continue;
                uint64_t ns = 0, sb = 0;
                const void* dp = NULL;
                if ((r = starch_segment_count(_ctx[d], &ns)) || (r = starch_streams_device(_ctx[d], &dp, &sb))) return r;
                streams[d].resize(sb);
                if (sb && (r = starch_streams_copy(_ctx[d], &streams[d][0], sb))) return r;
                std::vector<starch_segment> sd(ns + 1);
                if (ns && (r = starch_segments(_ctx[d], &sd[0], ns))) return r;
                for (uint64_t k = 0; k < ns; ++k) {
                    std::string nm(sd[k].name_len, '\0');
                    uint64_t len = 0;
                    if ((r = starch_segment_name(_ctx[d], k, nm.empty() ? NULL : &nm[0], nm.size(), &len))) return r;
                    segs.push_back(sd[k]);
                    names.push_back(nm);
                    dev_of.push_back(d);
                }
            }
            const uint64_t ns = segs.size();
            std::vector<uint64_t> unit_of(ns + 1), bytes(ns + 1), order(ns + 1), off(ns + 1);
            for (uint64_t k = 0; k < ns; ++k) { unit_of[k] = segs[k].unit; bytes[k] = segs[k].stream_bytes; }
            uint64_t nend = end;
            if (ns && (r = starch_archive_layout(&unit_of[0], &bytes[0], ns, end, &order[0], &off[0], &nend))) return r;
            for (uint64_t j = 0; j < ns; ++j) {
                const uint64_t k = order[j];
                const std::vector<unsigned char>& sv = streams[dev_of[k]];
                if (segs[k].stream_bytes) std::fwrite(&sv[segs[k].stream_offset], 1, segs[k].stream_bytes, _out_stream);
                starch_segment g = segs[k];
                g.stream_offset = off[k];          // (the layout's offsets are by segment)
                all.push_back(g);
                all_names.push_back(names[k]);
            }
            end = nend;
            next_unit += n;
            return STARCH_OK;
        });
        if (rc) return rc;
        if (o.emit_index && !o.reference_compat) {
            std::vector<const char*> np(all.size() + 1);
            std::vector<uint64_t> nl(all.size() + 1);
            for (size_t k = 0; k < all.size(); ++k) { np[k] = all_names[k].data(); nl[k] = all_names[k].size(); }
            uint64_t n = 0;
            rc = starch_build_index_opt(all.empty() ? NULL : &all[0], &np[0], &nl[0], all.size(), end, &o, NULL, 0, &n);
            if (rc) return rc;
            std::vector<char> idx(n + 1);
            rc = starch_build_index_opt(all.empty() ? NULL : &all[0], &np[0], &nl[0], all.size(), end, &o, &idx[0], n, &n);
            if (rc) return rc;
            std::fwrite(&idx[0], 1, n, _out_stream);
        }
        std::fflush(_out_stream);
        return STARCH_OK;
    }

    // The per-chromosome hand-off (hpp:393-407), static as in the reference:
    // the chromosome's transformed text goes through starch3::self's bz_stream
    // (BZ2_bzCompress with BZ_FINISH, on the GPU), its stream to the out stream;
    // the block-close callback records the index entry.  Then the
    // transformation state and tf_buffer are reset as in the reference.
    static void process_tf_buffer(shared_buffer_t* sb);

    // consume_tf_buffer's loop (hpp:371-391) over the GPU transform: the in
    // stream is read in batches of whole chromosome runs (for_each_run_batch;
    // memory: one batch, or the longest run -- the reference's tf_buffer
    // holds a whole chromosome's text too, hpp:409-426), each batch is
    // transformed on the GPU with the sscanf values current before it, and
    // every chromosome segment is handed to process_tf_buffer in input order.
    int transform_and_flush_in_stream(void)
    {
        _tr.t0 = _tr.last = Trace::now();
        // two contexts: batch k is transformed (on a helper thread) while the
        // main thread hands batch k-1's chromosomes to process_tf_buffer; the
        // devices may still be opening while the first batch is read
        starch_ctx* c[2] = {NULL, NULL};
        uint64_t k = 0;
        int pending = -1;              // context holding a transformed batch not yet handed off
        int rc = for_each_run_batch(512ull << 20, [&](const unsigned char* bed, const starch_unit* u, uint64_t n) -> int {
            const uint64_t beg = u[0].offset, len = u[n - 1].offset + u[n - 1].length - beg;
            _tr.lap(_tr.read);
            if (!c[0]) {
                const int r = open_devices();
                if (r) return r;
                c[0] = _ctx[0];
                if (!_ctx_aux && starch_create(_devices[0], &_ctx_aux) != STARCH_OK) _ctx_aux = NULL;
                c[1] = _ctx_aux;       // (none: one context, no overlap)
                _tr.lap(_tr.open);
            }
            const int cur = c[1] ? (int)(k & 1) : 0;
            int tr = STARCH_OK, r = STARCH_OK;
            if (pending >= 0 && c[1]) {
                std::thread t([&]() {
                    tr = starch_transform_host_init(c[cur], bed + beg, len, u[0].init_start, u[0].init_stop);
                });
                r = flush_transformed(c[pending]);
                t.join();
            } else {
                if (pending >= 0) r = flush_transformed(c[pending]);
                if (!r) tr = starch_transform_host_init(c[cur], bed + beg, len, u[0].init_start, u[0].init_stop);
            }
            _tr.lap(_tr.tf);
            ++k;
            pending = cur;
            return r ? r : tr;
        });
        if (!rc && pending >= 0) rc = flush_transformed(c[pending]);
        return rc;
    }

    // hand every segment of the context's last transform to process_tf_buffer
    int flush_transformed(starch_ctx* c)
    {
        int rc;
        uint64_t nseg = 0, tb = 0;
        if ((rc = starch_segment_count(c, &nseg)) || (rc = starch_text_size(c, &tb))) return rc;
        std::vector<starch_segment> segs(nseg + 1);
        if (nseg && (rc = starch_segments(c, &segs[0], nseg))) return rc;
        for (uint64_t s = 0; s < nseg; ++s) {
            std::string name(segs[s].name_len, '\0');
            uint64_t len = 0;
            if ((rc = starch_segment_name(c, s, name.empty() ? NULL : &name[0], name.size(), &len))) return rc;
            // the state consume_line leaves for the flush: current_chr, line_count, tf_buffer
            std::free(_tf_state.current_chr);
            _tf_state.current_chr = static_cast<char*>(std::malloc(name.size() + 1));
            std::memcpy(_tf_state.current_chr, name.data(), name.size());
            _tf_state.current_chr[name.size()] = '\0';
            _tf_state.line_count = (int64_t)segs[s].line_count;
            if (!text_pool_put(buffer.tf_buffer)) std::free(buffer.tf_buffer);
            buffer.tf_buffer_capacity = segs[s].text_bytes + 1;
            buffer.tf_buffer = text_pool_get(buffer.tf_buffer_capacity);
            if (!buffer.tf_buffer) return STARCH_ERR_MEM;
            // the segment's text straight into its tf_buffer (transform-only
            // results carry the text offset in stream_offset)
            if ((rc = starch_text_read(c, segs[s].stream_offset, buffer.tf_buffer, segs[s].text_bytes))) return rc;
            buffer.tf_buffer_size = segs[s].text_bytes;
            _closing_name_len = name.size();
            _tr.lap(_tr.text);
            process_tf_buffer(&buffer);
            _tr.lap(_tr.hand);
            if (_hook_error) return STARCH_ERR_INTERNAL;
        }
        return STARCH_OK;
    }

    // Write the index of the streams process_tf_buffer wrote (after the magic
    // initialize_out_stream wrote and the streams themselves).
    int finish_tf_buffers(void)
    {
        _tr.last = Trace::now();
        hook_drain(true);
        hook_stop();
        _tr.lap(_tr.drain);
        _tr.report();
        if (_hook_error) return STARCH_ERR_INTERNAL;
        if (_emit_index) {
            std::vector<starch_segment> segs;
            std::vector<const char*> names;
            std::vector<uint64_t> lens;
            for (size_t i = 0; i < _closed.size(); ++i) {
                segs.push_back(_closed[i].seg);
                names.push_back(_closed[i].chr.data());
                lens.push_back(_closed[i].chr.size());
            }
            uint64_t n = 0;
            starch_options o = options();
            int rc = starch_build_index_opt(segs.empty() ? NULL : &segs[0], names.empty() ? NULL : &names[0],
                                            lens.empty() ? NULL : &lens[0], segs.size(), _stream_end, &o, NULL, 0, &n);
            if (rc) return rc;
            std::vector<char> idx(n);
            rc = starch_build_index_opt(segs.empty() ? NULL : &segs[0], names.empty() ? NULL : &names[0],
                                        lens.empty() ? NULL : &lens[0], segs.size(), _stream_end, &o, &idx[0], n, &n);
            if (rc) return rc;
            std::fwrite(&idx[0], 1, n, _out_stream);
        }
        _closed.clear();
        _stream_end = 4;
        std::fflush(_out_stream);
        return STARCH_OK;
    }

private:
    // ---- process_tf_buffer's hand-off, asynchronous ---------------------------
    // A chromosome handed to process_tf_buffer is compressed by one of four
    // worker threads, each with its own bz_stream on the patched-libbz2 ABI
    // (BZ2_bzCompressInit / BZ2_bzCompress(BZ_FINISH) / block_close_functor /
    // BZ2_bzCompressEnd: the GPU encodes up to four streams at once), while the
    // caller goes on to the next chromosome; streams are written to the out
    // stream, and their index entries recorded, strictly in hand-off order.
    // STARCH_HOOK_SYNC=1: each chromosome through self's own bz_stream at once.
    // The workers' streams carry their own block-close callbacks (they record
    // the index entries in hand-off order), so a block_close_functor a caller
    // installs on self's stream is not called on this path; STARCH_HOOK_SYNC=1
    // codes through self's stream (re-initialised per chromosome by
    // initialize_bz_stream_ptr / setup_bz_stream_callbacks, as the reference's
    // hand-off does).
    struct HookJob {
        uint64_t seq;
        std::string chr;
        int64_t lines;
        char* text;
        size_t len;
        std::unique_ptr<char[]> out;
        uint64_t out_bytes;
        unsigned nb, crc;
        bool closed;                     // block_close_functor ran (BZ_STREAM_END)
        int rc;
        bz_stream* z;
    };
    std::mutex _hmu;
    std::condition_variable _hcv;
    std::deque<HookJob*> _hq;            // waiting for a worker
    std::map<uint64_t, HookJob*> _hdone; // finished, not yet written
    std::vector<std::thread> _hworkers;
    uint64_t _hseq = 0, _hwrite = 0;     // next hand-off / next to write
    bool _hstop = false;

    static bool hook_sync()
    {
        const char* e = std::getenv("STARCH_HOOK_SYNC");
        return e && !std::strcmp(e, "1");
    }
    static void hook_block_close(void* h)   // the worker's stream reached BZ_STREAM_END
    {
        HookJob* j = static_cast<HookJob*>(h);
        starch_bzstream_info(j->z, &j->nb, &j->crc);
        j->out_bytes = (uint64_t)j->z->total_out_hi32 << 32 | j->z->total_out_lo32;
        j->closed = true;
    }
    void hook_worker()
    {
        for (;;) {
            HookJob* j = NULL;
            {
                std::unique_lock<std::mutex> lk(_hmu);
                while (_hq.empty() && !_hstop) _hcv.wait(lk);
                if (_hq.empty()) return;
                j = _hq.front();
                _hq.pop_front();
            }
            bz_stream z;
            std::memset(&z, 0, sizeof(z));
            j->z = &z;
            j->rc = BZ2_bzCompressInit(&z, _block_size, 0, 30);
            if (j->rc == BZ_OK) {
                z.handler = j;
                z.block_close_functor = hook_block_close;
                // room for the whole stream: one drain (bzip2 grows incompressible text by < 1 %)
                const size_t cap = j->len + j->len / 64 + (1u << 20);
                j->out.reset(new char[cap]);
                z.next_in = j->text;
                z.avail_in = (unsigned int)j->len;
                size_t got = 0;
                int r;
                const double tb = Trace::now();
                do {
                    const size_t room = std::min<size_t>(cap - got, 0xFFFFFFFFu);
                    z.next_out = j->out.get() + got;
                    z.avail_out = (unsigned int)room;
                    r = BZ2_bzCompress(&z, BZ_FINISH);
                    got += room - z.avail_out;
                } while (r == BZ_FINISH_OK && got < cap);
                {
                    std::lock_guard<std::mutex> lk(_tr.mu);
                    _tr.bz += Trace::now() - tb;
                }
                j->rc = r == BZ_STREAM_END && j->closed ? BZ_OK : (r < 0 ? r : BZ_SEQUENCE_ERROR);
                BZ2_bzCompressEnd(&z);
            }
            if (!text_pool_put(j->text)) std::free(j->text);
            j->text = NULL;
            {
                std::lock_guard<std::mutex> lk(_hmu);
                _hdone[j->seq] = j;
            }
            _hcv.notify_all();
        }
    }
    // write the finished streams that are next in hand-off order (all: wait
    // for every stream handed off; else at most `keep` may stay in flight)
    void hook_drain(bool all, size_t keep = 8)
    {
        for (;;) {
            HookJob* j = NULL;
            {
                std::unique_lock<std::mutex> lk(_hmu);
                const bool must = all ? _hwrite < _hseq : (_hseq - _hwrite > keep);
                if (must)
                    while (_hdone.find(_hwrite) == _hdone.end()) _hcv.wait(lk);
                std::map<uint64_t, HookJob*>::iterator it = _hdone.find(_hwrite);
                if (it == _hdone.end()) return;
                j = it->second;
                _hdone.erase(it);
                ++_hwrite;
            }
            if (j->rc != BZ_OK) {
                std::fprintf(stderr, "Error: bzip2 compression failed (%d)\n", j->rc);
                _hook_error = true;
            } else {
                if (j->out_bytes && _out_stream) std::fwrite(j->out.get(), 1, j->out_bytes, _out_stream);
                starch_segment sg;
                std::memset(&sg, 0, sizeof(sg));
                sg.line_count = (uint64_t)j->lines;
                sg.text_bytes = j->len;
                sg.stream_offset = _stream_end;
                sg.stream_bytes = j->out_bytes;
                sg.name_len = j->chr.size();
                sg.n_blocks = j->nb;
                sg.combined_crc = j->crc;
                sg.unit = _closed.size();
                _stream_end += sg.stream_bytes;
                _closed.push_back(Closed(j->chr, sg));
            }
            delete j;
        }
    }
    void hook_submit(const std::string& chr, int64_t lines, char* text, size_t len)
    {
        HookJob* j = new HookJob();
        j->chr = chr;
        j->lines = lines;
        j->text = text;
        j->len = len;
        j->out_bytes = 0;
        j->nb = j->crc = 0;
        j->closed = false;
        j->rc = BZ_OK;
        j->z = NULL;
        {
            std::lock_guard<std::mutex> lk(_hmu);
            j->seq = _hseq++;
            _hq.push_back(j);
            if (_hworkers.empty()) {
                _hstop = false;
                for (int i = 0; i < 4; ++i) _hworkers.push_back(std::thread(&Starch::hook_worker, this));
            }
        }
        _hcv.notify_all();
        hook_drain(false);
    }
    void hook_stop()
    {
        {
            std::lock_guard<std::mutex> lk(_hmu);
            _hstop = true;
        }
        _hcv.notify_all();
        for (size_t i = 0; i < _hworkers.size(); ++i) _hworkers[i].join();
        _hworkers.clear();
    }

    // STARCH_HOOK_TRACE=1: where transform_and_flush_in_stream's time goes (stderr)
    struct Trace {
        double t0 = 0, last = 0, open = 0, read = 0, tf = 0, text = 0, hand = 0, drain = 0, bz = 0;
        std::mutex mu;
        static double now()
        {
            return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
        }
        void lap(double& acc)
        {
            const double t = now();
            acc += t - last;
            last = t;
        }
        void report()
        {
            const char* e = std::getenv("STARCH_HOOK_TRACE");
            if (!e || std::strcmp(e, "1")) return;
            std::fprintf(stderr, "hook trace: total %.1f ms  device open wait %.1f  read+plan %.1f  transform (not overlapped) %.1f  text %.1f"
                         "  hand-off %.1f  final drain %.1f  (workers: bzCompress %.1f)\n", (now() - t0) * 1e3, open * 1e3, read * 1e3, tf * 1e3,
                         text * 1e3, hand * 1e3, drain * 1e3, bz * 1e3);
        }
    } _tr;

    struct Closed {
        std::string chr;
        starch_segment seg;
        Closed(const std::string& c, const starch_segment& s) : chr(c), seg(s) {}
    };

    // hpp:523-536
    static void reset_transformation_state(transform_state_t** tfs)
    {
        (*tfs)->line_count = 0;
        (*tfs)->last_start = 0;
        (*tfs)->last_stop = 0;
        (*tfs)->last_coord_diff = 0;
        (*tfs)->current_start = 0;
        (*tfs)->current_stop = 0;
        (*tfs)->current_coord_diff = 0;
        (*tfs)->base_count_unique = 0;
        (*tfs)->base_count_nonunique = 0;
    }

    int open_devices(void)
    {
        if (_opener.joinable()) {
            _opener.join();
            if (_open_rc) return _open_rc;
        }
        return open_devices_now();
    }
    int open_devices_now(void)
    {
        if (!_ctx.empty()) return STARCH_OK;
        for (size_t i = 0; i < _devices.size(); ++i) {
            starch_ctx* c = NULL;
            int rc = starch_create(_devices[i], &c);
            if (rc) {
                for (size_t k = 0; k < _ctx.size(); ++k) starch_destroy(_ctx[k]);
                _ctx.clear();
                return rc;
            }
            _ctx.push_back(c);
        }
        return STARCH_OK;
    }
    starch_options options(void)
    {
        starch_options o;
        starch_options_init(&o);
        o.block_size_100k = _block_size;
        o.emit_index = _emit_index ? 1 : 0;
        o.reference_compat = _reference_compat ? 1 : 0;
        o.note = _note.empty() ? NULL : _note.c_str();
        o.base_counts = _base_counts ? 1 : 0;
        return o;
    }

    std::string _input_fn;
    std::string _note;
    bz_stream* _bz_stream_ptr;
    bool _bz_stream_used;
    FILE* _in_stream;
    FILE* _out_stream;
    compression_method_t _compression_method;
    unsigned char _header_magic_bytes[4];
    std::vector<int> _devices;
    std::vector<starch_ctx*> _ctx;
    int _block_size;
    bool _reference_compat;
    bool _emit_index;
    bool _base_counts;
    transform_state_t _tf_state;
    std::vector<Closed> _closed;
    uint64_t _stream_end;
    std::string _closing_chr;
    int64_t _closing_lines = 0;
    uint64_t _closing_text = 0;
    size_t _closing_name_len = 0;
    bool _hook_error = false;
    std::thread _opener;
    int _open_rc = STARCH_OK;
    starch_ctx* _ctx_aux = NULL;         // transform_and_flush_in_stream's second context
    // tf_buffers of flush_transformed: page-aligned, page-locked once
    // (starch_host_register) and reused, so starch_text_read and the
    // bz_stream's input copy run by DMA (fresh malloc'ed text ran at ~6 GB/s)
    struct PoolBuf {
        char* p;
        size_t cap;
        bool free_, reg;
    };
    std::mutex _pmu;
    std::vector<PoolBuf> _pool;
    char* text_pool_get(size_t n)
    {
        std::lock_guard<std::mutex> lk(_pmu);
        size_t best = _pool.size();
        for (size_t i = 0; i < _pool.size(); ++i)
            if (_pool[i].free_ && _pool[i].cap >= n && (best == _pool.size() || _pool[i].cap < _pool[best].cap)) best = i;
        if (best < _pool.size()) {
            _pool[best].free_ = false;
            return _pool[best].p;
        }
        const size_t cap = (std::max<size_t>(n, 1) + (2u << 20) - 1) & ~(size_t)((2u << 20) - 1);
        void* q = NULL;
        if (posix_memalign(&q, 2u << 20, cap)) return NULL;
        PoolBuf b;
        b.p = static_cast<char*>(q);
        b.cap = cap;
        b.free_ = false;
        b.reg = false;
        if (cap >= (4u << 20)) {
            // fresh memory: 2 MiB pages where the kernel has them, first touched
            // by 8 threads (one thread faulting and zeroing ran at ~5 GB/s),
            // then page-locked once for all its reuses
            (void)madvise(q, cap, MADV_HUGEPAGE);
            std::vector<std::thread> th;
            const size_t per = ((cap / 8) + 4095) & ~(size_t)4095;
            for (int t = 0; t < 8; ++t)
                th.push_back(std::thread([=]() {
                    const size_t o = (size_t)t * per;
                    if (o < cap) std::memset(static_cast<char*>(q) + o, 0, std::min(per, cap - o));
                }));
            for (size_t t = 0; t < th.size(); ++t) th[t].join();
            b.reg = starch_host_register(q, cap) == STARCH_OK;
        }
        _pool.push_back(b);
        return b.p;
    }
    // back to the pool (true), or not a pool buffer (false).  The pool keeps at
    // most STARCH_HOOK_POOL_MAX bytes (default 4 GiB) of buffers: a buffer
    // returned while the pool holds more is unregistered and freed (per-base
    // BED runs to GBs of text per chromosome; the buffers in flight are bounded
    // by the hook's job count, the idle ones by this cap)
    static size_t text_pool_max()
    {
        const char* e = std::getenv("STARCH_HOOK_POOL_MAX");
        return e ? (size_t)std::strtoull(e, NULL, 10) : ((size_t)4 << 30);
    }
    bool text_pool_put(char* p)
    {
        std::lock_guard<std::mutex> lk(_pmu);
        size_t total = 0;
        for (size_t i = 0; i < _pool.size(); ++i) total += _pool[i].cap;
        for (size_t i = 0; i < _pool.size(); ++i)
            if (_pool[i].p == p) {
                if (total > text_pool_max()) {
                    if (_pool[i].reg) (void)starch_host_unregister(_pool[i].p);
                    std::free(_pool[i].p);
                    _pool.erase(_pool.begin() + (std::ptrdiff_t)i);
                    return true;            // released: the caller must not free it
                }
                _pool[i].free_ = true;
                return true;
            }
        return false;
    }
    void text_pool_clear()
    {
        std::lock_guard<std::mutex> lk(_pmu);
        for (size_t i = 0; i < _pool.size(); ++i) {
            if (_pool[i].reg) (void)starch_host_unregister(_pool[i].p);
            std::free(_pool[i].p);
        }
        _pool.clear();
    }
};

extern Starch* self;   // hpp:921; the program defines it (cpp:10)

inline void Starch::process_tf_buffer(shared_buffer_t* sb)
{
    if (!sb->tf_buffer) return;
    Starch* s = self;
    if (s && !hook_sync()) {   // the chromosome's text to a worker's bz_stream (it owns the buffer now)
        const char* chr = sb->tf_state && sb->tf_state->current_chr ? sb->tf_state->current_chr : "";
        const std::string name(chr, s->_closing_name_len ? s->_closing_name_len : std::strlen(chr));
        s->_closing_name_len = 0;
        s->hook_submit(name, sb->tf_state ? sb->tf_state->line_count : 0, sb->tf_buffer, sb->tf_buffer_size);
        sb->tf_buffer = NULL;
    } else if (s) {
        if (!s->_bz_stream_ptr || s->_bz_stream_used) {   // one bzip2 stream per chromosome
            s->delete_bz_stream_ptr();
            s->initialize_bz_stream_ptr();
            s->setup_bz_stream_callbacks(s);
        }
        bz_stream* z = s->_bz_stream_ptr;
        const char* chr = sb->tf_state && sb->tf_state->current_chr ? sb->tf_state->current_chr : "";
        s->_closing_chr.assign(chr, s->_closing_name_len ? s->_closing_name_len : std::strlen(chr));
        s->_closing_name_len = 0;
        s->_closing_lines = sb->tf_state ? sb->tf_state->line_count : 0;
        s->_closing_text = sb->tf_buffer_size;
        z->next_in = sb->tf_buffer;
        z->avail_in = (unsigned int)sb->tf_buffer_size;
        std::vector<char> out(1 << 20);
        int rc;
        do {
            z->next_out = &out[0];
            z->avail_out = (unsigned int)out.size();
            rc = BZ2_bzCompress(z, BZ_FINISH);
            const size_t k = out.size() - z->avail_out;
            if (k && s->_out_stream) std::fwrite(&out[0], 1, k, s->_out_stream);
        } while (rc == BZ_FINISH_OK);
        s->_bz_stream_used = true;
        if (rc != BZ_STREAM_END) {
            std::fprintf(stderr, "Error: bzip2 compression failed (%d)\n", rc);
            s->_hook_error = true;
        }
    }
    reset_transformation_state(&sb->tf_state);   // hpp:396-405
    if (!s || !s->text_pool_put(sb->tf_buffer)) std::free(sb->tf_buffer);
    sb->tf_buffer = static_cast<char*>(std::calloc(tf_buffer_initial_length, sizeof(*sb->tf_buffer)));
    if (!sb->tf_buffer) {
        std::fprintf(stderr, "Error: Not enough memory for shared_buffer_t transformation buffer\n");
        std::exit(ENOMEM);
    }
    sb->tf_buffer_capacity = tf_buffer_initial_length;
    sb->tf_buffer_size = 0;
}
}  // namespace starch3

#endif  // STARCH3_AMD_HPP_
