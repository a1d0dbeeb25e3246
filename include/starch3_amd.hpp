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
 * stream.  The per-chromosome hand-off process_tf_buffer (hpp:393-407) keeps
 * its role as a hook: given one chromosome's transformed text it compresses
 * it on the GPU into that chromosome's stream; finish_tf_buffers() then writes
 * the collected streams and the index.
 *
 * Link with -lstarch_amd.  Compiles as C++11.
 */
#ifndef STARCH3_AMD_HPP_
#define STARCH3_AMD_HPP_

#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <cinttypes>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "starch_amd.h"

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

    Starch()
        : _in_stream(NULL), _out_stream(NULL), _block_size(9), _reference_compat(false), _emit_index(true),
          _base_counts(false)
    {
        set_note(std::string());
        set_compression_method(k_compression_method_undefined);   // hpp:912-916
        initialize_header_magic_bytes();
        _devices.push_back(0);
    }
    ~Starch() { delete_out_compression_stream(); }

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
            open_devices();
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
    starch_ctx* context(void) { return _ctx.empty() ? NULL : _ctx[0]; }

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
    // initialize_out_stream wrote) to the out stream.
    int compress_in_stream(void)
    {
        std::vector<unsigned char> in, arch;
        std::vector<unsigned char> buf(1 << 24);
        size_t k;
        while ((k = std::fread(&buf[0], 1, buf.size(), _in_stream)) > 0) in.insert(in.end(), buf.begin(), buf.begin() + k);
        int rc = compress(in.empty() ? NULL : &in[0], in.size(), &arch);
        if (rc) return rc;
        if (arch.size() > 4) std::fwrite(&arch[4], 1, arch.size() - 4, _out_stream);
        std::fflush(_out_stream);
        return STARCH_OK;
    }

    // The per-chromosome hand-off (hpp:393-407): one chromosome's transformed
    // text -> its bzip2 -N stream, compressed on the GPU and kept for
    // finish_tf_buffers().
    int process_tf_buffer(const std::string& chr, int64_t line_count, const char* tf_buffer, size_t tf_buffer_size)
    {
        int rc = open_devices();
        if (rc) return rc;
        std::vector<unsigned char> st(tf_buffer_size + tf_buffer_size / 50 + 4096);
        uint64_t len = 0;
        rc = starch_bz2_compress_host(_ctx[0], tf_buffer, tf_buffer_size, _block_size, &st[0], st.size(), &len);
        if (rc) return rc;
        st.resize(len);
        starch_segment s;
        std::memset(&s, 0, sizeof(s));
        s.line_count = (uint64_t)line_count;
        s.text_bytes = tf_buffer_size;
        s.stream_bytes = len;
        s.name_len = chr.size();
        s.unit = _pending.size();
        uint32_t nb = 0, crc = 0;
        if ((rc = starch_bz2_stream_info(_ctx[0], &nb, &crc))) return rc;
        s.n_blocks = nb;
        s.combined_crc = crc;
        _pending.push_back(Pending(chr, s, st));
        return STARCH_OK;
    }

    // Write the streams collected by process_tf_buffer, then the index, to the
    // out stream (after the magic initialize_out_stream wrote).
    int finish_tf_buffers(void)
    {
        uint64_t off = 4;
        std::vector<starch_segment> segs;
        std::vector<const char*> names;
        std::vector<uint64_t> lens;
        for (size_t i = 0; i < _pending.size(); ++i) {
            _pending[i].seg.stream_offset = off;
            off += _pending[i].stream.size();
            if (!_pending[i].stream.empty())
                std::fwrite(&_pending[i].stream[0], 1, _pending[i].stream.size(), _out_stream);
            segs.push_back(_pending[i].seg);
            names.push_back(_pending[i].chr.data());
            lens.push_back(_pending[i].chr.size());
        }
        if (_emit_index) {
            uint64_t n = 0;
            int rc = starch_build_index(segs.empty() ? NULL : &segs[0], names.empty() ? NULL : &names[0],
                                        lens.empty() ? NULL : &lens[0], segs.size(), off, _note.c_str(),
                                        _block_size, NULL, 0, &n);
            if (rc) return rc;
            std::vector<char> idx(n);
            rc = starch_build_index(segs.empty() ? NULL : &segs[0], names.empty() ? NULL : &names[0],
                                    lens.empty() ? NULL : &lens[0], segs.size(), off, _note.c_str(), _block_size,
                                    &idx[0], n, &n);
            if (rc) return rc;
            std::fwrite(&idx[0], 1, n, _out_stream);
        }
        _pending.clear();
        std::fflush(_out_stream);
        return STARCH_OK;
    }

private:
    struct Pending {
        std::string chr;
        starch_segment seg;
        std::vector<unsigned char> stream;
        Pending(const std::string& c, const starch_segment& s, const std::vector<unsigned char>& st)
            : chr(c), seg(s), stream(st) {}
    };

    int open_devices(void)
    {
        if (!_ctx.empty()) return STARCH_OK;
        for (size_t i = 0; i < _devices.size(); ++i) {
            starch_ctx* c = NULL;
            int rc = starch_create(_devices[i], &c);
            if (rc) {
                delete_out_compression_stream();
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
    std::vector<Pending> _pending;
};
}  // namespace starch3

#endif  // STARCH3_AMD_HPP_
