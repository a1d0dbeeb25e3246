// tools/starch3_hpp_example.cpp -- the reference's main() (src/starch3.cpp:14-70)
// written against include/starch3_amd.hpp: same call order on starch3::Starch,
// with the four pthreads replaced by compress_in_stream().  With --hook the
// archive is produced through the per-chromosome hand-off instead: the GPU
// transform gives each chromosome's text, process_tf_buffer (hpp:393-407)
// compresses it, finish_tf_buffers writes streams + index.  Both must give the
// same bytes as the starch3 CLI.
#include <cstring>

#include "../include/starch3_amd.hpp"

int main(int argc, char** argv)
{
    starch3::Starch starch;
    bool hook = argc > 1 && std::strcmp(argv[1], "--hook") == 0;
    if (argc > 1 + (hook ? 1 : 0)) starch.set_input_fn(argv[1 + (hook ? 1 : 0)]);
    starch.set_compression_method(starch3::Starch::k_bzip2);
    starch.test_stdin_availability();
    starch.initialize_in_stream();
    starch.initialize_out_stream();
    starch.initialize_out_compression_stream();
    int rc;
    if (!hook) {
        rc = starch.compress_in_stream();
    } else {
        std::vector<unsigned char> in, buf(1 << 20);
        size_t k;
        while ((k = std::fread(&buf[0], 1, buf.size(), starch.get_in_stream())) > 0)
            in.insert(in.end(), buf.begin(), buf.begin() + k);
        starch_ctx* c = starch.context();
        rc = starch_transform_host(c, in.empty() ? NULL : &in[0], in.size());
        uint64_t nseg = 0, tb = 0;
        if (!rc) rc = starch_segment_count(c, &nseg);
        if (!rc) rc = starch_text_size(c, &tb);
        std::vector<char> text(tb + 1);
        std::vector<starch_segment> segs(nseg + 1);
        if (!rc) rc = starch_text_copy(c, &text[0], tb);
        if (!rc) rc = starch_segments(c, &segs[0], nseg);
        for (uint64_t s = 0; s < nseg && !rc; ++s) {
            std::string name(segs[s].name_len, '\0');
            uint64_t len = 0;
            rc = starch_segment_name(c, s, name.empty() ? NULL : &name[0], name.size(), &len);
            if (!rc)   // transform-only results carry the text offset in stream_offset
                rc = starch.process_tf_buffer(name, (int64_t)segs[s].line_count, &text[segs[s].stream_offset],
                                              segs[s].text_bytes);
        }
        if (!rc) rc = starch.finish_tf_buffers();
    }
    if (rc) {
        std::fprintf(stderr, "Error: %s\n", starch_strerror(rc));
        return EINVAL;
    }
    starch.delete_out_compression_stream();
    return EXIT_SUCCESS;
}
