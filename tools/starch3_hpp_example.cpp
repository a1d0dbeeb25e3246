// tools/starch3_hpp_example.cpp -- the reference's main() (src/starch3.cpp:14-70)
// written against include/starch3_amd.hpp: same call order on starch3::Starch,
// with the four pthreads replaced by compress_in_stream().  With --hook the
// archive is produced through the reference's per-chromosome hand-off
// instead: the GPU transform gives each chromosome's text in `buffer`, and
// the static process_tf_buffer (hpp:393-407) feeds it to the bz_stream set up
// by initialize_bz_stream_ptr / setup_bz_stream_callbacks (hpp:819-862, the
// GPU-backed patched-libbz2 ABI), whose block_close_functor records the index
// entry; finish_tf_buffers writes the index.  Both must give the same bytes as
// the starch3 CLI.
#include <cstring>

#include "../include/starch3_amd.hpp"

starch3::Starch* starch3::self = NULL;   // cpp:10

int main(int argc, char** argv)
{
    starch3::Starch starch;
    starch3::self = &starch;
    // --hook: the per-chromosome hand-off; --vdev N: N virtual devices (all on
    // GPU 0: the multi-device batch path of compress_in_stream);
    // --reference-compat: stdout is the reference's (the magic bytes only)
    bool hook = false;
    int a = 1;
    for (; a < argc && argv[a][0] == '-' && argv[a][1] == '-'; ++a) {
        if (std::strcmp(argv[a], "--hook") == 0) hook = true;
        else if (std::strcmp(argv[a], "--reference-compat") == 0) starch.set_reference_compat(true);
        else if (std::strcmp(argv[a], "--vdev") == 0 && a + 1 < argc) starch.set_devices(std::vector<int>(std::atoi(argv[++a]), 0));
    }
    if (a < argc) starch.set_input_fn(argv[a]);
    starch.set_compression_method(starch3::Starch::k_bzip2);
    starch.test_stdin_availability();
    starch.initialize_in_stream();
    starch.initialize_out_stream();
    starch.initialize_out_compression_stream();
    int rc;
    if (!hook) {
        rc = starch.compress_in_stream();
    } else {
        starch.initialize_bz_stream_ptr();          // hpp:773-776
        starch.setup_bz_stream_callbacks(&starch);
        rc = starch.transform_and_flush_in_stream();
        if (!rc) rc = starch.finish_tf_buffers();
        starch.delete_bz_stream_ptr();
    }
    if (rc) {
        std::fprintf(stderr, "Error: %s\n", starch_strerror(rc));
        return EINVAL;
    }
    starch.delete_out_compression_stream();
    return EXIT_SUCCESS;
}
