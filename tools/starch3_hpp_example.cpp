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
#include <unistd.h>

#include <chrono>
#include <cstring>

#include "../include/starch3_amd.hpp"

starch3::Starch* starch3::self = NULL;   // cpp:10

static double now_s()
{
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv)
{
    const double t0 = now_s();
    const char* tr = std::getenv("STARCH_HOOK_TRACE");
    const bool trace = tr && !std::strcmp(tr, "1");
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
        const double t1 = now_s();
        rc = starch.transform_and_flush_in_stream();
        if (!rc) rc = starch.finish_tf_buffers();
        const double t2 = now_s();
        starch.delete_bz_stream_ptr();
        if (trace)
            std::fprintf(stderr, "example: setup %.1f ms  hook %.1f ms  bz stream delete %.1f ms\n", (t1 - t0) * 1e3,
                         (t2 - t1) * 1e3, (now_s() - t2) * 1e3);
    }
    if (rc) {
        std::fprintf(stderr, "Error: %s (%s)\n", starch_strerror(rc),
                     starch.context() ? starch_last_error(starch.context()) : "");
        return EINVAL;
    }
    const double t3 = now_s();
    starch.delete_out_compression_stream();
    if (trace) std::fprintf(stderr, "example: out stream delete %.1f ms, main %.1f ms\n", (now_s() - t3) * 1e3, (now_s() - t0) * 1e3);
    // The archive is out (and flushed): the bzlib ABI's encoder slots, pinned
    // stages and the HIP runtime go back with the process instead of one by
    // one at static destruction (~0.1-0.2 s); STARCH_HPP_TEARDOWN=1 returns
    // normally.  Same as tools/starch3_cli.cpp.
    const char* td = std::getenv("STARCH_HPP_TEARDOWN");
    if (td && !std::strcmp(td, "1")) return EXIT_SUCCESS;
    if (std::fflush(stdout) != 0 || std::ferror(stdout)) {
        std::fprintf(stderr, "Error: writing the archive failed\n");
        std::fflush(stderr);
        _exit(EIO);
    }
    std::fflush(stderr);
    _exit(EXIT_SUCCESS);
}
