/*
 * include/bzlib.h -- the name the reference includes (include/starch3api.hpp:16,
 * #include "bzlib.h"): with -I<repo>/include, the reference's engine and CLI
 * compile against libstarch_amd.so's patched-libbz2 ABI (starch_bzlib.h)
 * instead of the vendored third-party/bzip2-1.0.6.
 */
#include "starch_bzlib.h"
