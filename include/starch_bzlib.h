/*
 * include/starch_bzlib.h -- drop-in replacement for the compression half of
 * the PATCHED libbz2 the reference builds against
 * (third-party/bzip2-1.0.6.tar.gz: bzlib.h:48-69 layout, bzlib.h:103-117
 * prototypes), implemented on MI355X by libstarch_amd.so.
 *
 * Code written against the reference's include/starch3api.hpp (which calls
 * BZ2_bzCompressInit(s, 9, 0|4, 30) at hpp:835/837, installs handler and
 * block_close_functor at hpp:857-862 and calls BZ2_bzCompressEnd at hpp:868)
 * compiles unchanged against this header and links with -lstarch_amd.
 *
 * Differences from the patched library (documented in INTEGRATION.md):
 *  - a NULL block_close_functor is allowed (the patched library calls it
 *    unconditionally at BZ_STREAM_END, bz:bzlib.c:470, and crashes);
 *  - the compressed bytes are produced on the GPU.  The state machine is the
 *    library's step for step (bz:bzlib.c:369-471): BZ_RUN buffers input with
 *    libbz2's RLE1 bookkeeping and emits a block as soon as nblockMAX bytes
 *    are held (the pending run carried into the next block), BZ_FLUSH makes
 *    every whole byte so far readable (BZ_FLUSH_OK while it does not fit
 *    avail_out, then BZ_RUN_OK), BZ_FINISH ends the stream.  The bytes, the
 *    return codes and total_in / total_out after EVERY call (BZ_RUN included)
 *    are identical to the patched library for the same call sequence;
 *  - a GPU failure inside BZ2_bzCompress returns BZ_CONFIG_ERROR and ENDS the
 *    stream: the input of that call may already be consumed (next_in /
 *    avail_in / total_in advanced), every later BZ2_bzCompress returns
 *    BZ_SEQUENCE_ERROR, and BZ2_bzCompressEnd is the only valid call left.
 */
#ifndef STARCH_BZLIB_H_
#define STARCH_BZLIB_H_

#ifdef __cplusplus
extern "C" {
#endif

#define BZ_RUN 0
#define BZ_FLUSH 1
#define BZ_FINISH 2

#define BZ_OK 0
#define BZ_RUN_OK 1
#define BZ_FLUSH_OK 2
#define BZ_FINISH_OK 3
#define BZ_STREAM_END 4
#define BZ_SEQUENCE_ERROR (-1)
#define BZ_PARAM_ERROR (-2)
#define BZ_MEM_ERROR (-3)
#define BZ_DATA_ERROR (-4)
#define BZ_DATA_ERROR_MAGIC (-5)
#define BZ_IO_ERROR (-6)
#define BZ_UNEXPECTED_EOF (-7)
#define BZ_OUTBUFF_FULL (-8)
#define BZ_CONFIG_ERROR (-9)

typedef struct {
    char* next_in;
    unsigned int avail_in;
    unsigned int total_in_lo32;
    unsigned int total_in_hi32;

    char* next_out;
    unsigned int avail_out;
    unsigned int total_out_lo32;
    unsigned int total_out_hi32;

    void* state;

    void* (*bzalloc)(void*, int, int);
    void (*bzfree)(void*, void*);
    void* opaque;

    void* handler;                      /* patched fields (bz:bzlib.h:66-67) */
    void (*block_close_functor)(void*);
} bz_stream;

int BZ2_bzCompressInit(bz_stream* strm, int blockSize100k, int verbosity, int workFactor);
int BZ2_bzCompress(bz_stream* strm, int action);
int BZ2_bzCompressEnd(bz_stream* strm);
const char* BZ2_bzlibVersion(void);

/* Not in libbz2: blocks written so far and their combined CRC (the value the
 * stream trailer carries; bz:compress.c:606-608) -- what a block-close
 * callback needs for the archive index. */
int starch_bzstream_info(bz_stream* strm, unsigned int* n_blocks, unsigned int* combined_crc);

#ifdef __cplusplus
}
#endif
#endif
