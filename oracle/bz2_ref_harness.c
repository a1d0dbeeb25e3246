/*
 * oracle/bz2_ref_harness.c -- TEST INFRASTRUCTURE ONLY (not product code).
 *
 * A small driver for the reference's own vendored, patched libbz2 1.0.6
 * (third-party/bzip2-1.0.6.tar.gz), compiled together with it by
 * oracle/build_ref.sh into oracle/_ref/libbz2ref.so.  It mirrors how the
 * reference would drive the library (hpp:819-888): BZ2_bzCompressInit(s, bs,
 * 0, wf), then install a block-close functor (the patched library calls it
 * unconditionally at BZ_STREAM_END, bz:bzlib.c:470), then BZ2_bzCompress.
 * Used by tests (golden streams, bzlib-ABI call-sequence parity) and by
 * bench.py's cpu_baseline leg (kind "reference").
 */
#include <stdint.h>
#include <stddef.h>
#include <string.h>
#include "bzlib.h"

static void ref_noop_functor(void* h) { (void)h; }

/* Single BZ_FINISH call over the whole input. */
int ref_bz2_compress(const uint8_t* in, size_t n, int bs100k, int wf,
                     uint8_t* out, size_t cap, size_t* out_len)
{
    bz_stream s;
    memset(&s, 0, sizeof(s));
    int rc = BZ2_bzCompressInit(&s, bs100k, 0, wf);
    if (rc != BZ_OK) return rc;
    s.block_close_functor = ref_noop_functor;
    s.handler = NULL;
    s.next_in = (char*)in;
    s.avail_in = (unsigned int)n;
    s.next_out = (char*)out;
    s.avail_out = (unsigned int)cap;
    do { rc = BZ2_bzCompress(&s, BZ_FINISH); } while (rc == BZ_FINISH_OK && s.avail_out > 0);
    *out_len = cap - s.avail_out;
    BZ2_bzCompressEnd(&s);
    return rc == BZ_STREAM_END ? 0 : (rc < 0 ? rc : -100);
}

/*
 * Scripted call sequence: ops[2k] = action (0 RUN, 1 FLUSH, 2 FINISH),
 * ops[2k+1] = number of fresh input bytes supplied with that call.  Each op
 * is repeated until it completes (RUN: input consumed; FLUSH: BZ_RUN_OK;
 * FINISH: BZ_STREAM_END).  out_chunk bounds avail_out per call so the
 * FINISH_OK/FLUSH_OK draining loops are exercised.  rcs[k] gets the last
 * return code of op k.
 */
int ref_bz2_script_trace(const uint8_t* in, const int32_t* ops, int nops, int bs100k, int wf,
                         size_t out_chunk, uint8_t* out, size_t cap, size_t* out_len, int32_t* rcs,
                         uint64_t* produced_after);

int ref_bz2_script(const uint8_t* in, const int32_t* ops, int nops, int bs100k, int wf,
                   size_t out_chunk, uint8_t* out, size_t cap, size_t* out_len, int32_t* rcs)
{
    return ref_bz2_script_trace(in, ops, nops, bs100k, wf, out_chunk, out, cap, out_len, rcs, NULL);
}

/* Same, and produced_after[k] = total output bytes once op k completed (the
 * library's total_out after each call: what BZ_FLUSH makes readable). */
int ref_bz2_script_trace(const uint8_t* in, const int32_t* ops, int nops, int bs100k, int wf,
                         size_t out_chunk, uint8_t* out, size_t cap, size_t* out_len, int32_t* rcs,
                         uint64_t* produced_after)
{
    bz_stream s;
    memset(&s, 0, sizeof(s));
    int rc = BZ2_bzCompressInit(&s, bs100k, 0, wf);
    if (rc != BZ_OK) return rc;
    s.block_close_functor = ref_noop_functor;
    size_t used = 0, produced = 0;
    for (int k = 0; k < nops; ++k) {
        int act = ops[2 * k];
        s.next_in = (char*)(in + used);
        s.avail_in = (unsigned int)ops[2 * k + 1];
        used += (size_t)ops[2 * k + 1];
        for (;;) {
            size_t room = cap - produced;
            if (out_chunk && room > out_chunk) room = out_chunk;
            s.next_out = (char*)(out + produced);
            s.avail_out = (unsigned int)room;
            rc = BZ2_bzCompress(&s, act);
            produced += room - s.avail_out;
            rcs[k] = rc;
            if (rc < 0) { *out_len = produced; BZ2_bzCompressEnd(&s); return rc; }
            if (act == BZ_RUN && s.avail_in == 0) break;
            if (act == BZ_FLUSH && rc == BZ_RUN_OK) break;
            if (act == BZ_FINISH && rc == BZ_STREAM_END) break;
            if (produced >= cap) { *out_len = produced; BZ2_bzCompressEnd(&s); return -101; }
        }
        if (produced_after) produced_after[k] = produced;
    }
    *out_len = produced;
    BZ2_bzCompressEnd(&s);
    return 0;
}

const char* ref_bz2_version(void) { return BZ2_bzlibVersion(); }
