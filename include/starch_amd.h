/*
 * include/starch_amd.h -- C ABI of the MI355X Starch compressor
 * (libstarch_amd.so, built from starch_amd/csrc/ for gfx950).
 *
 * Plain pointers and sizes only; no C++ or torch types cross this boundary.
 * Every entry point returns an int status: STARCH_OK (0) or a negative code
 * (starch_strerror()).  Device pointers are HIP device pointers on the
 * context's device; host pointers are ordinary memory.  One context per
 * thread (a context owns its HIP stream and HBM workspace); contexts on
 * different devices are independent.
 *
 * What each entry point replaces in the reference (alexpreynolds/starch3):
 *   starch_encode_*      the whole starch3 pipeline: produce_line/consume_line
 *                        (include/starch3api.hpp:158-345), update_transformation_
 *                        state (hpp:428-504), per-chromosome flush
 *                        process_tf_buffer (hpp:393-407), and the libbz2
 *                        compressor the reference links for it (hpp:819-888,
 *                        initialize_bz_stream_ptr: BZ2_bzCompressInit(s, 9, .., 30))
 *   starch_transform_*   hpp:158-504 alone (the stderr "Content" text)
 *   starch_bz2_compress_* one BZ2_bzCompressInit + BZ2_bzCompress(BZ_FINISH)
 *                        stream (bz:bzlib.c:148-474), byte-identical
 *   starch_bz2_decompress_* / starch_unstarch_host
 *                        the decompression side: bzip2-1.0.6's
 *                        BZ2_bzDecompress (bz:decompress.c:106-646,
 *                        bz:bzlib.c:621-708) over concatenated streams, and the
 *                        inverse of hpp:428-504 (segment text -> BED lines),
 *                        which the reference does not ship (BEDOPS unstarch)
 *   the archive layout   magic bytes ca 5c ad 1a (hpp:765-769, 907-910), then
 *                        one bzip2 stream per chromosome segment, then a JSON
 *                        index and a 32-byte footer (DESIGN.md "Archive")
 * The patched-libbz2 streaming ABI (BZ2_bzCompress*) lives in
 * include/starch_bzlib.h.
 */
#ifndef STARCH_AMD_H_
#define STARCH_AMD_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define STARCH_OK 0
#define STARCH_ERR_ARG (-2)        /* bad argument (bz: BZ_PARAM_ERROR) */
#define STARCH_ERR_MEM (-3)        /* allocation / capacity (bz: BZ_MEM_ERROR) */
#define STARCH_ERR_STATE (-4)      /* no result yet */
#define STARCH_ERR_DEVICE (-10)    /* HIP runtime error or no MI355X */
#define STARCH_ERR_INTERNAL (-11)
#define STARCH_ERR_DATA (-12)       /* malformed / corrupt compressed data (bz: BZ_DATA_ERROR, BZ_DATA_ERROR_MAGIC) */

typedef struct starch_ctx starch_ctx;

typedef struct {
    int block_size_100k;     /* bzip2 level, 1..9 (reference uses 9, hpp:837) */
    int emit_index;          /* 1: append JSON index + footer after the streams */
    int reference_compat;    /* 1: archive is exactly the reference's stdout (magic only) */
    const char* note;        /* --note text for the index (may be NULL) */
    int base_counts;         /* 1: per-segment base counts (hpp:61-62) in the segments and the index */
    int compression_method;  /* STARCH_METHOD_BZIP2 (0, default) or STARCH_METHOD_GZIP (1): the reference's
                              * compression_method_t (hpp:23-27); gzip there exits ENOSYS (hpp:777-779),
                              * here every segment is one gzip member (fixed-Huffman deflate on the GPU) */
} starch_options;

#define STARCH_METHOD_BZIP2 0
#define STARCH_METHOD_GZIP 1

typedef struct {
    uint64_t line_count;     /* transform_state_t.line_count at flush (hpp:395) */
    uint64_t text_bytes;     /* transformed bytes of this segment */
    uint64_t stream_offset;  /* byte offset of its bzip2 stream in the archive */
    uint64_t stream_bytes;
    uint64_t name_len;       /* chromosome name length (starch_segment_name) */
    uint32_t n_blocks;       /* bzip2 blocks in the stream */
    uint32_t combined_crc;   /* bzip2 combined stream CRC */
    uint64_t unit;           /* input unit the segment came from (archive order = unit order) */
    /* transform_state_t.base_count_unique / _nonunique (hpp:61-62; declared,
     * never computed by the reference), filled when starch_options.base_counts:
     * nonunique = sum of (stop - start) over the segment's lines, unique = sum
     * of max(0, stop - max(start, largest earlier stop)) = size of the union
     * of the intervals for a BED sorted by start; modulo 2^64. */
    int64_t base_count_unique;
    int64_t base_count_nonunique;
} starch_segment;

/* A unit: a byte range of the input whose first line starts a chromosome
 * segment, i.e. its chr token differs from the previous line's (hpp:325-342).
 * Units are encoded independently and their streams concatenate to the
 * whole input's.  init_start / init_stop are the sscanf values current before
 * the unit (a field that fails to parse keeps the previous line's value,
 * hpp:306-307); 0 for the first unit. */
typedef struct {
    uint64_t offset;
    uint64_t length;
    int64_t init_start;
    int64_t init_stop;
} starch_unit;

typedef struct {
    uint64_t input_bytes, n_lines, n_segments, text_bytes, archive_bytes;
    uint64_t n_blocks, rle_bytes, bwt_rounds, periodic_blocks;
    uint64_t bwt_tied;       /* rotations re-sorted by prefix-doubling rounds (ties of the packed key) */
    uint64_t dedup_blocks;   /* blocks that reused a byte-identical block's sort/MTF/tables */
    float ms_transform, ms_rle, ms_bwt, ms_mtf, ms_tables, ms_emit, ms_total;
} starch_stats;

int starch_version(void);                         /* 0x000100 = 0.1.0 */
const char* starch_strerror(int code);
const char* starch_last_error(starch_ctx* ctx);   /* detail text of the last failure */

int starch_create(int device, starch_ctx** out);
void starch_destroy(starch_ctx* ctx);
/* Run the context's work on an external hipStream_t, e.g.
 * torch.cuda.current_stream().cuda_stream.  NULL (0) is the HIP null stream
 * itself: work the caller queued there (an H2D copy, a generator kernel) is
 * ordered before the encode with no host synchronisation.  The context still
 * uses private streams inside a call; they wait for the selected stream on
 * entry and the selected stream waits for them before the call returns. */
int starch_set_stream(starch_ctx* ctx, void* hip_stream);
/* Back to the context's own non-blocking stream (the default after
 * starch_create; not ordered with the null stream). */
int starch_use_own_stream(starch_ctx* ctx);
/* Encoder lanes of this context's device-path encodes (starch_encode_device,
 * starch_encode_host below its pipelined size, starch_encode_units_device):
 * after the one transform, the segments split into `lanes` contiguous runs of
 * about equal text, each encoded (RLE1 .. Huffman tables) by its own encoder
 * on its own stream and host thread, then emitted in order -- the archive
 * bytes do not depend on it.  1: one encoder; 2..8; 0: the default (the
 * STARCH_DEV_LANES environment variable, else 2).  Inputs under 16 MB of text
 * (STARCH_DEV_LANES_MIN) always take one.  Stage times in starch_stats are then
 * wall time during which any lane ran the stage. */
int starch_set_lanes(starch_ctx* ctx, int lanes);
void starch_options_init(starch_options* opt);

/* Whole pipeline.  Input BED bytes already in HBM (d_bed, n bytes).  The
 * archive stays in context-owned HBM until the next call. */
int starch_encode_device(starch_ctx* ctx, const void* d_bed, uint64_t n, const starch_options* opt);
/* Same, from host memory (copied to HBM first; the copy is not in ms_total). */
int starch_encode_host(starch_ctx* ctx, const void* bed, uint64_t n, const starch_options* opt);
/* Host bytes in, archive bytes out into the caller's host buffer out[0, cap)
 * (*out_len = its size; STARCH_ERR_MEM if cap is short, with *out_len = the
 * size needed and out's contents undefined -- finished batches may already
 * have been written into it).  For large pinned
 * inputs every chromosome batch's finished streams go device-to-host while
 * later batches still cross PCIe / encode, so the archive's PCIe trip
 * overlaps the work (pinned out recommended).  Same bytes as
 * starch_encode_host + starch_archive_copy; the archive also stays readable
 * through the accessors below.  (The reference writes its archive to stdout
 * from starch3.cpp's main loop, hpp:758-776.) */
int starch_encode_host_into(starch_ctx* ctx, const void* bed, uint64_t n, const starch_options* opt, void* out,
                            uint64_t cap, uint64_t* out_len);

/* ---- multi-GPU: per-chromosome units sharded across devices ----
 * Plan: split host BED bytes (up to the first 0xFF, hpp:181) into at most
 * max_units units (out must hold max_units entries) by galloping + bisection
 * over line starts -- the chromosome runs of a sorted BED, never a full scan. */
int starch_plan_units(const void* bed, uint64_t n, uint64_t max_units, starch_unit* out, uint64_t* nunits);
/* The same for bytes that continue an input: (init_start, init_stop) are the
 * sscanf values current before byte 0 (hpp:306-307; a batch that starts at a
 * chromosome change whose first lines do not parse keeps them). */
int starch_plan_units_from(const void* bed, uint64_t n, uint64_t max_units, int64_t init_start, int64_t init_stop,
                           starch_unit* out, uint64_t* nunits);
/* Longest-processing-time assignment of units to nshards (by byte length). */
int starch_assign_shards(const starch_unit* units, uint64_t nunits, int nshards, int32_t* shard_of);
/* One shard: encode units resident in HBM (offsets relative to d_base, in
 * input order; unit_ids = their global indices, NULL = 0..nunits-1).  The
 * result is the segments' bzip2 streams back to back (no magic, no index):
 * starch_streams_device/_copy; starch_segments gives each segment's unit and
 * stream_offset within the streams. */
int starch_encode_units_device(starch_ctx* ctx, const void* d_base, const starch_unit* units,
                               const uint64_t* unit_ids, uint64_t nunits, const starch_options* opt);
int starch_streams_device(starch_ctx* ctx, const void** d_ptr, uint64_t* n);
int starch_streams_copy(starch_ctx* ctx, void* dst, uint64_t cap);
/* Archive order of gathered segments (stable by unit) and their byte offsets
 * from base; *end = base + total stream bytes (the index offset). */
int starch_archive_layout(const uint64_t* unit_of, const uint64_t* bytes, uint64_t nseg, uint64_t base,
                          uint64_t* order, uint64_t* offset, uint64_t* end);
/* In-process multi-device encode of host bytes over nctx contexts (one host
 * thread per context; contexts may share a device -- "virtual shards").  The
 * finished streams are gathered into ctxs[0]'s HBM (hipMemcpyPeerAsync over
 * xGMI) and the archive is read through ctxs[0] as after starch_encode_host:
 * byte-identical to the one-context archive. */
int starch_encode_multi_host(starch_ctx* const* ctxs, int nctx, const void* bed, uint64_t n,
                             const starch_options* opt);

/* Same as starch_encode_units_device with the units in host memory (offsets
 * relative to bed): only the listed units are copied to HBM, packed. */
int starch_encode_units_host(starch_ctx* ctx, const void* bed, const starch_unit* units, const uint64_t* unit_ids,
                             uint64_t nunits, const starch_options* opt);

/* ---- the multi-rank gather (one process per GPU) ----------
 * Every rank encodes its units (starch_encode_units_*); starch_gather_archive
 * then collects all ranks' streams into rank 0's archive -- magic + streams in
 * unit order + index, byte-identical to the one-GPU archive -- with RCCL over
 * xGMI: an all-gather of segment counts, an all-gather of the segment records
 * and names, and grouped ncclSend/ncclRecv of the stream bytes straight into
 * their archive offsets.  Rank 0 reads the result through starch_archive_*,
 * starch_segments, starch_segment_name; other ranks see archive size 0.
 * Collective: every rank of the communicator calls it.  librccl is loaded on
 * first use (STARCH_ERR_DEVICE if absent). */
typedef struct starch_comm starch_comm;
#define STARCH_COMM_ID_BYTES 128
/* rank 0: a fresh RCCL unique id (ncclGetUniqueId) to hand to every rank */
int starch_comm_id(void* id);
/* one communicator per process, on the context's device */
int starch_comm_create(int device, int rank, int world, const void* id, starch_comm** out);
/* same, with the id handed out by rank 0 over TCP (rank 0 listens on port;
 * the others connect to host:port, retrying for up to 10 minutes) */
int starch_comm_create_tcp(int device, int rank, int world, const char* host, int port, starch_comm** out);
void starch_comm_destroy(starch_comm* comm);
/* Path of the librccl the gather uses (loaded on first use; "" when RCCL is
 * unavailable).  In a process that already loaded torch-ROCm's RCCL this is
 * that library: both resolve SONAME librccl.so.1 to one object. */
const char* starch_rccl_library(void);
const char* starch_comm_last_error(void);   /* detail of the last failed starch_comm_* / starch_gather_host */
int starch_gather_archive(starch_ctx* ctx, starch_comm* comm, const starch_options* opt);

/* The same gather over caller-supplied primitives on host memory (a test or
 * non-RCCL transport, e.g. torch.distributed gloo): all_gather(send, recv,
 * bytes) fills recv with world x bytes in rank order; send/recv post point-
 * to-point transfers whose order per peer pair matches on both sides and
 * which complete by the next group_end.  segs/names: this rank's segments
 * (stream_offset into streams; unit = global unit index).  Rank 0 receives
 * the archive in *archive (free with starch_free); elsewhere *archive = NULL. */
typedef struct {
    int rank, world;
    void* user;
    int (*all_gather)(void* user, const void* send, void* recv, uint64_t bytes);
    int (*send)(void* user, const void* buf, uint64_t n, int peer);
    int (*recv)(void* user, void* buf, uint64_t n, int peer);
    int (*group_end)(void* user);
} starch_host_comm;
int starch_gather_host(const starch_host_comm* comm, const starch_segment* segs, const char* const* names,
                       const uint64_t* name_lens, uint64_t nseg, const void* streams, const starch_options* opt,
                       void** archive, uint64_t* len);
void starch_free(void* p);
/* Page-lock [p, p + n) of caller memory (its whole pages) for the process,
 * so copies to and from it (starch_encode_host*, starch_transform_host*,
 * starch_text_read, the bzlib ABI's BZ2_bzCompress input) run by DMA at the
 * PCIe rate; a buffer reused across calls pays the pinning once (~0.03 s per
 * GB for memory already touched).  starch_host_unregister(p) with the same p
 * before the memory is freed (a read-only mapping is registered for reads
 * only: copies from it).  The library records the range and DMAs from it
 * only within it; a range overlapping one already registered (or one a
 * running call registered for itself) is refused with STARCH_ERR_ARG.
 * Memory page-locked by other means (hipHostMalloc, a framework's pinned
 * allocator) is used up to the end of its allocation.  No counterpart in the
 * reference (it has no device copies); the hpp's process_tf_buffer pool uses
 * them. */
int starch_host_register(const void* p, uint64_t n);
int starch_host_unregister(const void* p);

/* Streaming ingestion (replaces the reference's line-at-a-time
 * produce_line / consume_line hand-off, include/starch3api.hpp:158-345, and
 * the per-chromosome flush, hpp:393-407).  Feed host BED bytes in pieces of
 * any size (lines may straddle pieces); whenever at least batch_bytes
 * (0 = 256 MiB) are held, everything before the last chromosome change among
 * the complete lines is handed to the session's encoder thread (H2D, GPU
 * encode, D2H) while the caller keeps feeding into the other of two pinned
 * buffers; finished streams become readable with starch_stream_read (the
 * magic is readable at once).  Make no other calls on the context while a
 * session is open.
 * starch_stream_end encodes the rest and appends the index.  The bytes read
 * out, in order, are exactly the archive starch_encode_host gives for the
 * concatenated input.  A 0xFF byte ends the input (hpp:181): later bytes are
 * ignored.  After end, segments/stats describe the whole stream; the archive
 * accessors below report STARCH_ERR_STATE (the bytes went out by read). */
int starch_stream_begin(starch_ctx* ctx, const starch_options* opt, uint64_t batch_bytes);
int starch_stream_feed(starch_ctx* ctx, const void* bed, uint64_t n);
/* Zero-copy feed: a window of >= min_bytes in the session's pinned buffer to
 * read input into directly (e.g. read(2) from a file or pipe), then commit the
 * n bytes written there.  feed() = window + memcpy + commit. */
int starch_stream_window(starch_ctx* ctx, uint64_t min_bytes, void** ptr, uint64_t* cap);
int starch_stream_commit(starch_ctx* ctx, uint64_t n);
int starch_stream_end(starch_ctx* ctx);
int starch_stream_available(starch_ctx* ctx, uint64_t* n);
int starch_stream_read(starch_ctx* ctx, void* dst, uint64_t cap, uint64_t* len);

int starch_archive_size(starch_ctx* ctx, uint64_t* n);
int starch_archive_device(starch_ctx* ctx, const void** d_ptr);
int starch_archive_copy(starch_ctx* ctx, void* dst, uint64_t cap);
int starch_segment_count(starch_ctx* ctx, uint64_t* n);
int starch_segments(starch_ctx* ctx, starch_segment* out, uint64_t cap);
int starch_segment_name(starch_ctx* ctx, uint64_t i, char* buf, uint64_t cap, uint64_t* len);
int starch_get_stats(starch_ctx* ctx, starch_stats* out);

/* Transform stage only: afterwards starch_text_size/starch_text_copy give the
 * concatenated segment texts and starch_segments the per-segment counts. */
int starch_transform_host(starch_ctx* ctx, const void* bed, uint64_t n);
/* The same for bytes that start a segment of a longer input, with the sscanf
 * values current before them (a batch of whole chromosome runs). */
int starch_transform_host_init(starch_ctx* ctx, const void* bed, uint64_t n, int64_t init_start, int64_t init_stop);
int starch_transform_device(starch_ctx* ctx, const void* d_bed, uint64_t n);   /* BED bytes in HBM */
int starch_text_size(starch_ctx* ctx, uint64_t* n);
int starch_text_copy(starch_ctx* ctx, void* dst, uint64_t cap);
/* n bytes of that text from offset off (a segment's, at its stream_offset)
 * into dst: one chromosome's tf_buffer without a copy of the whole text. */
int starch_text_read(starch_ctx* ctx, uint64_t off, void* dst, uint64_t n);

/* One bzip2 stream (BZ_FINISH semantics) of n bytes; result to host. */
int starch_bz2_compress_host(starch_ctx* ctx, const void* in, uint64_t n, int block_size_100k, void* out,
                             uint64_t cap, uint64_t* out_len);
/* Block count and combined CRC of the (first) stream of the last
 * starch_bz2_compress_* call (the index fields of a process_tf_buffer hook). */
int starch_bz2_stream_info(starch_ctx* ctx, uint32_t* n_blocks, uint32_t* combined_crc);

/* Several independent bzip2 streams in one launch sequence (device memory):
 * stream k = d_in[offs[k] .. offs[k]+lens[k]); results packed back to back in
 * d_out (4-byte aligned), out_offs[k]/out_lens[k] filled. */
int starch_bz2_compress_many_device(starch_ctx* ctx, const void* d_in, const uint64_t* offs, const uint64_t* lens,
                                    uint64_t nstreams, int block_size_100k, void* d_out, uint64_t cap,
                                    uint64_t* out_offs, uint64_t* out_lens);

/* Synthetic hg38 BED generator (bench/tests): writes the lines of the given
 * chromosomes (indices into the 24 hg38 chromosomes in sort-bed order) into
 * dst; kind 0 = BED3 (cfg2), 1 = narrowPeak BED6+4 (cfg4), 2 = per-position
 * (cfg5).  total_lines is the whole-genome line count the per-chromosome
 * counts are derived from.  Returns bytes written via *len; pass dst = NULL to
 * size. */
int starch_gen_bed(int kind, uint64_t seed, uint64_t total_lines, const int32_t* chroms, int nchroms, void* dst,
                   uint64_t cap, uint64_t* len);
/* The per-position input (kind 2: "<chr>\t<p>\t<p+1>\n" for p in [first,
 * first + count)) of one chromosome written by the GPU into device memory
 * d_dst (cap bytes) on `stream` (asynchronous); *len = its byte count, which
 * d_dst = NULL returns alone (no GPU needed).  Same bytes as starch_gen_bed
 * kind 2 for that chromosome (cfg5's 73.6 GB input without the host). */
int starch_gen_perpos_device(int chrom, uint64_t first, uint64_t count, void* d_dst, uint64_t cap, uint64_t* len,
                             void* stream);
/* Per-chromosome byte counts of starch_gen_bed's output (sizes[k] for chroms[k]). */
int starch_gen_bed_sizes(int kind, uint64_t seed, uint64_t total_lines, const int32_t* chroms, int nchroms,
                         uint64_t* sizes);

/* Archive index writer: the JSON index + footer for a set of segments
 * (used by the multi-GPU gather to assemble rank 0's archive). */
int starch_build_index(const starch_segment* segs, const char* const* names, const uint64_t* name_lens,
                       uint64_t nseg, uint64_t index_offset, const char* note, int block_size_100k, char* dst,
                       uint64_t cap, uint64_t* len);
/* Same, with the index options taken from opt (note, block size, base counts). */
int starch_build_index_opt(const starch_segment* segs, const char* const* names, const uint64_t* name_lens,
                           uint64_t nseg, uint64_t index_offset, const starch_options* opt, char* dst, uint64_t cap,
                           uint64_t* len);

/* ---- decompression / unstarch -------------------------------
 * Results stay in the context: starch_output_size / _copy / _device. */
typedef struct {
    uint64_t in_beg, in_end;     /* the stream's bytes in the input */
    uint64_t out_off, out_len;   /* its decompressed bytes in the output */
    uint32_t level;              /* blockSize100k of its "BZh" header */
    uint32_t n_blocks;
    uint32_t combined_crc;       /* stored = recomputed (checked) */
} starch_dec_stream;

/* Every bzip2 stream of in[0, n) (concatenated streams, as bzip2 -d), decoded
 * on the GPU with every block CRC and stream CRC checked; STARCH_ERR_DATA on
 * malformed input or a CRC mismatch (bz: BZ_DATA_ERROR).  Randomised blocks
 * (bzip2 < 0.9.5) are refused. */
int starch_bz2_decompress_host(starch_ctx* ctx, const void* in, uint64_t n);
int starch_bz2_decompress_device(starch_ctx* ctx, const void* d_in, uint64_t n);
int starch_bz2_stream_count(starch_ctx* ctx, uint64_t* n);
int starch_bz2_streams(starch_ctx* ctx, starch_dec_stream* out, uint64_t cap);
/* Inverse transform of one segment's text: "chr\tstart\tstop[\trem]\n" lines.
 * Exact for canonical BED (decimal coordinates, stop >= start); a negative
 * p-value (whose newline the forward transform drops, hpp:440,452) or a
 * malformed line gives STARCH_ERR_DATA. */
int starch_untransform_host(starch_ctx* ctx, const void* text, uint64_t n, const char* chr, uint64_t chr_len);
/* A whole archive of this library (magic, streams, index, footer) back to BED:
 * every stream decoded and inverse-transformed on the GPU, in index order. */
int starch_unstarch_host(starch_ctx* ctx, const void* archive, uint64_t n);
int starch_output_size(starch_ctx* ctx, uint64_t* n);
int starch_output_copy(starch_ctx* ctx, void* dst, uint64_t cap);
int starch_output_device(starch_ctx* ctx, const void** d_ptr);

#ifdef __cplusplus
}
#endif
#endif
