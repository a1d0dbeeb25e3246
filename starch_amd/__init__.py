"""starch_amd -- host-side (Python) mirror of the Starch operator interface.

The compute lives in ``starch_amd/_build/libstarch_amd.so`` (HIP kernels for
gfx950 behind the C ABI of ``include/starch_amd.h``).  This module only loads
that library with ctypes and marshals arguments; there is no Python or CPU
fallback: if the library or an MI355X is missing, every call raises.

Names follow the reference (alexpreynolds/starch3): ``Starch`` mirrors
``starch3::Starch`` (include/starch3api.hpp:21-584) -- ``set_note``,
``set_compression_method``, ``initialize_header_magic_bytes`` -- and
``Starch.compress(bed)`` is the whole produce_line -> consume_line ->
update_transformation_state -> process_tf_buffer -> bzip2 path.
"""
import ctypes
import json
import os

__all__ = ["Starch", "StarchError", "load", "gen_bed", "build_index", "parse_archive", "plan_units", "assign_shards",
           "archive_layout", "compress_multi", "Unit", "Segment", "Comm", "gather_host", "MAGIC", "HG38", "HG38_LEN"]

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("STARCH_AMD_LIB") or os.path.join(_HERE, "_build", "libstarch_amd.so")
MAGIC = b"\xca\x5c\xad\x1a"          # hpp:907-910
HG38 = [  # sort-bed order; index = chromosome id used by gen_bed
    "chr1", "chr10", "chr11", "chr12", "chr13", "chr14", "chr15", "chr16", "chr17", "chr18", "chr19",
    "chr2", "chr20", "chr21", "chr22", "chr3", "chr4", "chr5", "chr6", "chr7", "chr8", "chr9", "chrX", "chrY",
]
HG38_LEN = [  # hg38 lengths, same order (per-position input has one line per base)
    248956422, 133797422, 135086622, 133275309, 114364328, 107043718, 101991189, 90338345, 83257441, 80373285,
    58617616, 242193529, 64444167, 46709983, 50818468, 198295559, 190214555, 181538259, 170805979, 159345973,
    145138636, 138394717, 156040895, 57227415,
]

# compression methods (hpp:23-27)
K_BZIP2, K_GZIP, K_UNDEFINED = 0, 1, 2


class StarchError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("starch error %d: %s" % (code, msg))
        self.code = code


class Segment(ctypes.Structure):
    _fields_ = [("line_count", ctypes.c_uint64), ("text_bytes", ctypes.c_uint64),
                ("stream_offset", ctypes.c_uint64), ("stream_bytes", ctypes.c_uint64),
                ("name_len", ctypes.c_uint64), ("n_blocks", ctypes.c_uint32),
                ("combined_crc", ctypes.c_uint32), ("unit", ctypes.c_uint64),
                ("base_count_unique", ctypes.c_int64), ("base_count_nonunique", ctypes.c_int64)]


class Unit(ctypes.Structure):
    """starch_unit: an input byte range starting a chromosome segment, with the
    sscanf values current before it (hpp:306-307, 325-342)."""
    _fields_ = [("offset", ctypes.c_uint64), ("length", ctypes.c_uint64),
                ("init_start", ctypes.c_int64), ("init_stop", ctypes.c_int64)]


class Options(ctypes.Structure):
    _fields_ = [("block_size_100k", ctypes.c_int), ("emit_index", ctypes.c_int),
                ("reference_compat", ctypes.c_int), ("note", ctypes.c_char_p), ("base_counts", ctypes.c_int),
                ("compression_method", ctypes.c_int)]


class Stats(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint64) for n in ("input_bytes", "n_lines", "n_segments", "text_bytes",
                                               "archive_bytes", "n_blocks", "rle_bytes", "bwt_rounds",
                                               "periodic_blocks", "bwt_tied", "dedup_blocks")] + \
               [(n, ctypes.c_float) for n in ("ms_transform", "ms_rle", "ms_bwt", "ms_mtf", "ms_tables",
                                              "ms_emit", "ms_total")]


_lib = None

# starch_host_comm (include/starch_amd.h): the gather's four primitives
_AG_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64)
_SEND_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int)
_RECV_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int)
_END_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p)


class HostComm(ctypes.Structure):
    _fields_ = [("rank", ctypes.c_int), ("world", ctypes.c_int), ("user", ctypes.c_void_p),
                ("all_gather", _AG_FN), ("send", _SEND_FN), ("recv", _RECV_FN), ("group_end", _END_FN)]


class DecStream(ctypes.Structure):
    """starch_dec_stream: one decoded bzip2 stream."""
    _fields_ = [("in_beg", ctypes.c_uint64), ("in_end", ctypes.c_uint64), ("out_off", ctypes.c_uint64),
                ("out_len", ctypes.c_uint64), ("level", ctypes.c_uint32), ("n_blocks", ctypes.c_uint32),
                ("combined_crc", ctypes.c_uint32)]


def load():
    """Load libstarch_amd.so (raises if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise StarchError(-10, "native library missing: %s (run __graft_entry__.build())" % LIB_PATH)
    # One HIP runtime per process: PyTorch-ROCm ships its own libamdhip64
    # (same soname as /opt/rocm's).  Loading torch first makes this library
    # bind to torch's copy, so the two share devices, streams and memory;
    # loading ours first and torch later leaves the process with a runtime
    # torch's device setup then breaks for this library (seen as
    # hipErrorNoDevice from starch_create).
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(LIB_PATH)
    vp, u64, pu64 = ctypes.c_void_p, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)
    sig = {
        "starch_version": ([], ctypes.c_int),
        "starch_strerror": ([ctypes.c_int], ctypes.c_char_p),
        "starch_last_error": ([vp], ctypes.c_char_p),
        "starch_create": ([ctypes.c_int, ctypes.POINTER(vp)], ctypes.c_int),
        "starch_destroy": ([vp], None),
        "starch_set_stream": ([vp, vp], ctypes.c_int),
        "starch_use_own_stream": ([vp], ctypes.c_int),
        "starch_set_lanes": ([vp, ctypes.c_int], ctypes.c_int),
        "starch_options_init": ([ctypes.POINTER(Options)], None),
        "starch_encode_device": ([vp, vp, u64, ctypes.POINTER(Options)], ctypes.c_int),
        "starch_encode_host": ([vp, ctypes.c_char_p, u64, ctypes.POINTER(Options)], ctypes.c_int),
        "starch_encode_host_into": ([vp, vp, u64, ctypes.POINTER(Options), vp, u64, ctypes.POINTER(u64)],
                                    ctypes.c_int),
        "starch_archive_size": ([vp, pu64], ctypes.c_int),
        "starch_archive_device": ([vp, ctypes.POINTER(vp)], ctypes.c_int),
        "starch_archive_copy": ([vp, vp, u64], ctypes.c_int),
        "starch_segment_count": ([vp, pu64], ctypes.c_int),
        "starch_segments": ([vp, ctypes.POINTER(Segment), u64], ctypes.c_int),
        "starch_segment_name": ([vp, u64, vp, u64, pu64], ctypes.c_int),
        "starch_get_stats": ([vp, ctypes.POINTER(Stats)], ctypes.c_int),
        "starch_transform_host": ([vp, ctypes.c_char_p, u64], ctypes.c_int),
        "starch_transform_device": ([vp, vp, u64], ctypes.c_int),
        "starch_text_size": ([vp, pu64], ctypes.c_int),
        "starch_text_copy": ([vp, vp, u64], ctypes.c_int),
        "starch_text_read": ([vp, u64, vp, u64], ctypes.c_int),
        "starch_bz2_compress_host": ([vp, ctypes.c_char_p, u64, ctypes.c_int, vp, u64, pu64], ctypes.c_int),
        "starch_bz2_compress_many_device": ([vp, vp, pu64, pu64, u64, ctypes.c_int, vp, u64, pu64, pu64],
                                            ctypes.c_int),
        "starch_gen_bed": ([ctypes.c_int, u64, u64, ctypes.POINTER(ctypes.c_int32), ctypes.c_int, vp, u64, pu64],
                           ctypes.c_int),
        "starch_gen_perpos_device": ([ctypes.c_int, u64, u64, vp, u64, pu64, vp], ctypes.c_int),
        "starch_build_index": ([ctypes.POINTER(Segment), ctypes.POINTER(ctypes.c_char_p), pu64, u64, u64,
                                ctypes.c_char_p, ctypes.c_int, vp, u64, pu64], ctypes.c_int),
        "starch_build_index_opt": ([ctypes.POINTER(Segment), ctypes.POINTER(ctypes.c_char_p), pu64, u64, u64,
                                    ctypes.POINTER(Options), vp, u64, pu64], ctypes.c_int),
        "starch_gen_bed_sizes": ([ctypes.c_int, u64, u64, ctypes.POINTER(ctypes.c_int32), ctypes.c_int, pu64],
                                 ctypes.c_int),
        "starch_plan_units": ([ctypes.c_char_p, u64, u64, ctypes.POINTER(Unit), pu64], ctypes.c_int),
        "starch_assign_shards": ([ctypes.POINTER(Unit), u64, ctypes.c_int, ctypes.POINTER(ctypes.c_int32)],
                                 ctypes.c_int),
        "starch_encode_units_device": ([vp, vp, ctypes.POINTER(Unit), pu64, u64, ctypes.POINTER(Options)],
                                       ctypes.c_int),
        "starch_streams_device": ([vp, ctypes.POINTER(vp), pu64], ctypes.c_int),
        "starch_streams_copy": ([vp, vp, u64], ctypes.c_int),
        "starch_archive_layout": ([pu64, pu64, u64, u64, pu64, pu64, pu64], ctypes.c_int),
        "starch_encode_multi_host": ([ctypes.POINTER(vp), ctypes.c_int, ctypes.c_char_p, u64,
                                      ctypes.POINTER(Options)], ctypes.c_int),
        "starch_stream_begin": ([vp, ctypes.POINTER(Options), u64], ctypes.c_int),
        "starch_stream_feed": ([vp, vp, u64], ctypes.c_int),
        "starch_stream_window": ([vp, u64, ctypes.POINTER(vp), pu64], ctypes.c_int),
        "starch_stream_commit": ([vp, u64], ctypes.c_int),
        "starch_stream_end": ([vp], ctypes.c_int),
        "starch_stream_available": ([vp, pu64], ctypes.c_int),
        "starch_stream_read": ([vp, vp, u64, pu64], ctypes.c_int),
        "starch_bz2_decompress_host": ([vp, ctypes.c_char_p, u64], ctypes.c_int),
        "starch_bz2_decompress_device": ([vp, vp, u64], ctypes.c_int),
        "starch_bz2_stream_count": ([vp, pu64], ctypes.c_int),
        "starch_bz2_streams": ([vp, ctypes.POINTER(DecStream), u64], ctypes.c_int),
        "starch_untransform_host": ([vp, ctypes.c_char_p, u64, ctypes.c_char_p, u64], ctypes.c_int),
        "starch_unstarch_host": ([vp, ctypes.c_char_p, u64], ctypes.c_int),
        "starch_output_size": ([vp, pu64], ctypes.c_int),
        "starch_output_copy": ([vp, vp, u64], ctypes.c_int),
        "starch_output_device": ([vp, ctypes.POINTER(vp)], ctypes.c_int),
        "starch_encode_units_host": ([vp, vp, ctypes.POINTER(Unit), pu64, u64, ctypes.POINTER(Options)],
                                     ctypes.c_int),
        "starch_comm_id": ([vp], ctypes.c_int),
        "starch_comm_create": ([ctypes.c_int, ctypes.c_int, ctypes.c_int, vp, ctypes.POINTER(vp)], ctypes.c_int),
        "starch_comm_create_tcp": ([ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_char_p, ctypes.c_int,
                                    ctypes.POINTER(vp)], ctypes.c_int),
        "starch_comm_destroy": ([vp], None),
        "starch_rccl_library": ([], ctypes.c_char_p),
        "starch_comm_last_error": ([], ctypes.c_char_p),
        "starch_gather_archive": ([vp, vp, ctypes.POINTER(Options)], ctypes.c_int),
        "starch_gather_host": ([ctypes.POINTER(HostComm), ctypes.POINTER(Segment), ctypes.POINTER(ctypes.c_char_p),
                                pu64, u64, vp, ctypes.POINTER(Options), ctypes.POINTER(vp), pu64], ctypes.c_int),
        "starch_free": ([vp], None),
    }
    for name, (args, res) in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    _lib = L
    return L


def _check(rc, ctx=None):
    if rc != 0:
        L = load()
        detail = L.starch_last_error(ctx).decode(errors="replace") if ctx else ""
        raise StarchError(rc, (L.starch_strerror(rc) or b"").decode() + (": " + detail if detail else ""))


class Starch:
    """One compression context on one MI355X (``starch3::Starch``, hpp:21-584)."""

    client_name = "starch3"
    client_version = "0.1"

    def __init__(self, device=0):
        L = load()
        h = ctypes.c_void_p()
        _check(L.starch_create(device, ctypes.byref(h)))
        self._h = h
        self._L = L
        self._note = ""
        self._method = K_BZIP2
        self.block_size_100k = 9
        self.base_counts = False       # per-segment base counts in segments() and the index (hpp:61-62)
        self._magic = MAGIC

    def close(self):
        if getattr(self, "_h", None):
            self._L.starch_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- starch3::Starch configuration surface -------------------------------
    def set_note(self, s):                      # hpp:807-809
        self._note = s

    def get_note(self):
        return self._note

    def set_compression_method(self, m):        # hpp:815-817
        if m not in (K_BZIP2, K_GZIP, K_UNDEFINED):
            raise StarchError(-2, "unknown compression method")
        self._method = m

    def get_compression_method(self):
        return self._method

    def initialize_header_magic_bytes(self):    # hpp:907-910
        self._magic = MAGIC
        return self._magic

    def set_stream(self, hip_stream_ptr):
        """Run on an external HIP stream; 0 is the HIP null stream (torch's default stream)."""
        _check(self._L.starch_set_stream(self._h, ctypes.c_void_p(hip_stream_ptr)), self._h)

    def set_lanes(self, lanes):
        """Encoder lanes of the device-path encodes (1..8; 0: the default, STARCH_DEV_LANES or 2)."""
        _check(self._L.starch_set_lanes(self._h, int(lanes)), self._h)

    def use_own_stream(self):
        """Back to the context's own non-blocking stream (the default)."""
        _check(self._L.starch_use_own_stream(self._h), self._h)

    # -- the hot path ----------------------------------------------------------
    def _opts(self, emit_index=True, reference_compat=False):
        if self._method == K_GZIP and reference_compat:
            raise StarchError(-38, "This method is unsupported at this time")      # hpp:777-779
        if self._method == K_UNDEFINED:
            raise StarchError(-38, "This method is undefined")                      # hpp:780-782
        o = Options()
        self._L.starch_options_init(ctypes.byref(o))
        o.block_size_100k = self.block_size_100k
        o.emit_index = 1 if emit_index else 0
        o.reference_compat = 1 if reference_compat else 0
        o.base_counts = 1 if self.base_counts else 0
        # gzip (-g): one gzip member per segment (fixed-Huffman deflate on the GPU);
        # the reference itself stops with ENOSYS (kept under reference_compat)
        o.compression_method = 1 if self._method == K_GZIP else 0
        self._note_b = self._note.encode() if self._note else None
        o.note = self._note_b
        return o

    def compress(self, bed: bytes, emit_index=True, reference_compat=False) -> bytes:
        """BED bytes (host) -> Starch archive bytes."""
        o = self._opts(emit_index, reference_compat)
        _check(self._L.starch_encode_host(self._h, bed, len(bed), ctypes.byref(o)), self._h)
        return self.archive()

    def compress_host_ptr(self, ptr: int, n: int, emit_index=True):
        """BED bytes at a host address (e.g. pinned memory) -> archive in HBM."""
        o = self._opts(emit_index)
        _check(self._L.starch_encode_host(self._h, ctypes.cast(ctypes.c_void_p(ptr), ctypes.c_char_p), n,
                                          ctypes.byref(o)), self._h)

    def compress_host_into(self, ptr: int, n: int, out_ptr: int, cap: int, emit_index=True) -> int:
        """BED bytes at a host address -> archive written to the host address
        out_ptr (cap bytes); finished batches go device-to-host while later
        ones encode (starch_encode_host_into).  Returns the archive size."""
        o = self._opts(emit_index)
        k = ctypes.c_uint64()
        _check(self._L.starch_encode_host_into(self._h, ctypes.c_void_p(ptr), n, ctypes.byref(o),
                                               ctypes.c_void_p(out_ptr), cap, ctypes.byref(k)), self._h)
        return k.value

    # -- streaming ingestion (starch_stream_*) ----------------------------------
    def stream_begin(self, batch_bytes=0, emit_index=True, reference_compat=False):
        """Start a streamed encode; feed pieces, read archive bytes as they finish."""
        self._stream_opts = self._opts(emit_index, reference_compat)
        _check(self._L.starch_stream_begin(self._h, ctypes.byref(self._stream_opts), batch_bytes), self._h)

    def stream_feed(self, piece, n=None):
        """Feed host bytes (bytes-like, or an address with n)."""
        if n is None:
            buf = ctypes.c_char_p(bytes(piece)) if not isinstance(piece, bytes) else ctypes.c_char_p(piece)
            _check(self._L.starch_stream_feed(self._h, ctypes.cast(buf, ctypes.c_void_p), len(piece)), self._h)
        else:
            _check(self._L.starch_stream_feed(self._h, ctypes.c_void_p(piece), n), self._h)

    def stream_end(self):
        _check(self._L.starch_stream_end(self._h), self._h)

    def stream_read(self, into=None, cap=None) -> bytes:
        """Drain the archive bytes ready so far (or copy up to cap into an address; returns the count)."""
        if into is not None:
            k = ctypes.c_uint64()
            _check(self._L.starch_stream_read(self._h, ctypes.c_void_p(into), cap, ctypes.byref(k)), self._h)
            return k.value
        n = ctypes.c_uint64()
        _check(self._L.starch_stream_available(self._h, ctypes.byref(n)), self._h)
        buf = ctypes.create_string_buffer(max(1, n.value))
        k = ctypes.c_uint64()
        _check(self._L.starch_stream_read(self._h, buf, n.value, ctypes.byref(k)), self._h)
        return buf.raw[:k.value]

    def compress_stream(self, pieces, batch_bytes=0, emit_index=True, reference_compat=False) -> bytes:
        """Iterable of BED byte pieces -> the archive (streamed encode)."""
        self.stream_begin(batch_bytes, emit_index, reference_compat)
        out = [self.stream_read()]
        for p in pieces:
            self.stream_feed(p)
            out.append(self.stream_read())
        self.stream_end()
        out.append(self.stream_read())
        return b"".join(out)

    def archive_into(self, ptr: int, cap: int) -> int:
        """Copy the archive to a host address; returns its size."""
        n = self.archive_size()
        _check(self._L.starch_archive_copy(self._h, ctypes.c_void_p(ptr), cap), self._h)
        return n

    def compress_device(self, d_ptr: int, n: int, emit_index=True):
        """BED bytes already in HBM (device pointer) -> archive stays in HBM."""
        o = self._opts(emit_index)
        _check(self._L.starch_encode_device(self._h, ctypes.c_void_p(d_ptr), n, ctypes.byref(o)), self._h)

    def encode_units_device(self, d_base: int, units, unit_ids=None, emit_index=False):
        """One shard: units resident in HBM (offsets relative to d_base) -> this
        context's streams (no magic / index); segments() carry each unit id."""
        o = self._opts(emit_index)
        k = len(units)
        U = (Unit * max(1, k))(*units)
        ids = (ctypes.c_uint64 * max(1, k))(*(unit_ids if unit_ids is not None else range(k)))
        _check(self._L.starch_encode_units_device(self._h, ctypes.c_void_p(d_base), U, ids, k, ctypes.byref(o)),
               self._h)

    def encode_units_host(self, bed, units, unit_ids=None, emit_index=False):
        """One shard from host bytes: only the listed units (offsets into bed)
        are copied to HBM, packed; then as encode_units_device."""
        o = self._opts(emit_index)
        k = len(units)
        U = (Unit * max(1, k))(*units)
        ids = (ctypes.c_uint64 * max(1, k))(*(unit_ids if unit_ids is not None else range(k)))
        ptr = bed if isinstance(bed, int) else ctypes.cast(ctypes.c_char_p(bed), ctypes.c_void_p).value
        _check(self._L.starch_encode_units_host(self._h, ctypes.c_void_p(ptr), U, ids, k, ctypes.byref(o)), self._h)

    def gather_archive(self, comm, emit_index=True):
        """Collective over comm (one rank per GPU): every rank's streams from
        its last encode_units_* into rank 0's archive (RCCL, starch_gather_archive)."""
        o = self._opts(emit_index)
        _check(self._L.starch_gather_archive(self._h, comm._h, ctypes.byref(o)), self._h)

    def streams_device(self):
        """(device pointer, bytes) of the last starch_encode_units_device result."""
        p, n = ctypes.c_void_p(), ctypes.c_uint64()
        _check(self._L.starch_streams_device(self._h, ctypes.byref(p), ctypes.byref(n)), self._h)
        return p.value or 0, n.value

    def streams(self) -> bytes:
        n = self.streams_device()[1]
        buf = ctypes.create_string_buffer(max(1, n))
        _check(self._L.starch_streams_copy(self._h, buf, n), self._h)
        return buf.raw[:n]

    def archive_size(self):
        n = ctypes.c_uint64()
        _check(self._L.starch_archive_size(self._h, ctypes.byref(n)), self._h)
        return n.value

    def archive_device_ptr(self):
        p = ctypes.c_void_p()
        _check(self._L.starch_archive_device(self._h, ctypes.byref(p)), self._h)
        return p.value

    def archive(self) -> bytes:
        n = self.archive_size()
        buf = ctypes.create_string_buffer(max(1, n))
        _check(self._L.starch_archive_copy(self._h, buf, n), self._h)
        return buf.raw[:n]

    def segments(self):
        """[(chromosome bytes, Segment)] of the last call."""
        n = ctypes.c_uint64()
        _check(self._L.starch_segment_count(self._h, ctypes.byref(n)), self._h)
        arr = (Segment * max(1, n.value))()
        _check(self._L.starch_segments(self._h, arr, n.value), self._h)
        out = []
        for i in range(n.value):
            ln = ctypes.c_uint64()
            buf = ctypes.create_string_buffer(max(1, arr[i].name_len))
            _check(self._L.starch_segment_name(self._h, i, buf, arr[i].name_len, ctypes.byref(ln)), self._h)
            out.append((buf.raw[:ln.value], arr[i]))
        return out

    def stats(self):
        s = Stats()
        _check(self._L.starch_get_stats(self._h, ctypes.byref(s)), self._h)
        return {k: getattr(s, k) for k, _ in Stats._fields_}

    def transform(self, bed: bytes):
        """Transform stage only -> (text, [(chr, line_count, segment text)])."""
        _check(self._L.starch_transform_host(self._h, bed, len(bed)), self._h)
        n = ctypes.c_uint64()
        _check(self._L.starch_text_size(self._h, ctypes.byref(n)), self._h)
        buf = ctypes.create_string_buffer(max(1, n.value))
        _check(self._L.starch_text_copy(self._h, buf, n.value), self._h)
        text = buf.raw[:n.value]
        segs = []
        for name, s in self.segments():
            segs.append((name, s.line_count, text[s.stream_offset:s.stream_offset + s.text_bytes]))
        return text, segs

    def transform_device(self, d_ptr: int, n: int):
        """Transform stage only on BED bytes in HBM; the text stays in HBM
        (text_size / segments(); stats()["ms_transform"])."""
        _check(self._L.starch_transform_device(self._h, ctypes.c_void_p(d_ptr), n), self._h)

    def bz2_compress(self, data: bytes, level: int = 9) -> bytes:
        """One bzip2 stream, byte-identical to libbz2 BZ2_bzCompress(BZ_FINISH)."""
        cap = len(data) + len(data) // 50 + 4096
        buf = ctypes.create_string_buffer(cap)
        n = ctypes.c_uint64()
        _check(self._L.starch_bz2_compress_host(self._h, data, len(data), level, buf, cap, ctypes.byref(n)),
               self._h)
        return buf.raw[:n.value]

    def bz2_compress_many_device(self, d_in, offs, lens, level, d_out, cap):
        k = len(offs)
        O = (ctypes.c_uint64 * max(1, k))(*offs)
        N = (ctypes.c_uint64 * max(1, k))(*lens)
        oo = (ctypes.c_uint64 * max(1, k))()
        ol = (ctypes.c_uint64 * max(1, k))()
        _check(self._L.starch_bz2_compress_many_device(self._h, ctypes.c_void_p(d_in), O, N, k, level,
                                                       ctypes.c_void_p(d_out), cap, oo, ol), self._h)
        return list(oo[:k]), list(ol[:k])


    # ---- decompression / unstarch ----
    def _output(self) -> bytes:
        n = ctypes.c_uint64()
        _check(self._L.starch_output_size(self._h, ctypes.byref(n)), self._h)
        buf = ctypes.create_string_buffer(max(1, n.value))
        _check(self._L.starch_output_copy(self._h, buf, n.value), self._h)
        return buf.raw[:n.value]

    def bz2_decompress(self, data: bytes) -> bytes:
        """Concatenated bzip2 streams -> their bytes (GPU decode, CRCs checked)."""
        _check(self._L.starch_bz2_decompress_host(self._h, data, len(data)), self._h)
        return self._output()

    def bz2_decompress_device(self, d_ptr: int, n: int) -> int:
        """Device-resident streams; returns the output size (output_device_ptr())."""
        _check(self._L.starch_bz2_decompress_device(self._h, ctypes.c_void_p(d_ptr), n), self._h)
        k = ctypes.c_uint64()
        _check(self._L.starch_output_size(self._h, ctypes.byref(k)), self._h)
        return k.value

    def output_device_ptr(self) -> int:
        p = ctypes.c_void_p()
        _check(self._L.starch_output_device(self._h, ctypes.byref(p)), self._h)
        return p.value or 0

    def decoded_streams(self):
        n = ctypes.c_uint64()
        _check(self._L.starch_bz2_stream_count(self._h, ctypes.byref(n)), self._h)
        arr = (DecStream * max(1, n.value))()
        _check(self._L.starch_bz2_streams(self._h, arr, n.value), self._h)
        return [{f: getattr(arr[i], f) for f, _ in DecStream._fields_} for i in range(n.value)]

    def untransform(self, text: bytes, chromosome: bytes) -> bytes:
        """One segment's transformed text -> its BED lines (inverse of hpp:428-504)."""
        _check(self._L.starch_untransform_host(self._h, text, len(text), chromosome, len(chromosome)), self._h)
        return self._output()

    def unstarch(self, archive: bytes) -> bytes:
        """An archive of this library back to BED (decode + inverse transform on the GPU)."""
        _check(self._L.starch_unstarch_host(self._h, archive, len(archive)), self._h)
        return self._output()


def gen_bed(kind, total_lines, chroms=None, seed=20261015, into=None):
    """Synthetic hg38 BED (kind 0 BED3 / 1 narrowPeak / 2 per-position) for the
    given chromosome ids; returns bytes, or writes into a ctypes buffer."""
    L = load()
    chroms = list(range(24)) if chroms is None else list(chroms)
    C = (ctypes.c_int32 * max(1, len(chroms)))(*chroms)
    n = ctypes.c_uint64()
    _check(L.starch_gen_bed(kind, seed, total_lines, C, len(chroms), None, 0, ctypes.byref(n)))
    if into is not None:
        _check(L.starch_gen_bed(kind, seed, total_lines, C, len(chroms), into, n.value, ctypes.byref(n)))
        return n.value
    buf = ctypes.create_string_buffer(max(1, n.value))
    _check(L.starch_gen_bed(kind, seed, total_lines, C, len(chroms), buf, n.value, ctypes.byref(n)))
    return buf.raw[:n.value]


def gen_perpos_device(chrom, d_ptr=None, cap=0, first=0, count=None, stream=None):
    """Per-position lines of one chromosome written by the GPU at d_ptr (or,
    d_ptr None, just the byte count) -> byte count."""
    L = load()
    count = HG38_LEN[chrom] - first if count is None else count
    n = ctypes.c_uint64()
    _check(L.starch_gen_perpos_device(chrom, first, count, ctypes.c_void_p(d_ptr) if d_ptr else None, cap,
                                      ctypes.byref(n), ctypes.c_void_p(stream) if stream else None))
    return n.value


def gen_bed_sizes(kind, total_lines, chroms=None, seed=20261015):
    """Byte count of each chromosome's lines in gen_bed's output."""
    L = load()
    chroms = list(range(24)) if chroms is None else list(chroms)
    C = (ctypes.c_int32 * max(1, len(chroms)))(*chroms)
    out = (ctypes.c_uint64 * max(1, len(chroms)))()
    _check(L.starch_gen_bed_sizes(kind, seed, total_lines, C, len(chroms), out))
    return list(out[:len(chroms)])


def build_index(segs, names, index_offset, note=None, level=9, base_counts=False):
    """JSON index + 32-byte footer for already-placed streams (multi-GPU gather)."""
    L = load()
    k = len(segs)
    arr = (Segment * max(1, k))(*segs)
    nm = (ctypes.c_char_p * max(1, k))(*names)
    nl = (ctypes.c_uint64 * max(1, k))(*[len(x) for x in names])
    n = ctypes.c_uint64()
    note_b = note.encode() if note else None
    o = Options()
    L.starch_options_init(ctypes.byref(o))
    o.block_size_100k, o.note, o.base_counts = level, note_b, 1 if base_counts else 0
    _check(L.starch_build_index_opt(arr, nm, nl, k, index_offset, ctypes.byref(o), None, 0, ctypes.byref(n)))
    buf = ctypes.create_string_buffer(max(1, n.value))
    _check(L.starch_build_index_opt(arr, nm, nl, k, index_offset, ctypes.byref(o), buf, n.value, ctypes.byref(n)))
    return buf.raw[:n.value]


def plan_units(bed: bytes, max_units: int):
    """Split host BED bytes into <= max_units units whose boundaries are segment
    boundaries (starch_plan_units)."""
    L = load()
    out = (Unit * max(1, max_units))()
    n = ctypes.c_uint64()
    _check(L.starch_plan_units(bed, len(bed), max_units, out, ctypes.byref(n)))
    return [Unit(u.offset, u.length, u.init_start, u.init_stop) for u in out[:n.value]]


def assign_shards(units, nshards):
    """LPT assignment of units to shards -> list of shard indices."""
    L = load()
    k = len(units)
    U = (Unit * max(1, k))(*units)
    out = (ctypes.c_int32 * max(1, k))()
    _check(L.starch_assign_shards(U, k, nshards, out))
    return list(out[:k])


def archive_layout(unit_of, nbytes, base=4):
    """Archive order (stable by unit) and byte offsets of gathered segments ->
    (order, offsets, index offset)."""
    L = load()
    k = len(unit_of)
    A = (ctypes.c_uint64 * max(1, k))(*unit_of)
    B = (ctypes.c_uint64 * max(1, k))(*nbytes)
    o = (ctypes.c_uint64 * max(1, k))()
    f = (ctypes.c_uint64 * max(1, k))()
    end = ctypes.c_uint64()
    _check(L.starch_archive_layout(A, B, k, base, o, f, ctypes.byref(end)))
    return list(o[:k]), list(f[:k]), end.value


def compress_multi(ctxs, bed: bytes, emit_index=True, reference_compat=False) -> bytes:
    """In-process multi-device encode (starch_encode_multi_host): shards over
    the given contexts (they may share a device), archive read from ctxs[0]."""
    L = load()
    o = ctxs[0]._opts(emit_index, reference_compat)
    H = (ctypes.c_void_p * len(ctxs))(*[c._h.value for c in ctxs])
    _check(L.starch_encode_multi_host(H, len(ctxs), bed, len(bed), ctypes.byref(o)), ctxs[0]._h)
    return ctxs[0].archive()


class Comm:
    """One RCCL communicator per process (starch_comm_*): rank 0 makes the id
    (``Comm.new_id()``) and every rank passes it, or use ``Comm.tcp``."""

    def __init__(self, device, rank, world, comm_id):
        L = load()
        h = ctypes.c_void_p()
        rc = L.starch_comm_create(device, rank, world, ctypes.c_char_p(bytes(comm_id)), ctypes.byref(h))
        if rc:
            raise StarchError(rc, L.starch_comm_last_error().decode(errors="replace"))
        self._h, self._L, self.rank, self.world = h, L, rank, world

    @staticmethod
    def new_id() -> bytes:
        L = load()
        buf = ctypes.create_string_buffer(128)
        rc = L.starch_comm_id(buf)
        if rc:
            raise StarchError(rc, L.starch_comm_last_error().decode(errors="replace"))
        return buf.raw

    @classmethod
    def tcp(cls, device, rank, world, host, port):
        self = cls.__new__(cls)
        L = load()
        h = ctypes.c_void_p()
        rc = L.starch_comm_create_tcp(device, rank, world, host.encode(), port, ctypes.byref(h))
        if rc:
            raise StarchError(rc, L.starch_comm_last_error().decode(errors="replace"))
        self._h, self._L, self.rank, self.world = h, L, rank, world
        return self

    @staticmethod
    def rccl_library() -> str:
        """Path of the librccl the gather runs on (dladdr of its symbols)."""
        return (load().starch_rccl_library() or b"").decode(errors="replace")

    def close(self):
        if getattr(self, "_h", None):
            self._L.starch_comm_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def gather_host(rank, world, all_gather, send, recv, group_end, segs, names, streams: bytes, note=None, level=9,
                emit_index=True, base_counts=False, reference_compat=False):
    """The library's gather (starch_gather_host) over caller primitives on host
    bytes: all_gather(bytes) -> [bytes per rank]; send(bytes, peer);
    recv(n, peer) -> a handle; group_end() -> {handle: bytes} for the recvs
    posted since the last group_end.  Returns the archive on rank 0, else None."""
    L = load()
    pending = {}

    def _ag(_u, sp, rp, n):
        try:
            parts = all_gather(ctypes.string_at(sp, n))
            for r, p in enumerate(parts):
                ctypes.memmove(rp + r * n, p, n)
            return 0
        except Exception:
            return 1

    def _send(_u, p, n, peer):
        try:
            send(ctypes.string_at(p, n), peer)
            return 0
        except Exception:
            return 1

    def _recv(_u, p, n, peer):
        try:
            pending[recv(n, peer)] = (p, n)
            return 0
        except Exception:
            return 1

    def _end(_u):
        try:
            got = group_end()
            for h, data in got.items():
                p, n = pending.pop(h)
                ctypes.memmove(p, data, n)
            return 0
        except Exception:
            return 1

    hc = HostComm(rank, world, None, _AG_FN(_ag), _SEND_FN(_send), _RECV_FN(_recv), _END_FN(_end))
    k = len(segs)
    arr = (Segment * max(1, k))(*segs)
    nm = (ctypes.c_char_p * max(1, k))(*names)
    nl = (ctypes.c_uint64 * max(1, k))(*[len(x) for x in names])
    o = Options()
    L.starch_options_init(ctypes.byref(o))
    note_b = note.encode() if note else None
    o.block_size_100k, o.note, o.base_counts = level, note_b, 1 if base_counts else 0
    o.emit_index, o.reference_compat = 1 if emit_index else 0, 1 if reference_compat else 0
    sbuf = ctypes.create_string_buffer(streams, max(1, len(streams)))
    out, n = ctypes.c_void_p(), ctypes.c_uint64()
    rc = L.starch_gather_host(ctypes.byref(hc), arr, nm, nl, k, sbuf, ctypes.byref(o), ctypes.byref(out),
                              ctypes.byref(n))
    if rc:
        raise StarchError(rc, L.starch_comm_last_error().decode(errors="replace"))
    if not out.value:
        return None
    try:
        return ctypes.string_at(out.value, n.value)
    finally:
        L.starch_free(out)


def parse_archive(blob: bytes):
    """Split an archive into (index dict, [stream bytes]) using its footer."""
    if blob[:4] != MAGIC:
        raise ValueError("bad magic")
    foot = blob[-32:]
    off = int(foot[:20])
    idx = json.loads(blob[off:-32].decode("utf-8"))
    streams = [blob[s["offset"]:s["offset"] + s["size"]] for s in idx["streams"]]
    return idx, streams
