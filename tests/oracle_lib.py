"""ctypes access to the CPU oracle (TEST INFRASTRUCTURE ONLY).

oracle/_build/libstarch_oracle.so : the C restatement (oracle/starch_oracle.c)
oracle/_ref/libbz2ref.so          : the reference's vendored libbz2 (optional;
                                    built here from /root/reference, travels
                                    to the GPU box as a prebuilt binary)
"""
import ctypes
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(ROOT, "oracle", "_build", "libstarch_oracle.so")
REF_SO = os.path.join(ROOT, "oracle", "_ref", "libbz2ref.so")


class Seg(ctypes.Structure):
    _fields_ = [("name_off", ctypes.c_uint64), ("name_len", ctypes.c_uint64),
                ("line_count", ctypes.c_uint64), ("text_off", ctypes.c_uint64),
                ("text_len", ctypes.c_uint64)]


_lib = None
_ref = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"),
                                   os.path.join(ROOT, "oracle", "_build", "libstarch_oracle.so")])
        L = ctypes.CDLL(ORACLE_SO)
        L.oracle_transform.restype = ctypes.c_size_t
        L.oracle_transform_init.restype = ctypes.c_size_t
        L.oracle_bz2_compress.restype = ctypes.c_size_t
        L.oracle_crc32_bzip2.restype = ctypes.c_uint32
        L.oracle_block_sort.restype = ctypes.c_int32
        L.oracle_base_counts.restype = ctypes.c_size_t
        L.oracle_untransform.restype = ctypes.c_size_t
        _lib = L
    return _lib


def ref():
    """The reference's libbz2 (None when oracle/_ref was not built)."""
    global _ref
    if _ref is None and os.path.exists(REF_SO):
        R = ctypes.CDLL(REF_SO)
        R.ref_bz2_compress.restype = ctypes.c_int
        R.ref_bz2_script.restype = ctypes.c_int
        R.ref_bz2_script_trace.restype = ctypes.c_int
        R.ref_bz2_version.restype = ctypes.c_char_p
        _ref = R
    return _ref


def transform(data: bytes, init_start=0, init_stop=0):
    """-> (text bytes, [(chr bytes, line_count, text bytes)]); init_* are the
    sscanf values current before the first line (0 for a whole input)."""
    L = lib()
    cap = 2 * len(data) + 64 * (data.count(b"\n") + 1) + 1024
    seg_cap = data.count(b"\n") + 2
    out = ctypes.create_string_buffer(cap)
    segs = (Seg * seg_cap)()
    nseg = ctypes.c_size_t(0)
    n = L.oracle_transform_init(data, ctypes.c_size_t(len(data)), out, ctypes.c_size_t(cap),
                                segs, ctypes.c_size_t(seg_cap), ctypes.byref(nseg),
                                ctypes.c_int64(init_start), ctypes.c_int64(init_stop))
    assert n != ctypes.c_size_t(-1).value
    text = out.raw[:n]
    res = []
    for s in segs[:nseg.value]:
        res.append((data[s.name_off:s.name_off + s.name_len], s.line_count,
                    text[s.text_off:s.text_off + s.text_len]))
    return text, res


def base_counts(data: bytes, init_start=0, init_stop=0):
    """-> [(unique, nonunique)] per segment (int64; oracle/starch_oracle.c
    oracle_base_counts)."""
    L = lib()
    seg_cap = data.count(b"\n") + 2
    bu = (ctypes.c_uint64 * seg_cap)()
    bn = (ctypes.c_uint64 * seg_cap)()
    nseg = ctypes.c_size_t(0)
    r = L.oracle_base_counts(data, ctypes.c_size_t(len(data)), ctypes.c_int64(init_start), ctypes.c_int64(init_stop),
                             bu, bn, ctypes.c_size_t(seg_cap), ctypes.byref(nseg))
    assert r == 0
    s64 = lambda v: v - (1 << 64) if v >= 1 << 63 else v
    return [(s64(bu[i]), s64(bn[i])) for i in range(nseg.value)]


def bz2(data: bytes, bs: int = 9) -> bytes:
    L = lib()
    cap = len(data) + len(data) // 50 + 1024
    out = ctypes.create_string_buffer(cap)
    n = L.oracle_bz2_compress(data, ctypes.c_size_t(len(data)), bs, out, ctypes.c_size_t(cap))
    assert n != ctypes.c_size_t(-1).value
    return out.raw[:n]


def ref_bz2(data: bytes, bs: int = 9, wf: int = 30) -> bytes:
    R = ref()
    cap = len(data) + len(data) // 50 + 1024
    out = ctypes.create_string_buffer(cap)
    n = ctypes.c_size_t(0)
    rc = R.ref_bz2_compress(data, ctypes.c_size_t(len(data)), bs, wf, out, ctypes.c_size_t(cap),
                            ctypes.byref(n))
    assert rc == 0, rc
    return out.raw[:n.value]


def ref_bz2_script(data: bytes, ops, bs=9, wf=30, out_chunk=0):
    """ops: [(action, nbytes)] -> (stream bytes, [rc per op])"""
    R = ref()
    arr = (ctypes.c_int32 * (2 * len(ops)))(*[v for op in ops for v in op])
    rcs = (ctypes.c_int32 * len(ops))()
    cap = len(data) + len(data) // 50 + 4096 + 64 * len(ops)
    out = ctypes.create_string_buffer(cap)
    n = ctypes.c_size_t(0)
    rc = R.ref_bz2_script(data, arr, len(ops), bs, wf, ctypes.c_size_t(out_chunk), out,
                          ctypes.c_size_t(cap), ctypes.byref(n), rcs)
    assert rc == 0, rc
    return out.raw[:n.value], list(rcs)


def ref_bz2_script_trace(data: bytes, ops, bs=9, wf=30, out_chunk=0):
    """ops: [(action, nbytes)] -> (stream bytes, [rc per op], [total output after each op])"""
    R = ref()
    arr = (ctypes.c_int32 * (2 * len(ops)))(*[v for op in ops for v in op])
    rcs = (ctypes.c_int32 * len(ops))()
    after = (ctypes.c_uint64 * len(ops))()
    cap = len(data) + len(data) // 50 + 4096 + 64 * len(ops)
    out = ctypes.create_string_buffer(cap)
    n = ctypes.c_size_t(0)
    rc = R.ref_bz2_script_trace(data, arr, len(ops), bs, wf, ctypes.c_size_t(out_chunk), out,
                                ctypes.c_size_t(cap), ctypes.byref(n), rcs, after)
    assert rc == 0, rc
    return out.raw[:n.value], list(rcs), list(after)


def block_sort(block: bytes):
    L = lib()
    fmap = (ctypes.c_uint32 * max(1, len(block)))()
    op = L.oracle_block_sort(block, ctypes.c_int32(len(block)), fmap)
    return op, list(fmap[:len(block)])


def untransform(text: bytes, chromosome: bytes):
    """One segment's text -> BED lines (oracle_untransform), or None when the
    text is not invertible (negative p-value, malformed line)."""
    L = lib()
    cap = 4 * len(text) + (len(chromosome) + 48) * (text.count(b"\n") + 1) + 1024
    out = ctypes.create_string_buffer(cap)
    n = L.oracle_untransform(text, ctypes.c_size_t(len(text)), chromosome, ctypes.c_size_t(len(chromosome)), out,
                             ctypes.c_size_t(cap))
    if n == ctypes.c_size_t(-1).value:
        return None
    return out.raw[:n]


POOL_SO = os.path.join(ROOT, "oracle", "_build", "libcpu_pool.so")
_pool = None


def cpu_pool(buf, spans, threads, level=9, use_ref=True):
    """CPU baseline (oracle/cpu_pool.c): transform + bzip2 of every (offset,
    length) piece of `buf` (bytes, or an int host address) on a C pthread
    pool, largest piece first, the reference libbz2 when built ->
    (seconds, [seconds per piece], [bz2 bytes per piece], codec kind)."""
    global _pool
    if _pool is None:
        if not os.path.exists(POOL_SO):
            subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), POOL_SO])
        _pool = ctypes.CDLL(POOL_SO)
        _pool.cpu_pool_run.restype = ctypes.c_int
    n = len(spans)
    offs = (ctypes.c_uint64 * max(1, n))(*[o for o, _ in spans])
    lens = (ctypes.c_uint64 * max(1, n))(*[l for _, l in spans])
    secs = (ctypes.c_double * max(1, n))()
    outb = (ctypes.c_uint64 * max(1, n))()
    tot = ctypes.c_double(0)
    ref_path = REF_SO if (use_ref and os.path.exists(REF_SO)) else ""
    ptr = ctypes.c_void_p(buf) if isinstance(buf, int) else ctypes.c_char_p(buf)
    rc = _pool.cpu_pool_run(ptr, offs, lens, n, threads, level, ref_path.encode(), ctypes.byref(tot), secs, outb)
    assert rc == 0, rc
    return tot.value, list(secs[:n]), list(outb[:n]), ("reference" if ref_path else "port")
