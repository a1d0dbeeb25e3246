"""The patched-libbz2 ABI (include/starch_bzlib.h) exported by
libstarch_amd.so, driven with the same call sequences as the reference's
vendored libbz2 (oracle/_ref/libbz2ref.so): identical bytes and return codes."""
import ctypes
import random

import pytest

from tests import oracle_lib

pytestmark = pytest.mark.gpu

BZ_RUN, BZ_FLUSH, BZ_FINISH = 0, 1, 2
BZ_RUN_OK, BZ_FINISH_OK, BZ_STREAM_END = 1, 3, 4


class BzStream(ctypes.Structure):
    _fields_ = [("next_in", ctypes.c_void_p), ("avail_in", ctypes.c_uint), ("total_in_lo32", ctypes.c_uint),
                ("total_in_hi32", ctypes.c_uint), ("next_out", ctypes.c_void_p), ("avail_out", ctypes.c_uint),
                ("total_out_lo32", ctypes.c_uint), ("total_out_hi32", ctypes.c_uint), ("state", ctypes.c_void_p),
                ("bzalloc", ctypes.c_void_p), ("bzfree", ctypes.c_void_p), ("opaque", ctypes.c_void_p),
                ("handler", ctypes.c_void_p), ("block_close_functor", ctypes.c_void_p)]


def _lib():
    import starch_amd
    L = starch_amd.load()
    for n in ("BZ2_bzCompressInit", "BZ2_bzCompress", "BZ2_bzCompressEnd"):
        getattr(L, n).restype = ctypes.c_int
    return L


def _ref_lib():
    R = oracle_lib.ref()
    for n in ("BZ2_bzCompressInit", "BZ2_bzCompress", "BZ2_bzCompressEnd"):
        getattr(R, n).restype = ctypes.c_int
    return R


def run_script(data, ops, bs=9, out_chunk=0, trace=None, lib=None, calls=None, src=None):
    """Drive a bzlib ABI (default: the GPU one) like ref_bz2_script does
    (trace: list that gets the total output after each op; calls: list that
    gets (op, rc, total_in, total_out) after EVERY BZ2_bzCompress call)."""
    L = lib or _lib()
    s = BzStream()
    assert L.BZ2_bzCompressInit(ctypes.byref(s), bs, 0, 30) == 0
    called = []
    CB = ctypes.CFUNCTYPE(None, ctypes.c_void_p)
    cb = CB(lambda h: called.append(h))
    s.block_close_functor = ctypes.cast(cb, ctypes.c_void_p)
    if src is None:
        src = ctypes.create_string_buffer(data, len(data) + 1)
    cap = len(data) + len(data) // 50 + 4096 + 64 * len(ops)
    out = ctypes.create_string_buffer(cap)
    used = produced = 0
    rcs = []
    for act, nbytes in ops:
        s.next_in = ctypes.addressof(src) + used
        s.avail_in = nbytes
        used += nbytes
        while True:
            room = cap - produced
            if out_chunk:
                room = min(room, out_chunk)
            s.next_out = ctypes.addressof(out) + produced
            s.avail_out = room
            rc = L.BZ2_bzCompress(ctypes.byref(s), act)
            produced += room - s.avail_out
            if calls is not None:
                calls.append((len(rcs), rc, s.total_in_hi32 << 32 | s.total_in_lo32,
                              s.total_out_hi32 << 32 | s.total_out_lo32))
            if rc < 0:
                raise AssertionError("rc %d" % rc)
            if act == BZ_RUN and s.avail_in == 0:
                break
            if act == BZ_FLUSH and rc == BZ_RUN_OK:
                break
            if act == BZ_FINISH and rc == BZ_STREAM_END:
                break
        rcs.append(rc)
        if trace is not None:
            trace.append(produced)
    assert (s.total_in_hi32 << 32 | s.total_in_lo32) == used
    assert (s.total_out_hi32 << 32 | s.total_out_lo32) == produced
    assert L.BZ2_bzCompressEnd(ctypes.byref(s)) == 0
    assert called, "block_close_functor not called at BZ_STREAM_END"
    return out.raw[:produced], rcs


def test_single_finish_matches_reference():
    r = random.Random(5)
    for n in (0, 1, 100, 5000, 250000):
        data = bytes(r.choice(b"0123\np-") for _ in range(n))
        got, rcs = run_script(data, [(BZ_FINISH, n)])
        assert got == oracle_lib.bz2(data, 9)
        assert rcs == [BZ_STREAM_END]


@pytest.mark.skipif(oracle_lib.ref() is None, reason="oracle/_ref not built")
def test_call_sequences_match_reference_lib():
    r = random.Random(17)
    for trial in range(12):
        n = r.randint(1000, 300000)
        if trial % 3 == 0:
            data = b"ab" * (n // 2)
        elif trial % 3 == 1:
            data = b"".join(bytes([r.randrange(3) + 48]) * r.choice([1, 2, 5, 255, 300]) for _ in range(n // 60))
        else:
            data = bytes(r.choice(b"0123456789\n") for _ in range(n))
        # random split into RUN / FLUSH pieces, then FINISH with the tail (maybe empty)
        ops, left = [], len(data)
        while left > 0 and len(ops) < 6:
            k = r.randint(0, left)
            ops.append((r.choice([BZ_RUN, BZ_RUN, BZ_FLUSH]), k))
            left -= k
        ops.append((BZ_FINISH, left))
        bs = r.choice([1, 9])
        want, _ = oracle_lib.ref_bz2_script(data, ops, bs=bs)
        got, _ = run_script(data, ops, bs=bs, out_chunk=r.choice([0, 997]))
        assert got == want, (trial, ops, bs)


@pytest.mark.skipif(oracle_lib.ref() is None, reason="oracle/_ref not built")
def test_full_block_then_empty_finish_final_run_rule():
    # RUN all input so that the last byte leaves a full block behind, then an
    # empty FINISH: the final single-byte run must start a new block
    # (bz:bzlib.c:399-402 in RUN mode) -- unlike a FINISH that carries it.
    base = bytes((i * 7919) % 251 for i in range(99981))   # fills a level-1 block exactly
    for data in (base + b"Z", base + b"ZZ", base[:-1] + b"QZ"):
        for ops in ([(BZ_RUN, len(data)), (BZ_FINISH, 0)], [(BZ_FINISH, len(data))],
                    [(BZ_RUN, len(data) - 1), (BZ_FINISH, 1)]):
            want, _ = oracle_lib.ref_bz2_script(data, ops, bs=1)
            got, _ = run_script(data, ops, bs=1)
            assert got == want, ops


@pytest.mark.skipif(oracle_lib.ref() is None, reason="oracle/_ref not built")
def test_flush_emits_the_flushed_blocks():
    """BZ_FLUSH makes every whole byte so far readable, as the patched library
    does (bz:bzlib.c:437-459, the bit buffer carried across blocks by
    bz:compress.c:609): after every FLUSH the GPU ABI has produced exactly the
    bytes the reference libbz2 has (prefix of the final stream), also when the
    output arrives in 997-byte pieces (BZ_FLUSH_OK draining)."""
    r = random.Random(23)
    for trial in range(10):
        n = r.randint(2000, 600000)
        data = bytes(r.choice(b"0123456789\np-") for _ in range(n))
        ops, left = [], n
        while left > 1 and len(ops) < 7:
            act = r.choice([BZ_RUN, BZ_FLUSH, BZ_FLUSH])
            k = r.randint(1 if act == BZ_RUN else 0, left // 2 + 1)
            ops.append((act, k))
            left -= k
        ops.append((BZ_FLUSH, 0))                    # an empty flush: nothing new
        ops.append((BZ_FINISH, left))
        bs = r.choice([1, 9])
        chunk = r.choice([0, 997])
        want, wrcs, wafter = oracle_lib.ref_bz2_script_trace(data, ops, bs=bs, out_chunk=chunk)
        trace = []
        got, rcs = run_script(data, ops, bs=bs, out_chunk=chunk, trace=trace)
        assert got == want, (trial, ops)
        assert rcs == wrcs, (trial, ops)
        assert trace == wafter, (trial, ops, trace, wafter)   # BZ_RUN included: full blocks go out at once


def test_param_and_sequence_errors():
    L = _lib()
    s = BzStream()
    assert L.BZ2_bzCompressInit(ctypes.byref(s), 0, 0, 30) == -2
    assert L.BZ2_bzCompressInit(ctypes.byref(s), 9, 0, 251) == -2
    assert L.BZ2_bzCompressInit(ctypes.byref(s), 9, 0, 0) == 0
    # BZ_RUN without input makes no progress -> BZ_PARAM_ERROR (bz:bzlib.c:432-434)
    s.avail_in = 0
    assert L.BZ2_bzCompress(ctypes.byref(s), BZ_RUN) == -2
    out = ctypes.create_string_buffer(64)
    s.next_out = ctypes.addressof(out)
    s.avail_out = 64
    assert L.BZ2_bzCompress(ctypes.byref(s), BZ_FINISH) == BZ_STREAM_END   # functor NULL: allowed
    assert L.BZ2_bzCompress(ctypes.byref(s), BZ_FINISH) == -1              # IDLE -> sequence error
    assert L.BZ2_bzCompressEnd(ctypes.byref(s)) == 0
    assert L.BZ2_bzCompressEnd(ctypes.byref(s)) == -2


def test_threads_encode_concurrently_and_keep_their_device():
    """Streams of several threads (the encode must not depend on or
    change the calling thread's current HIP device)."""
    import threading
    import torch
    r = random.Random(17)
    inputs = [bytes(r.choice(b"0123456789\np-") for _ in range(r.randint(1000, 400000))) for _ in range(6)]
    results, devs = [None] * len(inputs), [None] * len(inputs)

    def work(i):
        results[i] = run_script(inputs[i], [(BZ_FINISH, len(inputs[i]))])[0]
        devs[i] = torch.cuda.current_device()

    ths = [threading.Thread(target=work, args=(i,)) for i in range(len(inputs))]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    for i, d in enumerate(inputs):
        assert results[i] == oracle_lib.bz2(d, 9), i
    assert devs == [0] * len(inputs)


def test_default_allocators_installed():
    """bzalloc / bzfree default to malloc / free like bz:bzlib.c:165-166."""
    L = _lib()
    s = BzStream()
    assert L.BZ2_bzCompressInit(ctypes.byref(s), 9, 0, 30) == 0
    assert s.bzalloc and s.bzfree and s.state
    assert L.BZ2_bzCompressEnd(ctypes.byref(s)) == 0
    assert not s.state


@pytest.mark.skipif(oracle_lib.ref() is None, reason="oracle/_ref not built")
@pytest.mark.parametrize("seed", range(6))
def test_every_call_matches_reference_lib(seed):
    _every_call(seed, (0, 4093, 65536))


@pytest.mark.skipif(oracle_lib.ref() is None, reason="oracle/_ref not built")
@pytest.mark.parametrize("seed", range(6))
def test_every_call_matches_reference_lib_small_ahead(seed, monkeypatch):
    """The same with the coded-ahead limit at 300 KB (STARCH_BZ_AHEAD): FLUSH /
    FINISH commitments and BZ_RUN input larger than it are coded in open
    plans whose last block is dropped and re-planned from the pending run."""
    monkeypatch.setenv("STARCH_BZ_AHEAD", "300000")
    _every_call(seed, (0, 65536))


def _script(seed):
    r = random.Random(100 + seed)
    bs = 1 if seed % 2 == 0 else 9
    n = r.randint(300_000, 2_600_000) if bs == 1 else r.randint(1_000_000, 3_000_000)
    kind = seed % 3
    if kind == 0:
        data = bytes(r.choice(b"0123456789\np-") for _ in range(n))
    elif kind == 1:
        data = b"".join(bytes([r.randrange(4) + 48]) * r.choice([1, 1, 2, 3, 4, 5, 255, 256, 700]) for _ in range(n // 40))
    else:
        data = (b"p1\n" + b"0\n" * (n // 2))[:n]
    ops, left = [], len(data)
    while left > 0 and len(ops) < 9:
        act = r.choice([BZ_RUN, BZ_RUN, BZ_RUN, BZ_FLUSH])
        k = r.randint(1, max(1, left // 2)) if act == BZ_RUN else r.randint(0, left // 3)
        ops.append((act, k))
        left -= k
    ops.append((BZ_FINISH, left))
    return data, ops, bs


@pytest.mark.skipif(oracle_lib.ref() is None, reason="oracle/_ref not built")
@pytest.mark.parametrize("ahead", [0, 300000])
def test_concurrent_streams_share_plans(ahead, monkeypatch):
    """Streams of eight threads at once, levels 1 and 9 mixed: their blocks are
    coded in shared GPU plans (one plan per free encoder slot for every queued
    request of the same block size; with a 300 KB coded-ahead limit some
    pieces are open) and every call of every stream still matches the
    reference library (return code, total_in, total_out, bytes)."""
    import threading
    if ahead:
        monkeypatch.setenv("STARCH_BZ_AHEAD", str(ahead))
    scripts = [_script(s) for s in range(8)]
    want = []
    for data, ops, bs in scripts:
        calls = []
        out, rcs = run_script(data, ops, bs=bs, lib=_ref_lib(), calls=calls)
        want.append((out, rcs, calls))
    got = [None] * len(scripts)

    def work(i):
        data, ops, bs = scripts[i]
        calls = []
        out, rcs = run_script(data, ops, bs=bs, calls=calls)
        got[i] = (out, rcs, calls)

    ths = [threading.Thread(target=work, args=(i,)) for i in range(len(scripts))]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    for i in range(len(scripts)):
        assert got[i] is not None, i
        assert got[i][0] == want[i][0], i
        assert got[i][1] == want[i][1], i
        assert got[i][2] == want[i][2], i


def _every_call(seed, chunks):
    """libbz2's state machine call for call (bz:bzlib.c:369-471): the reference
    library and the GPU ABI driven by the same Python loop give the same return
    code, total_in and total_out after EVERY BZ2_bzCompress call -- BZ_RUN
    closing blocks at nblockMAX and stopping input while output is pending,
    FLUSH / FINISH draining in small pieces -- at levels 1 and 9, over
    multi-block inputs (runs across block ends included)."""
    data, ops, bs = _script(seed)
    for chunk in chunks:
        want_calls, got_calls = [], []
        want, wrcs = run_script(data, ops, bs=bs, out_chunk=chunk, lib=_ref_lib(), calls=want_calls)
        got, rcs = run_script(data, ops, bs=bs, out_chunk=chunk, calls=got_calls)
        assert got == want, (seed, chunk)
        assert rcs == wrcs
        assert got_calls == want_calls, (seed, chunk, ops)


@pytest.mark.skipif(oracle_lib.ref() is None, reason="oracle/_ref not built")
def test_run_emits_blocks_before_finish():
    """BZ_RUN with 1 MiB pieces over 20 MB: output appears while input is
    still arriving (every completed block), call for call as the library."""
    import starch_amd
    data = starch_amd.gen_bed(0, 900_000)[:20_000_000]
    ops = [(BZ_RUN, len(data[i:i + (1 << 20)])) for i in range(0, len(data), 1 << 20)] + [(BZ_FINISH, 0)]
    want_calls, got_calls = [], []
    want, _ = run_script(data, ops, lib=_ref_lib(), calls=want_calls)
    got, _ = run_script(data, ops, calls=got_calls)
    assert got == want and got_calls == want_calls
    assert got_calls[len(ops) // 2][3] > 0          # bytes out halfway through the RUN calls


def test_threads_share_one_large_input_buffer():
    """two streams coding from ONE shared caller buffer of >= 16 MiB
    at once (the bzlib ABI DMAs such input from a registration made for the
    call): the registration is shared and refcounted, so neither thread's copy
    runs after the other unregistered it.  Repeated, with the threads started
    together, and checked against system libbz2."""
    import bz2
    import threading
    import starch_amd
    data = bytes(starch_amd.gen_bed(0, 2_000_000)[:40_000_000])
    want = bz2.compress(data, 9)
    src = ctypes.create_string_buffer(data, len(data) + 1)
    for rep in range(3):
        got = [None, None]
        go = threading.Barrier(2)

        def work(i):
            go.wait()
            got[i] = run_script(data, [(BZ_FINISH, len(data))], src=src)[0]

        ths = [threading.Thread(target=work, args=(i,)) for i in range(2)]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        assert got[0] == want and got[1] == want, rep


@pytest.mark.skipif(oracle_lib.ref() is None, reason="oracle/_ref not built")
def test_finish_closes_block_coded_ahead_on_its_closing_byte():
    """a block coded ahead as closed by nblockMAX whose closing byte
    is the last byte of a FLUSH / FINISH (so libbz2 flushes the pending run
    into it instead): coded again from the bytes the call just consumed.
    Level 1, text without runs, the FLUSH / FINISH ending around each of the
    first block ends."""
    r = random.Random(31)
    data = bytes(r.choice(b"0123456789\np-") for _ in range(420_000))
    m = 99981
    for end in (m, m + 1, 2 * m, 2 * m + 1, 2 * m + 2, 3 * m + 1):
        for first in (BZ_RUN, BZ_FLUSH):
            ops = [(first, 50_000), (BZ_RUN, 250_000), (BZ_FINISH, end + 1 - 300_000 if end + 1 > 300_000 else 0)]
            if end + 1 <= 300_000:
                ops = [(first, 50_000), (BZ_RUN, end - 50_000), (BZ_FINISH, 1)]
            n = sum(k for _, k in ops)
            d = data[:n]
            want_calls, got_calls = [], []
            want, _ = run_script(d, ops, bs=1, lib=_ref_lib(), calls=want_calls)
            got, _ = run_script(d, ops, bs=1, calls=got_calls)
            assert got == want and got_calls == want_calls, (end, first)
