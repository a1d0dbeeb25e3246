"""Streaming ingestion: BED bytes fed in pieces of any size
through starch_stream_begin/feed/end, finished chromosome runs encoded on the
GPU as the input passes them, archive bytes read out as they finish.  The
concatenated output must equal the one-call archive of the whole input byte
for byte (the same bar as the multi-GPU shard path), whatever the piece sizes
and batch thresholds, including pieces that split lines, tokens and CRLF-free
tails, stale sscanf values across a cut, revisited chromosomes, NUL bytes and
a 0xFF that ends the input mid-piece."""
import os
import subprocess
import sys

import pytest

from tests import corpus

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _one_call(data, **kw):
    import starch_amd
    c = starch_amd.Starch(0)
    a = c.compress(data, **kw)
    c.close()
    return a


def _pieces(data, size):
    return [data[i:i + size] for i in range(0, len(data), size)]


def _streamed(data, piece, batch, **kw):
    import starch_amd
    c = starch_amd.Starch(0)
    a = c.compress_stream(_pieces(data, piece), batch_bytes=batch, **kw)
    st = c.stats()
    c.close()
    return a, st


@pytest.mark.parametrize("piece,batch", [(1 << 20, 1), (65_537, 300_000), (4_093, 1 << 20), (10 ** 9, 0)])
def test_stream_hg38_identical(piece, batch):
    import starch_amd
    data = starch_amd.gen_bed(0, 400_000)
    ref = _one_call(data)
    got, st = _streamed(data, piece, batch)
    assert got == ref
    assert st["input_bytes"] == len(data)
    assert st["n_segments"] == 24


@pytest.mark.parametrize("seed", range(4))
def test_stream_quirky_inputs(seed):
    data = (corpus.fuzz_bed(seed, 3000) + corpus.multi_chrom_bed(5, 400, seed, "bed6") +
            corpus.parseable_fuzz_bed(seed, 2000) + b"chr9\tx\ty\nchr9\t1")
    ref = _one_call(data)
    for piece, batch in ((997, 1), (7, 5000), (1 << 16, 1 << 16)):
        got, _ = _streamed(data, piece, batch)
        assert got == ref, (piece, batch)


def test_stream_stale_values_across_cut():
    """A chromosome whose first lines do not parse keeps the previous
    chromosome's last values (hpp:306-307): the streamed cut must carry them."""
    data = (b"chrA\t10\t20\nchrA\t30\t45\n" + b"chrB\tq\tz\nchrB\t7\tw\n" * 50 +
            b"chrC\t5\t9\nchrC\tx\t12\n" + b"chrD\tx\ty\n" * 30)
    ref = _one_call(data)
    for piece in (1, 3, 16, 31):
        got, _ = _streamed(data, piece, 1)
        assert got == ref, piece


def test_stream_ff_ends_input():
    import starch_amd
    head = starch_amd.gen_bed(0, 20_000)
    data = head + b"chrZ\t1\t2\n\xffchrZ\t3\t4\n" + head
    ref = _one_call(data)
    got, st = _streamed(data, 4096, 1)
    assert got == ref
    assert st["input_bytes"] == data.index(b"\xff")


def test_stream_ff_in_large_piece():
    """Pieces >= 8 MiB are copied by the session's thread pool, which finds the
    first 0xFF while copying: the input still ends there."""
    import starch_amd
    head = starch_amd.gen_bed(0, 1_500_000)
    data = head + b"chrZ\t1\t2\n\xffchrZ\t3\t4\n" + head
    ref = _one_call(data)
    got, st = _streamed(data, 24 << 20, 1 << 20)
    assert got == ref
    assert st["input_bytes"] == data.index(b"\xff")


@pytest.mark.parametrize("kw", [dict(emit_index=False), dict(reference_compat=True)])
def test_stream_options(kw):
    import starch_amd
    data = starch_amd.gen_bed(1, 50_000)
    assert _streamed(data, 10_000, 100_000, **kw)[0] == _one_call(data, **kw)


def test_stream_empty_and_tiny():
    assert _streamed(b"", 1, 1)[0] == _one_call(b"")
    assert _streamed(b"chr1\t1\t2", 1, 1)[0] == _one_call(b"chr1\t1\t2")


def test_stream_segments_and_reads_interleaved():
    """Streams become readable before end(); segments() after end() describe
    the whole archive (offsets into the streamed bytes)."""
    import starch_amd
    data = starch_amd.gen_bed(0, 200_000)
    c = starch_amd.Starch(0)
    c.stream_begin(batch_bytes=1 << 20)
    out = [c.stream_read()]
    assert out[0] == starch_amd.MAGIC
    early = 0
    for p in _pieces(data, 1 << 20):
        c.stream_feed(p)
        out.append(c.stream_read())
        early += len(out[-1])
    assert early > 0                      # streams came out while input was still arriving
    c.stream_end()
    out.append(c.stream_read())
    arch = b"".join(out)
    assert arch == _one_call(data)
    idx, streams = starch_amd.parse_archive(arch)
    segs = c.segments()
    assert [n.decode() for n, _ in segs] == starch_amd.HG38
    for (n, s), st in zip(segs, streams):
        assert arch[s.stream_offset:s.stream_offset + s.stream_bytes] == st
    with pytest.raises(starch_amd.StarchError):
        c.archive()                       # the bytes went out through stream_read
    c.close()


def test_cli_streams_stdin(tmp_path):
    """starch3 < file (streamed, small batches) == starch3 --slurp == one call."""
    import starch_amd
    data = starch_amd.gen_bed(0, 300_000) + corpus.fuzz_bed(3, 500)
    f = tmp_path / "in.bed"
    f.write_bytes(data)
    exe = os.path.join(ROOT, "starch_amd", "_build", "starch3")
    with open(f, "rb") as fin:
        a = subprocess.run([exe, "--batch-mb", "1"], stdin=fin, capture_output=True, timeout=120)
    b = subprocess.run([exe, "--slurp", str(f)], capture_output=True, timeout=120)
    assert a.returncode == 0 and b.returncode == 0, (a.stderr, b.stderr)
    assert a.stdout == b.stdout == _one_call(data)


def test_pipelined_host_encode_equals_device_encode():
    """starch_encode_host on pinned input >= 256 MiB takes the pipelined path
    (batches of chromosome units, H2D of the next batch on a copy stream while
    one encodes): the archive equals the device-resident encode byte for byte."""
    import ctypes
    import torch
    import starch_amd
    n = sum(starch_amd.gen_bed_sizes(0, 12_000_000))
    host = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    starch_amd.gen_bed(0, 12_000_000, into=ctypes.c_void_p(host.data_ptr()))
    assert n >= (256 << 20)
    c = starch_amd.Starch(0)
    dev = host.to("cuda")
    c.compress_device(dev.data_ptr(), n)
    want = c.archive()
    c.compress_host_ptr(host.data_ptr(), n)
    got = c.archive()
    assert got == want
    segs = c.segments()
    assert [nm.decode() for nm, _ in segs] == starch_amd.HG38
    assert c.stats()["n_lines"] == 12_000_000
    c.close()


def test_host_into_equals_device_encode():
    """starch_encode_host_into: the pipelined encode writes every finished
    batch's streams straight into the caller's host buffer while later batches
    encode; magic + streams + index equal the device-resident archive, a short
    buffer is refused, and a pageable / small input takes the one-copy path."""
    import ctypes
    import torch
    import starch_amd
    n = sum(starch_amd.gen_bed_sizes(0, 12_000_000, seed=3))
    host = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    starch_amd.gen_bed(0, 12_000_000, seed=3, into=ctypes.c_void_p(host.data_ptr()))
    c = starch_amd.Starch(0)
    dev = host.to("cuda")
    c.compress_device(dev.data_ptr(), n)
    want = c.archive()
    out = torch.zeros(len(want) + 4096, dtype=torch.uint8, pin_memory=True)
    for _ in range(2):
        k = c.compress_host_into(host.data_ptr(), n, out.data_ptr(), out.numel())
        assert k == len(want) and out[:k].numpy().tobytes() == want
    assert c.archive() == want
    with pytest.raises(starch_amd.StarchError):
        c.compress_host_into(host.data_ptr(), n, out.data_ptr(), len(want) // 2)
    small = bytes(host[:5_000_000].numpy())
    small = small[:small.rfind(b"\n") + 1]
    ref = c.compress(small)
    buf = ctypes.create_string_buffer(len(ref) + 64)
    sbuf = ctypes.create_string_buffer(small, len(small))
    k = c.compress_host_into(ctypes.addressof(sbuf), len(small), ctypes.addressof(buf), len(buf))
    assert buf.raw[:k] == ref
    c.close()


@pytest.mark.parametrize("lanes", ["1", "3"])
def test_pipelined_lanes_and_batches(lanes):
    """The lane count and batch count of the pipelined path change only the
    schedule: 1 and 3 lanes (subprocess, STARCH_LANES / STARCH_PIPE_BATCHES read
    at first use) give the device-resident archive."""
    env = dict(os.environ, STARCH_LANES=lanes, STARCH_PIPE_BATCHES="5")
    r = subprocess.run([sys.executable, "-c", _PIPE_SRC], cwd=ROOT, env=env, capture_output=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    assert r.stdout.decode().strip().endswith("same")


def test_pipelined_input_with_0xff_falls_back():
    """A 0xFF (EOF for the reference, hpp:181) inside a pipelined input: the
    batch that meets it abandons the pipeline and the one-copy path encodes
    the input -- archive == device encode (which stops at the 0xFF)."""
    import ctypes
    import torch
    import starch_amd
    n = sum(starch_amd.gen_bed_sizes(0, 12_000_000))
    host = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    starch_amd.gen_bed(0, 12_000_000, into=ctypes.c_void_p(host.data_ptr()))
    host[n // 2 + 12345] = 0xFF
    c = starch_amd.Starch(0)
    dev = host.to("cuda")
    c.compress_device(dev.data_ptr(), n)
    want = c.archive()
    c.compress_host_ptr(host.data_ptr(), n)
    assert c.archive() == want
    assert c.stats()["n_lines"] < 12_000_000
    c.close()


_PIPE_SRC = r'''
import ctypes, torch, starch_amd
n = sum(starch_amd.gen_bed_sizes(0, 12_000_000, seed=7))
host = torch.empty(n, dtype=torch.uint8, pin_memory=True)
starch_amd.gen_bed(0, 12_000_000, seed=7, into=ctypes.c_void_p(host.data_ptr()))
c = starch_amd.Starch(0)
dev = host.to("cuda")
c.compress_device(dev.data_ptr(), n)
want = c.archive()
c.compress_host_ptr(host.data_ptr(), n)
got = c.archive()
c.compress_host_ptr(host.data_ptr(), n)
again = c.archive()
c.close()
print("same" if got == want and again == want else "differ")
'''


@pytest.mark.parametrize("batch", [1 << 20, 3_000_000, 7_777_777])
def test_stream_inside_one_chromosome(batch):
    """A single chromosome run longer than a batch is not held whole: batches
    are cut at a complete line inside it and its bzip2 stream is encoded in
    pieces (complete blocks per batch, the rest of the text, the last partial
    byte and the combined CRC carried to the next piece).  The archive equals
    the one-call archive byte for byte."""
    import starch_amd
    data = starch_amd.gen_bed(0, 1_500_000, chroms=[0])
    ref = _one_call(data)
    got, st = _streamed(data, 1 << 20, batch)
    assert got == ref
    assert st["n_segments"] == 1
    assert st["input_bytes"] == len(data)


def test_stream_inside_chromosome_runs_and_revisits():
    """Pieces whose cuts fall inside long byte runs (RLE1 chunks of 255), a
    chromosome revisited later, lines that do not parse (stale values carried
    across an inside cut) and a multi-block tail."""
    import random
    rnd = random.Random(7)
    lines = []
    pos = 1000
    for i in range(60_000):
        pos += rnd.randrange(0, 50)
        rem = "\t" + "A" * rnd.choice([0, 3, 4, 5, 254, 255, 256, 600]) if i % 7 == 0 else ""
        if i % 501 == 0:
            lines.append("chr1\tx\t%d%s\n" % (pos + 5, rem))
        else:
            lines.append("chr1\t%d\t%d%s\n" % (pos, pos + rnd.randrange(1, 400), rem))
    data = "".join(lines).encode() + b"chr2\t5\t9\n" * 3000 + "".join(lines[:20_000]).encode()
    ref = _one_call(data)
    for piece, batch in ((1 << 16, 200_000), (12_345, 1_000_000), (1 << 20, 1)):
        got, _ = _streamed(data, piece, batch)
        assert got == ref, (piece, batch)


def test_stream_inside_chromosome_hold_knob():
    """STARCH_STREAM_HOLD=1 keeps the chromosome-boundary-only cuts (the same
    archive, one batch per chromosome run)."""
    import starch_amd
    data = starch_amd.gen_bed(0, 300_000, chroms=[0, 1])
    ref = _one_call(data)
    code = ("import sys; sys.path.insert(0, %r); import starch_amd\n"
            "d = starch_amd.gen_bed(0, 300_000, chroms=[0, 1])\n"
            "c = starch_amd.Starch(0)\n"
            "a = c.compress_stream([d[i:i + 65536] for i in range(0, len(d), 65536)], batch_bytes=1 << 20)\n"
            "sys.stdout.buffer.write(a)\n") % ROOT
    env = dict(os.environ, STARCH_STREAM_HOLD="1")
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, timeout=300, check=True).stdout
    assert out == ref


def test_stream_large_open_pieces_wait_for_their_copy():
    """Batches cut inside one large chromosome (the piece path, with a context
    line) must not be read by the encoder before their H2D copy on the copy
    stream has landed (starch_api.hip stream_encode waits on the batch's copy
    event before both paths).  chr1 of cfg2 (~190 MB) in 48 MiB pieces and
    64 MiB batches: every batch is an open piece whose copy is tens of MB."""
    import starch_amd
    data = starch_amd.gen_bed(0, 100_000_000, chroms=[0])
    ref = _one_call(data)
    for piece, batch in ((48 << 20, 64 << 20), (96 << 20, 32 << 20)):
        got, st = _streamed(data, piece, batch)
        assert got == ref, (piece, batch)
        assert st["n_segments"] == 1
