"""The gzip method (-g).  The reference declares it
(starch3api.hpp:23-27, src/starch3.cpp:84,124) but exits ENOSYS when it is
chosen (hpp:777-779), so there is no reference output to pin: parity is
unpinned, and the contract tested here is that every segment's member is a
valid RFC 1952 gzip member (any zlib inflates it, CRC-32 and ISIZE included)
whose content is exactly the segment's transformed text as the oracle
restates it, that the index names the method, and that the archive does not
depend on the entry point (one call, streaming, virtual shards, the CLI)."""
import gzip
import os
import random
import subprocess
import zlib

import pytest

from tests import corpus, oracle_lib

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def ctx():
    import starch_amd
    c = starch_amd.Starch(0)
    c.set_compression_method(starch_amd.K_GZIP)
    yield c
    c.close()


def _check(arch, data):
    import starch_amd
    idx, members = starch_amd.parse_archive(arch)
    assert idx["archive"]["compressionFormat"] == "gzip"
    _, osegs = oracle_lib.transform(data)
    assert len(members) == len(osegs)
    for m, meta, (chr_, lines, text) in zip(members, idx["streams"], osegs):
        assert meta["chromosome"].encode("latin-1") == chr_ and meta["uncompressedLineCount"] == lines
        assert m[:3] == b"\x1f\x8b\x08"
        assert gzip.decompress(m) == text
        assert meta["combinedCRC"] == zlib.crc32(text)
    return members


def _cases():
    r = random.Random(3)
    yield "cfg1", corpus.cfg1_bed(10000)
    yield "multi", corpus.multi_chrom_bed(5, 3000, seed=4, kind="bed6")
    yield "fuzz", corpus.parseable_fuzz_bed(7, 4000)
    # long runs in the text: 258-byte matches, overlapping distance-1 copies
    yield "runs", b"".join(b"chrR\t%d\t%d\t%s\n" % (i, i + 1, b"A" * r.choice([1, 300, 5000])) for i in range(200))
    # bytes >= 144 as literals (9-bit codes) and no repeats
    yield "highbytes", b"".join(b"chrH\t%d\t%d\t%s\n" % (i, i + 5, bytes(r.randrange(128, 256) for _ in range(40)))
                                for i in range(2000))
    yield "one_line", b"chr1\t10\t20\n"


@pytest.mark.parametrize("name,data", list(_cases()), ids=lambda x: x if isinstance(x, str) else "")
def test_gzip_members_inflate_to_transform(ctx, name, data):
    _check(ctx.compress(data), data)


def test_gzip_generated_hg38(ctx):
    import starch_amd
    data = bytes(starch_amd.gen_bed(0, 600_000))
    arch = ctx.compress(data)
    members = _check(arch, data)
    # fixed-Huffman LZ77 over 4 KiB blocks: BED text compresses to well under half
    assert sum(len(m) for m in members) < 0.5 * sum(len(t) for _, _, t in oracle_lib.transform(data)[1])


def test_gzip_stream_identical(ctx):
    import starch_amd
    data = bytes(starch_amd.gen_bed(1, 100_000, chroms=[0, 5, 21]))
    one = ctx.compress(data)
    pieces = [data[i:i + 1_000_003] for i in range(0, len(data), 1_000_003)]
    assert ctx.compress_stream(pieces, batch_bytes=4 << 20) == one
    _check(one, data)


def test_cli_gzip(tmp_path):
    import starch_amd
    data = corpus.multi_chrom_bed(3, 2000, seed=9, kind="bed3")
    f = tmp_path / "in.bed"
    f.write_bytes(data)
    cli = os.path.join(ROOT, "starch_amd", "_build", "starch3")
    r = subprocess.run([cli, "-g", str(f)], capture_output=True, timeout=120)
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    c = starch_amd.Starch(0)
    c.set_compression_method(starch_amd.K_GZIP)
    assert r.stdout == c.compress(data)
    c.close()
    _check(r.stdout, data)
