"""GPU parity: the HIP path (through the C ABI) against the oracle and the
reference goldens.  Bit-exact everywhere (integer/byte work)."""
import bz2 as pybz2
import hashlib
import random

import pytest

from tests import corpus, golden_lib, oracle_lib

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    import starch_amd
    c = starch_amd.Starch(0)
    yield c
    c.close()


# ---------------------------------------------------------------- transform
@pytest.mark.parametrize("case", golden_lib.transform_cases(), ids=lambda c: c[0])
def test_transform_matches_reference_goldens(ctx, case):
    name, data, segs = case
    _, got = ctx.transform(data)
    assert len(got) == len(segs), name
    for (gchr, glines, gtext), (chr_, lines, content, sha, ln) in zip(got, segs):
        assert gchr == chr_ and glines == lines
        if content is not None:
            assert gtext == content
        else:
            assert len(gtext) == ln and hashlib.sha256(gtext).hexdigest() == sha


def test_transform_matches_oracle_fuzz(ctx):
    for seed in range(30):
        data = corpus.fuzz_bed(seed=50000 + seed, nlines=300)
        text, segs = ctx.transform(data)
        otext, osegs = oracle_lib.transform(data)
        assert text == otext
        assert segs == osegs


def test_transform_fused_path_fuzz(ctx):
    """All values parse: the fused two-pass kernels run, with fast (SWAR) and
    byte-serial lines mixed inside and across 256-line groups."""
    for seed in range(6):
        data = corpus.parseable_fuzz_bed(seed=7000 + seed, nlines=3000 + 97 * seed)
        text, segs = ctx.transform(data)
        otext, osegs = oracle_lib.transform(data)
        assert text == otext
        assert segs == osegs


def test_transform_empty_and_unterminated(ctx):
    assert ctx.transform(b"") == (b"", [])
    assert ctx.transform(b"chr1\t1\t2") == (b"", [])
    assert ctx.transform(b"\xff") == (b"", [])


def test_transform_generated_narrowpeak_and_bed3(ctx):
    import starch_amd
    for kind in (0, 1):
        data = starch_amd.gen_bed(kind, 200000, chroms=[0, 11, 23])
        text, segs = ctx.transform(data)
        otext, osegs = oracle_lib.transform(data)
        assert text == otext and segs == osegs


# ---------------------------------------------------------------- bzip2
@pytest.mark.parametrize("kat", golden_lib.kat_files(), ids=lambda k: "sample%d" % k[0])
def test_bz2_known_answer_files(ctx, kat):
    level, data, stream = kat
    assert ctx.bz2_compress(data, level) == stream


@pytest.mark.parametrize("case", golden_lib.bz2_cases(include_large=True), ids=lambda c: c[0])
def test_bz2_matches_reference_libbz2_goldens(ctx, case):
    name, data, bs, stream, sha = case
    got = ctx.bz2_compress(data, bs)
    if stream is not None:
        assert got == stream
    else:
        assert hashlib.sha256(got).hexdigest() == sha


def test_bz2_fuzz_vs_oracle(ctx):
    r = random.Random(1234)
    for i in range(40):
        kind = i % 4
        n = r.randint(0, 20000)
        if kind == 0:
            data = bytes(r.randrange(256) for _ in range(n))
        elif kind == 1:
            unit = bytes(r.choice(b"ab\n0") for _ in range(r.randint(1, 9)))
            data = unit * r.randint(1, 2000)
        elif kind == 2:
            data = b"".join(bytes([r.randrange(3) + 97]) * r.choice([1, 3, 4, 5, 255, 256, 300, 1000])
                            for _ in range(r.randint(1, 60)))
        else:
            data = corpus.fuzz_bed(seed=i, nlines=200)
        bs = r.choice([1, 9])
        assert ctx.bz2_compress(data, bs) == oracle_lib.bz2(data, bs), (i, kind, n, bs)


def test_bz2_runs_across_tiles_vs_oracle(ctx):
    """RLE1 run positions carried across 4 KiB tiles (k_rle_sum/k_rle_carry/
    k_rle_pos): runs longer than a tile, runs ending exactly at a tile edge,
    runs of 255k +- 1 bytes straddling edges, single-byte alternations."""
    r = random.Random(4321)
    cases = [b"a" * 4096, b"a" * 4097, b"a" * 12289 + b"b", b"x" * 4095 + b"yy" + b"x" * 4095,
             b"ab" * 5000, b"a" * (255 * 17 + 1) + b"b" * (255 * 3 - 1) + b"a" * 4]
    for _ in range(12):
        parts = []
        for _ in range(r.randint(1, 12)):
            parts.append(bytes([97 + r.randrange(3)]) * r.choice([1, 4, 254, 255, 256, 509, 510, 511, 4093, 4096, 9000]))
        cases.append(b"".join(parts))
    for data in cases:
        for bs in (1, 9):
            assert ctx.bz2_compress(data, bs) == oracle_lib.bz2(data, bs), (len(data), bs)


def test_bz2_many_streams_one_launch(ctx):
    import torch
    r = random.Random(99)
    pieces = [bytes(r.choice(b"0123456789\np-") for _ in range(r.randint(0, 5000))) for _ in range(64)]
    pieces[3] = b""
    pieces[7] = b"z" * 3000
    blob = b"".join(pieces)
    offs, lens, o = [], [], 0
    for p in pieces:
        offs.append(o); lens.append(len(p)); o += len(p)
    d_in = torch.frombuffer(bytearray(blob + b"\0" * 64), dtype=torch.uint8).cuda()
    cap = len(blob) * 2 + 64 * 100 + 4096
    d_out = torch.zeros(cap, dtype=torch.uint8, device="cuda")
    oo, ol = ctx.bz2_compress_many_device(d_in.data_ptr(), offs, lens, 9, d_out.data_ptr(), cap)
    out = d_out.cpu().numpy().tobytes()
    for p, a, n in zip(pieces, oo, ol):
        assert out[a:a + n] == pybz2.compress(p, 9)


# ---------------------------------------------------------------- archive
def _check_archive(arch, data, note=None, level=9):
    import starch_amd
    idx, streams = starch_amd.parse_archive(arch)
    _, osegs = oracle_lib.transform(data)
    assert len(streams) == len(osegs)
    for st, (chr_, lines, text), meta in zip(streams, osegs, idx["streams"]):
        assert meta["chromosome"].encode("latin-1") == chr_
        assert meta["uncompressedLineCount"] == lines
        assert meta["transformedBytes"] == len(text)
        assert st == oracle_lib.bz2(text, level)
        assert pybz2.decompress(st) == text
    if note:
        assert idx["archive"]["note"] == note


@pytest.mark.parametrize("gen", sorted(corpus.TRANSFORM_GENERATORS), ids=str)
def test_archive_end_to_end(ctx, gen):
    data = corpus.TRANSFORM_GENERATORS[gen]()
    arch = ctx.compress(data)
    _check_archive(arch, data)


def test_archive_edge_inputs(ctx):
    for name, data in corpus.edge_cases():
        _check_archive(ctx.compress(data), data)
    arch = ctx.compress(b"")
    assert arch[:4] == b"\xca\x5c\xad\x1a"
    idx, streams = __import__("starch_amd").parse_archive(arch)
    assert streams == []


def test_archive_note_and_level(ctx):
    data = corpus.multi_chrom_bed(3, 300, seed=3)
    ctx.set_note("hello \"world\"\té")
    ctx.block_size_100k = 1
    try:
        arch = ctx.compress(data)
        _check_archive(arch, data, note="hello \"world\"\té", level=1)
    finally:
        ctx.set_note("")
        ctx.block_size_100k = 9


def test_reference_compat_is_magic_only(ctx):
    assert ctx.compress(corpus.cfg1_bed(100), reference_compat=True) == b"\xca\x5c\xad\x1a"


def test_cfg1_sizes(ctx):
    data = corpus.cfg1_bed(10000)
    arch = ctx.compress(data)
    idx, streams = __import__("starch_amd").parse_archive(arch)
    assert len(data) == 187819
    assert idx["streams"][0]["transformedBytes"] == 91757
    assert len(streams[0]) == len(pybz2.compress(oracle_lib.transform(data)[1][0][2], 9))
