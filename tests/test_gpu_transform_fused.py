"""The single-pass transform (k_tf_fused: 8 KiB tiles, LDS halo, decoupled
look-back) against the oracle on the shapes that exercise its edges: lines
across tile boundaries at every offset, 0xFF (EOF, hpp:181) in and around
tiles, a tile whose output or segment records overflow LDS (direct writes), a
text buffer that is too small (capacity retry), and the inputs it hands to the
two-pass path (lines longer than the halo, tiles of > 2048 lines, stale
sscanf values)."""
import random

import pytest

from tests import corpus, oracle_lib

pytestmark = pytest.mark.gpu

TILE = 8192


@pytest.fixture(scope="module")
def ctx():
    import starch_amd
    c = starch_amd.Starch(0)
    yield c
    c.close()


def _check(ctx, data):
    text, segs = ctx.transform(data)
    otext, osegs = oracle_lib.transform(data)
    assert text == otext
    assert segs == osegs


def test_lines_across_every_tile_offset(ctx):
    r = random.Random(3)
    for shift in range(0, 40, 3):
        lines, pos = ["x" * shift + "\t1\t2\n"], 0
        while sum(len(s) for s in lines) < 5 * TILE:
            pos += r.randint(0, 99)
            lines.append("chr%d\t%d\t%d\n" % (r.randint(1, 2), pos, pos + r.randint(1, 300)))
        _check(ctx, "".join(lines).encode())


@pytest.mark.parametrize("where", [0, 5, TILE - 1, TILE, TILE + 1, 3 * TILE - 700, 3 * TILE + 100, 6 * TILE - 2])
def test_ff_anywhere(ctx, where):
    base = bytearray(corpus.multi_chrom_bed(3, 900, seed=where % 17))
    assert len(base) > 6 * TILE
    base[where] = 0xFF
    _check(ctx, bytes(base))


def test_output_and_segments_overflow_lds(ctx):
    # alternating huge / tiny stops: deltas of 19 digits, output ~1.5x input per tile
    big = "".join("a\t1\t1000000000000000000\na\t1\t2\n" for _ in range(2000)).encode()
    _check(ctx, big)
    # a new segment on every line: > 64 segment records per tile
    _check(ctx, "".join("%s\t%d\t%d\n" % ("ab"[i & 1], i, i + 3) for i in range(9000)).encode())


def test_long_lines_and_dense_tiles_take_two_pass(ctx):
    r = random.Random(5)
    rem = "".join(r.choice("ACGT") for _ in range(3000))
    data = corpus.multi_chrom_bed(2, 600, seed=1) + ("chr9\t5\t9\t%s\n" % rem).encode() * 3 + \
        corpus.multi_chrom_bed(2, 600, seed=2)
    _check(ctx, data)
    _check(ctx, b"\n" * 20000 + corpus.multi_chrom_bed(2, 300, seed=3))
    _check(ctx, corpus.multi_chrom_bed(2, 3000, seed=4) + b"chr2\tx\t7\n" + corpus.multi_chrom_bed(1, 50, seed=5))


def test_unaligned_device_input(ctx):
    import torch
    data = corpus.multi_chrom_bed(4, 1500, seed=8, kind="bed6")
    want = ctx.compress(data)
    for off in (1, 3, 7, 13):
        buf = torch.zeros(len(data) + 64, dtype=torch.uint8)
        buf[off:off + len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8)
        dev = buf.to("cuda")
        ctx.compress_device(dev.data_ptr() + off, len(data))
        assert ctx.archive() == want, off


def test_repeated_calls_track_capacity(ctx):
    # a small-output input first (the text capacity follows the last ratio), then a large one
    _check(ctx, b"c\t1\t2\n" * 100000)
    _check(ctx, "".join("a\t1\t1000000000000000000\na\t1\t2\n" for _ in range(30000)).encode())
    _check(ctx, corpus.multi_chrom_bed(5, 2000, seed=9, kind="np"))
