"""MTF/RUNA-RUNB (bz:compress.c:119-231) across the alphabet-size paths: <= 16
symbols (nibble lists), 17..32 (byte lists in registers), > 32 (LDS lists),
each against the reference libbz2 stream, including runs of zeros that cross
512-symbol chunks and multi-block inputs."""
import random

import pytest

from tests import oracle_lib

pytestmark = pytest.mark.gpu


def _ref(data, bs=9):
    return oracle_lib.ref_bz2(data, bs) if oracle_lib.ref() is not None else oracle_lib.bz2(data, bs)


@pytest.fixture(scope="module")
def ctx():
    import starch_amd
    c = starch_amd.Starch(0)
    yield c
    c.close()


@pytest.mark.parametrize("nsym", [2, 15, 16, 17, 18, 24, 31, 32, 33, 40, 200])
def test_alphabet_sizes(ctx, nsym):
    r = random.Random(nsym)
    alpha = bytes(r.sample(range(256), nsym))
    out = bytearray()
    while len(out) < 300_000:
        k = r.random()
        if k < 0.2:
            out += bytes([r.choice(alpha)]) * r.randint(1, 3000)     # long runs: zero runs across chunks
        elif k < 0.5:
            w = bytes(r.choice(alpha) for _ in range(r.randint(2, 12)))
            out += w * r.randint(1, 40)
        else:
            out += bytes(r.choice(alpha) for _ in range(r.randint(1, 200)))
    data = bytes(out)
    assert ctx.bz2_compress(data, 9) == _ref(data, 9)
    assert ctx.bz2_compress(data[:150_000], 1) == _ref(data[:150_000], 1)


@pytest.mark.parametrize("nsym", [16, 17, 23, 24, 25, 26, 29, 30, 31, 32])
def test_alphabet_edges_without_runs(ctx, nsym):
    """No run of 4 (no RLE1 count bytes): nInUse is exactly nsym, at the
    boundaries between the nibble lists (<= 16), the three- and four-word
    byte lists (<= 24, <= 30) and the LDS path."""
    r = random.Random(100 + nsym)
    alpha = list(range(65, 65 + nsym))
    out, prev = [], None
    while len(out) < 200_000:
        c = r.choice(alpha)
        if c == prev:
            continue
        out.append(c)
        prev = c
    data = bytes(out)
    assert ctx.bz2_compress(data, 9) == _ref(data, 9)


def test_narrowpeak_text_multiblock(ctx):
    import starch_amd
    data = starch_amd.gen_bed(1, 300_000, chroms=[13])
    text, segs = ctx.transform(data)
    assert ctx.bz2_compress(segs[0][2], 9) == _ref(segs[0][2], 9)


def test_mixed_alphabet_classes_in_one_batch(ctx):
    """Blocks of every alphabet class in one stream (one sort / MTF batch):
    the batch launches each class's kernels once, every block takes its own."""
    r = random.Random(7)
    out = bytearray()
    for nsym in (10, 22, 28, 45, 12, 20):
        alpha = list(range(40, 40 + nsym))
        prev = None
        part = []
        while len(part) < 120_000:
            c = r.choice(alpha)
            if c == prev:
                continue
            part.append(c)
            prev = c
        out += bytes(part)
    data = bytes(out)
    assert ctx.bz2_compress(data, 1) == _ref(data, 1)       # 100 KB blocks: one class each, mostly
    assert ctx.bz2_compress(data, 9) == _ref(data, 9)
