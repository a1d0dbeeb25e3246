"""GPU block sort stress: full 900 KB blocks whose rotations stress every path
of the batch-wide sort (bz2_bwt3.hip) -- tie groups resolved by doubling,
huge equal-key groups, periodic blocks, every key width (2..256 symbols).
Checked byte-for-byte against the CPU oracle's bzip2 -N stream (fallbackSort
order), which the reference's own libbz2 pins (test_oracle.py)."""
import random

import pytest

from tests import oracle_lib

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    import starch_amd
    c = starch_amd.Starch(0)
    yield c
    c.close()


def _bed_text(kind, lines, chroms):
    import starch_amd
    data = starch_amd.gen_bed(kind, lines, chroms=chroms)
    _, segs = oracle_lib.transform(bytes(data))
    return b"".join(t for _, _, t in segs)


def _cases():
    r = random.Random(77)
    yield "cfg2_text", lambda: _bed_text(0, 12_000_000, [20])[:2_000_000]
    yield "cfg4_text", lambda: _bed_text(1, 6_000_000, [20])[:2_000_000]
    yield "near_periodic", lambda: b"p1\n7\n" + b"0\n" * 440_000 + b"x"
    yield "periodic", lambda: b"0\n" * 450_000
    yield "period3_break", lambda: (b"abc" * 300_000)[:-1] + b"d"
    yield "binary", lambda: bytes(r.choice(b"ab") for _ in range(900_000))
    yield "bytes256", lambda: bytes(r.randrange(256) for _ in range(900_000))
    yield "runs", lambda: b"".join(bytes([r.randrange(4) + 48]) * r.choice([1, 2, 4, 7, 300])
                                   for _ in range(20_000))
    yield "long_repeat_two", lambda: (lambda u: u * 2 + b"!")(bytes(r.randrange(5) + 65 for _ in range(400_000)))
    yield "digits_lowentropy", lambda: bytes(r.choice(b"0000000001\n") for _ in range(1_000_000))


@pytest.mark.parametrize("name,make", list(_cases()), ids=lambda x: x if isinstance(x, str) else "")
def test_bwt_full_blocks_vs_oracle(ctx, name, make):
    data = make()
    for bs in (9, 1):
        assert ctx.bz2_compress(data, bs) == oracle_lib.bz2(data, bs), (name, bs)


def test_bwt_tiny_blocks(ctx):
    for data in (b"a", b"ab", b"ba", b"aa", b"aba", b"abab", b"\x00\xff", bytes(range(256)), b"z" * 5):
        assert ctx.bz2_compress(data, 9) == oracle_lib.bz2(data, 9), data[:8]
