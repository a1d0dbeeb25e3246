"""CPU: the oracle's inverse transform (oracle_untransform) is
pinned by round trips through the forward restatement, which the reference
binary's own transform goldens pin (test_oracle.py): for canonical sorted BED
(decimal coordinates, stop >= start) untransform(transform(bed)) == bed per
chromosome segment; a negative p-value (the forward drops its newline,
hpp:440,452) is refused."""
import random

import pytest

from tests import oracle_lib


def _bed(rng, nchr, nlines, rem=False, maxlen=500):
    out = []
    for c in range(nchr):
        pos = rng.randrange(0, 10000)
        for _ in range(nlines):
            pos += rng.randrange(0, 300)
            a = pos
            b = a + rng.randrange(0, maxlen)
            line = b"chr%d\t%d\t%d" % (c + 1, a, b)
            if rem:
                line += b"\tpeak%d\t%d\t.\t%.5f" % (rng.randrange(100000), rng.randrange(1001), rng.random() * 100)
            out.append(line + b"\n")
    return b"".join(out)


@pytest.mark.parametrize("seed,rem", [(1, False), (2, True), (3, False), (4, True)])
def test_oracle_untransform_round_trip(seed, rem):
    rng = random.Random(seed)
    bed = _bed(rng, 3, 2000, rem=rem)
    text, segs = oracle_lib.transform(bed)
    back = b"".join(oracle_lib.untransform(t, chr_) for chr_, _, t in segs)
    assert back == bed


def test_oracle_untransform_edges():
    # zero-length intervals, interval at 0, equal starts, a revisited chromosome
    bed = (b"chr1\t0\t0\nchr1\t0\t5\nchr1\t0\t5\nchr1\t7\t7\tx\ty\n"
           b"chr2\t100\t200\nchr1\t1\t2\n")
    text, segs = oracle_lib.transform(bed)
    assert len(segs) == 3
    assert b"".join(oracle_lib.untransform(t, c) for c, _, t in segs) == bed


def test_oracle_untransform_refuses_negative_p():
    text, segs = oracle_lib.transform(b"chr1\t10\t5\nchr1\t20\t30\n")
    assert oracle_lib.untransform(segs[0][2], b"chr1") is None
    assert oracle_lib.untransform(b"12\n7", b"chr1") is None          # last line without its newline
    assert oracle_lib.untransform(b"p\n", b"chr1") is None
