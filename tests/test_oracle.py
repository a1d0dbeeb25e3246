"""Pins the CPU oracle (oracle/starch_oracle.c) before anything is checked
against it: reference transform goldens, bzip2's own KAT files, per-stream
goldens from the reference's vendored libbz2, and system libbz2 via Python."""
import bz2 as pybz2
import hashlib
import random

import pytest

from tests import corpus, golden_lib, oracle_lib


@pytest.mark.parametrize("case", golden_lib.transform_cases(), ids=lambda c: c[0])
def test_oracle_transform_matches_reference_goldens(case):
    name, data, segs = case
    _, got = oracle_lib.transform(data)
    assert len(got) == len(segs), name
    for (gchr, glines, gtext), (chr_, lines, content, sha, ln) in zip(got, segs):
        assert gchr == chr_
        assert glines == lines
        if content is not None:
            assert gtext == content
        else:
            assert len(gtext) == ln and hashlib.sha256(gtext).hexdigest() == sha


def test_oracle_transform_empty_and_tail_only():
    assert oracle_lib.transform(b"") == (b"", [])
    assert oracle_lib.transform(b"chr1\t1\t2") == (b"", [])


@pytest.mark.parametrize("kat", golden_lib.kat_files(), ids=lambda k: "sample%d" % k[0])
def test_oracle_bz2_known_answer_files(kat):
    level, data, stream = kat
    assert oracle_lib.bz2(data, level) == stream


@pytest.mark.parametrize("case", golden_lib.bz2_cases(include_large=True), ids=lambda c: c[0])
def test_oracle_bz2_matches_reference_libbz2_goldens(case):
    name, data, bs, stream, sha = case
    got = oracle_lib.bz2(data, bs)
    if stream is not None:
        assert got == stream
    else:
        assert hashlib.sha256(got).hexdigest() == sha


def test_oracle_bz2_matches_system_libbz2_level9():
    r = random.Random(3)
    for n in (0, 1, 7, 100, 5000, 70000):
        data = bytes(r.choice(b"0123456789\np-\t") for _ in range(n))
        assert oracle_lib.bz2(data, 9) == pybz2.compress(data, 9)


def test_oracle_bz2_fuzz_against_reference_lib():
    if oracle_lib.ref() is None:
        pytest.skip("oracle/_ref not built")
    r = random.Random(77)
    for i in range(60):
        kind = i % 4
        n = r.randint(0, 6000)
        if kind == 0:
            data = bytes(r.randrange(256) for _ in range(n))
        elif kind == 1:
            p = r.randint(1, 12)
            unit = bytes(r.choice(b"ab\n") for _ in range(p))
            data = unit * r.randint(1, 400)
        elif kind == 2:
            data = b"".join(bytes([r.randrange(3) + 97]) * r.choice([1, 3, 4, 5, 255, 256, 300]) for _ in range(r.randint(1, 40)))
        else:
            data = corpus.fuzz_bed(seed=i, nlines=40)
        bs = r.choice([1, 9])
        assert oracle_lib.bz2(data, bs) == oracle_lib.ref_bz2(data, bs), (i, kind, n)


def test_oracle_block_sort_is_a_correct_rotation_sort():
    r = random.Random(9)
    for _ in range(30):
        n = r.randint(1, 300)
        b = bytes(r.choice(b"abc") for _ in range(n))
        op, fmap = oracle_lib.block_sort(b)
        rots = [b[i:] + b[:i] for i in range(n)]
        assert [rots[i] for i in fmap] == sorted(rots)
        assert fmap[op] == 0


def test_oracle_crc():
    L = oracle_lib.lib()
    # CRC-32/BZIP2 check value of "123456789"
    assert L.oracle_crc32_bzip2(b"123456789", 9) == 0xFC891918


# ---- base counts (hpp:61-62 declared, never computed) --------
@pytest.mark.parametrize("bed,want", [
    # union of [10,20) [15,30) [40,45) = 25; sum of lengths 30
    (b"chr1\t10\t20\nchr1\t15\t30\nchr1\t40\t45\n", [(25, 30)]),
    # nested interval adds nothing unique
    (b"chr1\t0\t100\nchr1\t10\t20\nchr1\t50\t150\n", [(150, 210)]),
    # a new segment resets the running maximum
    (b"chr1\t0\t100\nchr2\t0\t100\nchr1\t50\t60\n", [(100, 100), (100, 100), (10, 10)]),
    # stale start (x does not parse): the line is [5, 12)
    (b"chr2\t5\t9\nchr2\tx\t12\n", [(7, 11)]),
    # stop < start: nonunique goes negative, unique adds nothing
    (b"chr1\t50\t40\nchr1\t60\t70\n", [(10, 0)]),
    # the unterminated tail and everything after 0xFF are not lines
    (b"chr1\t1\t3\nchr1\t2\t9", [(2, 2)]),
    (b"chr1\t1\t3\n\xffchr1\t2\t9\n", [(2, 2)]),
    (b"", []),
])
def test_oracle_base_counts_known(bed, want):
    from tests import oracle_lib
    assert oracle_lib.base_counts(bed) == want


def test_oracle_base_counts_match_interval_union():
    """For sorted BED the unique count is the size of the union of the
    intervals (checked against a set of covered positions)."""
    import random
    from tests import oracle_lib
    rng = random.Random(7)
    for _ in range(20):
        lines, pos = [], 0
        for _ in range(rng.randint(1, 60)):
            pos += rng.randint(0, 30)
            lines.append((pos, pos + rng.randint(1, 50)))
        bed = b"".join(b"chrR\t%d\t%d\n" % (a, b) for a, b in lines)
        cover = set()
        for a, b in lines:
            cover.update(range(a, b))
        assert oracle_lib.base_counts(bed) == [(len(cover), sum(b - a for a, b in lines))]
