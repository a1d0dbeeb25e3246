"""Shard planning on the CPU (starch_amd/csrc/shard.cpp through the C ABI):
units cut the input only where a chromosome segment starts, carry the sscanf
values current before them, and the per-unit transforms concatenate to the
whole input's (checked with the oracle's transform, which takes the same
initial values).  No GPU needed: planning, LPT and layout are host code."""
import random

import pytest

from tests import corpus, oracle_lib


def _corpora():
    out = [(n, d) for n, d in corpus.edge_cases()]
    out += [("fuzz%d" % s, corpus.fuzz_bed(s, 400)) for s in range(12)]
    out += [("pfuzz%d" % s, corpus.parseable_fuzz_bed(s, 2000)) for s in range(3)]
    out += [("multi24", corpus.multi_chrom_bed(24, 300, seed=3)), ("np8", corpus.multi_chrom_bed(8, 200, 4, "np"))]
    # stale values across a chromosome change: the first lines of chr2 do not parse
    out.append(("stale_across", b"chr1\t10\t20\nchr1\t30\t45\nchr2\tx\ty\nchr2\t-\t9\nchr3\t\t\nchr3\t5\t6\n"))
    # chromosomes revisited (unsorted) and a long run that needs galloping
    r = random.Random(9)
    big = []
    for c in ["chrA", "chrB", "chrA", "chrC", "chrB"]:
        pos = 0
        for _ in range(r.randint(3000, 9000)):
            pos += r.randint(0, 50)
            big.append("%s\t%d\t%d\n" % (c, pos, pos + r.randint(1, 90)))
    out.append(("unsorted_big", "".join(big).encode()))
    return out


def _segments_by_units(data, units):
    segs = []
    for u in units:
        _, s = oracle_lib.transform(data[u.offset:u.offset + u.length], u.init_start, u.init_stop)
        segs += s
    return segs


@pytest.mark.parametrize("name,data", _corpora(), ids=[n for n, _ in _corpora()])
@pytest.mark.parametrize("max_units", [1, 2, 3, 7, 64])
def test_units_concatenate_to_whole_input(name, data, max_units):
    import starch_amd
    units = starch_amd.plan_units(data, max_units)
    lim = data.find(b"\xff")
    lim = len(data) if lim < 0 else lim
    assert len(units) <= max_units
    pos = 0
    for u in units:                       # contiguous cover of [0, lim)
        assert u.offset == pos and u.length > 0
        pos += u.length
    assert pos == lim
    for u in units[1:]:                   # every cut is at a line start
        assert data[u.offset - 1:u.offset] == b"\n"
    _, whole = oracle_lib.transform(data)
    assert _segments_by_units(data, units) == whole


def test_units_follow_chromosomes_of_sorted_bed():
    import starch_amd
    data = corpus.multi_chrom_bed(24, 2000, seed=5)
    units = starch_amd.plan_units(data, 1000)
    _, whole = oracle_lib.transform(data)
    assert len(units) == len(whole) == 24
    for u, (chr_, _, _) in zip(units, whole):
        assert data[u.offset:].startswith(chr_ + b"\t")


def test_init_values_carry_stale_fields():
    import starch_amd
    data = b"chr1\t10\t20\nchr1\t30\t45\nchr2\tx\ty\nchr2\t-\t9\n"
    units = starch_amd.plan_units(data, 8)
    assert [(u.init_start, u.init_stop) for u in units] == [(0, 0), (30, 45)]


def test_lpt_balances_hg38_chromosomes():
    import starch_amd
    units = [starch_amd.Unit(0, L, 0, 0) for L in starch_amd.HG38_LEN]
    for n in (2, 4, 8):
        sh = starch_amd.assign_shards(units, n)
        load = [0] * n
        for u, s in zip(units, sh):
            load[s] += u.length
        assert max(load) <= 1.1 * sum(load) / n, (n, load)
    assert starch_amd.assign_shards(units, 1) == [0] * 24


def test_archive_layout_orders_by_unit():
    import starch_amd
    # two parts: rank 0 holds units 0 and 2, rank 1 holds unit 1 (two segments)
    unit_of = [0, 2, 1, 1]
    nbytes = [10, 30, 5, 7]
    order, off, end = starch_amd.archive_layout(unit_of, nbytes, base=4)
    assert order == [0, 2, 3, 1]
    assert off == [4, 26, 14, 19]
    assert end == 56
