"""GPU decompression and unstarch, through the C ABI.

bzip2 decoding is checked against bzip2's own known-answer files
(tests/golden/kat/sample{1,2,3}.bz2, decoded by the system libbz2 through
Python's bz2 -- a library oracle, bz:decompress.c), streams from this
library's encoder (whose bytes the reference's libbz2 pins elsewhere), and
streams from Python's bz2 at several levels; every block CRC and stream CRC is
checked by the decoder.  The inverse transform is checked against the
oracle's restatement (oracle_untransform, itself pinned by round trips in
test_untransform_oracle.py) and by archive round trips:
unstarch(compress(bed)) == bed for canonical BED."""
import bz2 as pybz2
import os
import random

import pytest

from tests import corpus, oracle_lib
from tests.test_untransform_oracle import _bed

KAT = os.path.join(os.path.dirname(__file__), "golden", "kat")


@pytest.fixture(scope="module")
def ctx():
    import starch_amd
    c = starch_amd.Starch(0)
    yield c
    c.close()


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["sample1.bz2", "sample2.bz2", "sample3.bz2"])
def test_decode_kat(ctx, name):
    data = open(os.path.join(KAT, name), "rb").read()
    assert ctx.bz2_decompress(data) == pybz2.decompress(data)


def _inputs():
    rng = random.Random(7)
    yield "empty", b""
    yield "one", b"x"
    yield "runs", b"a" * 1000 + b"b" * 3 + b"c" * 4 + b"d" * 5 + b"e" * 255 + b"f" * 256 + b"g" * 260
    yield "random", bytes(rng.randrange(256) for _ in range(300_000))
    yield "small_alpha", bytes(rng.choice(b"ACGT\n") for _ in range(400_000))
    yield "periodic", b"0\n" * 500_000
    yield "text", corpus.multi_chrom_bed(2, 30_000, 5)


@pytest.mark.gpu
@pytest.mark.parametrize("level", [1, 9])
@pytest.mark.parametrize("name,data", list(_inputs()), ids=[n for n, _ in _inputs()])
def test_decode_own_and_system_streams(ctx, name, data, level):
    own = ctx.bz2_compress(data, level)
    assert ctx.bz2_decompress(own) == data
    sysb = pybz2.compress(data, level)
    assert ctx.bz2_decompress(sysb) == data
    st = ctx.decoded_streams()
    assert len(st) == 1 and st[0]["level"] == level and st[0]["out_len"] == len(data)


@pytest.mark.gpu
def test_decode_concatenated_streams(ctx):
    parts = [b"alpha\n" * 1000, b"", bytes(range(256)) * 5000, b"z" * 2_000_000]
    blob = b"".join(pybz2.compress(p, 1 + k % 9) for k, p in enumerate(parts))
    assert ctx.bz2_decompress(blob) == b"".join(parts)
    st = ctx.decoded_streams()
    assert [s["out_len"] for s in st] == [len(p) for p in parts]
    assert st[2]["n_blocks"] > 1 and st[1]["n_blocks"] == 0


@pytest.mark.gpu
def test_decode_rejects_corruption(ctx):
    import starch_amd
    data = bytes(random.Random(3).randrange(256) for _ in range(200_000))
    z = bytearray(pybz2.compress(data, 9))
    z[len(z) // 2] ^= 0x20
    with pytest.raises(starch_amd.StarchError) as e:
        ctx.bz2_decompress(bytes(z))
    assert e.value.code == -12
    with pytest.raises(starch_amd.StarchError):
        ctx.bz2_decompress(b"BZh9 not a stream")


@pytest.mark.gpu
@pytest.mark.parametrize("seed,rem", [(11, False), (12, True)])
def test_untransform_matches_oracle(ctx, seed, rem):
    bed = _bed(random.Random(seed), 2, 20_000, rem=rem)
    text, segs = oracle_lib.transform(bed)
    for chr_, _, t in segs:
        want = oracle_lib.untransform(t, chr_)
        assert want is not None
        assert ctx.untransform(t, chr_) == want


@pytest.mark.gpu
def test_untransform_refuses_negative_p(ctx):
    import starch_amd
    text, segs = oracle_lib.transform(b"chr1\t10\t5\nchr1\t20\t30\n")
    with pytest.raises(starch_amd.StarchError) as e:
        ctx.untransform(segs[0][2], b"chr1")
    assert e.value.code == -12


@pytest.mark.gpu
def test_unstarch_round_trip_generated(ctx):
    import starch_amd
    bed = starch_amd.gen_bed(0, 2_000_000)
    arch = ctx.compress(bed)
    assert ctx.unstarch(arch) == bed


@pytest.mark.gpu
def test_unstarch_round_trip_narrowpeak_and_revisits(ctx):
    import starch_amd
    bed = starch_amd.gen_bed(1, 300_000)
    # a revisited chromosome starts a new segment (hpp:331)
    bed = bed + b"chr1\t5\t10\tx\n"
    arch = ctx.compress(bed)
    assert ctx.unstarch(arch) == bed
