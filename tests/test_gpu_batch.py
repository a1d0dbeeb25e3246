"""Block-sort batches after the first: the encoder sorts the
distinct blocks in batches sized by free HBM (bz2_encoder.hip); every test
input fits one batch, so STARCH_BWT_BATCH caps it in a child process and the
archive must equal the one-batch archive byte for byte (per-batch scratch
reuse, k_tables32's batch-relative indexing, the host block-descriptor round
trips).  Reference behaviour: each block's stream bytes depend on that block
alone (bz:compress.c:602-667)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = ("import sys; sys.path.insert(0, %r); import starch_amd; "
         "d = open(sys.argv[1], 'rb').read(); c = starch_amd.Starch(0); "
         "sys.stdout.buffer.write(c.compress(d)); c.close()" % ROOT)


@pytest.mark.gpu
@pytest.mark.parametrize("cap", [1, 3])
def test_small_bwt_batches_bit_identical(tmp_path, cap):
    import starch_amd
    data = starch_amd.gen_bed(0, 600_000)
    c = starch_amd.Starch(0)
    arch = c.compress(data)
    nb = c.stats()["n_blocks"]
    c.close()
    assert nb > 2 * cap
    f = tmp_path / "in.bed"
    f.write_bytes(data)
    env = dict(os.environ, STARCH_BWT_BATCH=str(cap))
    out = subprocess.run([sys.executable, "-c", CHILD, str(f)], env=env, capture_output=True, timeout=300)
    assert out.returncode == 0, out.stderr.decode()[-2000:]
    assert out.stdout == arch


@pytest.mark.gpu
def test_wide_top_digit_bit_identical(tmp_path):
    """Blocks of 17..20 symbols (narrowPeak text) sort with the 8192-bin
    mixed-radix top-level digit (bz2_bwt3.hip top_digit); STARCH_WIDE=0 forces
    the binary 12-bit digit.  Any exact sort gives bzip2's order, so both must
    produce the same archive, also for a batch mixing 17..20-symbol blocks with
    smaller and larger alphabets."""
    import random

    import starch_amd
    from tests import oracle_lib
    r = random.Random(5)
    wide = starch_amd.gen_bed(1, 300_000, chroms=[20, 21])
    odd = b"".join(b"chrZ\t%d\t%d\t%s\n" % (i * 10, i * 10 + 5, bytes(r.choice(b"ABCDEFGHIJKLMNOPQRSTUVWXYZ")
                                                                     for _ in range(8)))
                   for i in range(30_000))
    data = bytes(wide) + starch_amd.gen_bed(0, 200_000, chroms=[22]) + odd
    c = starch_amd.Starch(0)
    arch = c.compress(data)
    c.close()
    idx, streams = starch_amd.parse_archive(arch)
    _, osegs = oracle_lib.transform(data)
    assert len(streams) == len(osegs)
    for st, (_, _, text) in zip(streams, osegs):
        assert st == oracle_lib.bz2(text, 9)
    f = tmp_path / "in.bed"
    f.write_bytes(data)
    env = dict(os.environ, STARCH_WIDE="0")
    out = subprocess.run([sys.executable, "-c", CHILD, str(f)], env=env, capture_output=True, timeout=300)
    assert out.returncode == 0, out.stderr.decode()[-2000:]
    assert out.stdout == arch


@pytest.mark.gpu
def test_alternate_lsd_block_sort_bit_identical(tmp_path):
    """STARCH_BWT=lsd selects the independent one-workgroup-per-block
    prefix-doubling sort (bz2_bwt.hip k_bwt): it must give
    the default sort's archive byte for byte -- BED3 and narrowPeak blocks, a
    periodic block (fallbackSort tie order) and long repeats."""
    import starch_amd
    data = (bytes(starch_amd.gen_bed(0, 200_000, chroms=[3, 20])) + bytes(starch_amd.gen_bed(1, 60_000, chroms=[21]))
            + b"".join(b"chrP\t%d\t%d\n" % (i, i + 1) for i in range(200_000)))
    c = starch_amd.Starch(0)
    arch = c.compress(data)
    c.close()
    f = tmp_path / "in.bed"
    f.write_bytes(data)
    env = dict(os.environ, STARCH_BWT="lsd")
    out = subprocess.run([sys.executable, "-c", CHILD, str(f)], env=env, capture_output=True, timeout=300)
    assert out.returncode == 0, out.stderr.decode()[-2000:]
    assert out.stdout == arch
