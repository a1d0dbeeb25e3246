"""Multi-GPU sharding through the real kernels on one MI355X: the input is
planned into chromosome units, LPT-sharded over 2 or 3 contexts ("virtual
shards" on device 0, each with its own HIP stream and host thread), and the
gathered archive must equal the one-context archive byte for byte
(SURVEY §4.4, §8e)."""
import subprocess

import pytest

from tests import corpus

pytestmark = pytest.mark.gpu


def _single(data, **kw):
    import starch_amd
    c = starch_amd.Starch(0)
    a = c.compress(data, **kw)
    c.close()
    return a


@pytest.mark.parametrize("nshards", [2, 3])
def test_virtual_shards_hg38_archive_identical(nshards):
    import starch_amd
    data = starch_amd.gen_bed(0, 2_000_000)
    ref = _single(data)
    ctxs = [starch_amd.Starch(0) for _ in range(nshards)]
    got = starch_amd.compress_multi(ctxs, data)
    assert got == ref
    segs = ctxs[0].segments()
    assert [n.decode() for n, _ in segs] == starch_amd.HG38
    assert sorted(s.unit for _, s in segs) == [s.unit for _, s in segs]
    for c in ctxs:
        c.close()


@pytest.mark.parametrize("seed", range(4))
def test_virtual_shards_quirky_inputs(seed):
    """Stale sscanf values across unit cuts, unsorted / revisited chromosomes,
    tab quirks, NUL bytes, an unterminated tail: still identical."""
    import starch_amd
    data = (corpus.fuzz_bed(seed, 3000) + corpus.multi_chrom_bed(5, 400, seed, "bed6") +
            corpus.parseable_fuzz_bed(seed, 2000) + b"chr9\tx\ty\nchr9\t1")
    ref = _single(data)
    for n in (2, 3):
        ctxs = [starch_amd.Starch(0) for _ in range(n)]
        assert starch_amd.compress_multi(ctxs, data) == ref, n
        for c in ctxs:
            c.close()


def test_encode_units_scattered_in_hbm():
    """starch_encode_units_device with units placed out of order and with gaps
    in HBM (the exact per-unit route): every stream equals the whole-input one."""
    import torch
    import starch_amd
    data = corpus.multi_chrom_bed(6, 3000, seed=2) + corpus.fuzz_bed(7, 500)
    ref_idx, ref_streams = starch_amd.parse_archive(_single(data))
    units = starch_amd.plan_units(data, 16)
    assert len(units) > 3
    buf = torch.zeros(len(data) + 4096 * len(units), dtype=torch.uint8)
    placed, pos = [], 0
    for u in reversed(units):                    # reverse placement, 4 KiB gaps
        buf[pos:pos + u.length] = torch.frombuffer(bytearray(data[u.offset:u.offset + u.length]), dtype=torch.uint8)
        placed.append(pos)
        pos += u.length + 4096
    placed = placed[::-1]
    dev = buf.to("cuda")
    c = starch_amd.Starch(0)
    dunits = [starch_amd.Unit(p, u.length, u.init_start, u.init_stop) for p, u in zip(placed, units)]
    c.encode_units_device(dev.data_ptr(), dunits, list(range(len(units))))
    blob = c.streams()
    segs = c.segments()
    assert len(segs) == len(ref_streams)
    for (name, s), meta, st in zip(segs, ref_idx["streams"], ref_streams):
        assert name.decode("latin-1") == meta["chromosome"]
        assert blob[s.stream_offset:s.stream_offset + s.stream_bytes] == st
    c.close()


def test_cli_devices_equals_single(tmp_path):
    import os
    import starch_amd
    exe = os.path.join(os.path.dirname(starch_amd.LIB_PATH), "starch3")
    data = starch_amd.gen_bed(1, 300_000)
    f = tmp_path / "in.bed"
    f.write_bytes(data)
    one = subprocess.run([exe, str(f)], capture_output=True, timeout=300)
    two = subprocess.run([exe, "--devices", "0,0", str(f)], capture_output=True, timeout=300)
    assert one.returncode == 0 and two.returncode == 0, (one.stderr, two.stderr)
    assert one.stdout == two.stdout == _single(data)
