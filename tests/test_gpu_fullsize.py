"""Full-size parity (north_star's target): every one of the 24 chromosome
streams of cfg2 (100 M-line hg38 BED3) and cfg4 (50 M-row narrowPeak) equals
the CPU path's stream -- the oracle transform followed by the reference's own
libbz2 1.0.6 at -9 -- by SHA-256 (tests/golden/fullsize_cfg*.json, made in the
CPU container by tools/make_fullsize_goldens.py)."""
import hashlib
import json
import os

import pytest

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.mark.parametrize("cfg", ["cfg2", "cfg4"])
def test_fullsize_streams_match_cpu_path(cfg):
    import torch
    import starch_amd
    g = json.load(open(os.path.join(GOLDEN, "fullsize_%s.json" % cfg)))
    n = sum(starch_amd.gen_bed_sizes(g["kind"], g["total_lines"], seed=g["seed"]))
    assert n == g["input_bytes"]
    host = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    import ctypes
    starch_amd.gen_bed(g["kind"], g["total_lines"], seed=g["seed"], into=ctypes.c_void_p(host.data_ptr()))
    dev = host.to("cuda")
    del host
    c = starch_amd.Starch(0)
    c.compress_device(dev.data_ptr(), n)
    idx, streams = starch_amd.parse_archive(c.archive())
    assert len(streams) == 24
    for st, meta, want in zip(streams, idx["streams"], g["streams"]):
        assert meta["chromosome"] == want["chromosome"]
        assert meta["uncompressedLineCount"] == want["lines"]
        assert meta["transformedBytes"] == want["text_bytes"]
        assert len(st) == want["stream_bytes"], want["chromosome"]
        assert hashlib.sha256(st).hexdigest() == want["sha256"], want["chromosome"]
    c.close()


@pytest.mark.parametrize("cfg", ["cfg2", "cfg4"])
def test_fullsize_unstarch_round_trip(cfg):
    """unstarch(archive) == input at the full configs (decode ->
    inverse transform on the GPU; a size-independent property)."""
    import ctypes
    import time
    import torch
    import starch_amd
    g = json.load(open(os.path.join(GOLDEN, "fullsize_%s.json" % cfg)))
    n = g["input_bytes"]
    host = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    starch_amd.gen_bed(g["kind"], g["total_lines"], seed=g["seed"], into=ctypes.c_void_p(host.data_ptr()))
    c = starch_amd.Starch(0)
    c.compress_host_ptr(host.data_ptr(), n)
    arch = c.archive()
    t0 = time.perf_counter()
    back = c.unstarch(arch)
    dt = time.perf_counter() - t0
    print("[unstarch %s] %.1f MB archive -> %.1f MB BED in %.3f s (host-to-host)" % (cfg, len(arch) / 1e6, n / 1e6, dt))
    assert len(back) == n
    assert torch.equal(torch.frombuffer(bytearray(back), dtype=torch.uint8), host)
    c.close()


def test_cfg5_all_24_fullsize():
    """cfg5 (per-position BED, every base of hg38: 3.09 G lines, 73.6 GB) at
    full size, all 24 chromosomes: each chromosome's input is generated in HBM
    by the GPU (starch_gen_perpos_device, the same bytes as starch_gen_bed
    kind 2) and encoded; every stream's SHA-256 equals the CPU path's
    (tests/golden/fullsize_cfg5.json), and the byte-identical "0\\n" blocks
    are sorted once (exact block reuse: a handful of distinct blocks per
    stream -- the BWT of bz:blocksort.c:1031-1089 is a pure function of the
    block bytes)."""
    import torch
    import starch_amd
    g = json.load(open(os.path.join(GOLDEN, "fullsize_cfg5.json")))
    want = {s["chromosome"]: s for s in g["streams"]}
    assert len(want) == 24
    cap = max(starch_amd.gen_perpos_device(c) for c in range(24))
    dev = torch.empty(cap + 64, dtype=torch.uint8, device="cuda")
    c = starch_amd.Starch(0)
    stream = torch.cuda.Stream()          # a non-default stream: generator and encoder ordered on it
    c.set_stream(stream.cuda_stream)
    done = 0
    for ci, name in enumerate(starch_amd.HG38):
        n = starch_amd.gen_perpos_device(ci, dev.data_ptr(), cap + 64, stream=stream.cuda_stream)
        w = want[name]
        assert n == w["input_bytes"], name
        c.compress_device(dev.data_ptr(), n)
        st = c.stats()
        idx, streams = starch_amd.parse_archive(c.archive())
        assert [m["chromosome"] for m in idx["streams"]] == [name]
        meta, s = idx["streams"][0], streams[0]
        assert meta["uncompressedLineCount"] == w["lines"]
        assert meta["transformedBytes"] == w["text_bytes"]
        assert len(s) == w["stream_bytes"], name
        assert hashlib.sha256(s).hexdigest() == w["sha256"], name
        assert st["n_blocks"] == meta["blocks"]
        assert st["n_blocks"] - st["dedup_blocks"] <= 4, (name, st["n_blocks"], st["dedup_blocks"])
        done += 1
    assert done == 24
    c.close()


def test_null_stream_orders_input_before_encode():
    """set_stream(0) is the HIP null stream (include/starch_amd.h): input written
    there -- the GPU generator, then torch's default stream (also the null
    stream) overwriting a prefix -- is ordered before the encode with no host
    synchronisation in between.  This is the race of a generator on the null
    stream and an encoder on the context's own stream ("split chr11").  chrY's
    1.29 GB per-position input must give the CPU path's stream."""
    import torch
    import starch_amd
    g = json.load(open(os.path.join(GOLDEN, "fullsize_cfg5.json")))
    w = {s["chromosome"]: s for s in g["streams"]}["chrY"]
    ci = starch_amd.HG38.index("chrY")
    n = starch_amd.gen_perpos_device(ci)
    dev = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    c = starch_amd.Starch(0)
    c.set_stream(0)
    for rep in range(2):
        torch.cuda.synchronize()
        dev.fill_(0x41)                    # garbage the encoder must never see
        got = starch_amd.gen_perpos_device(ci, dev.data_ptr(), n + 64, stream=0)
        assert got == n == w["input_bytes"]
        if rep == 1:
            # torch's default stream is the null stream: rewrite the first 64 MiB
            # there (same bytes) right before the encode
            assert torch.cuda.current_stream().cuda_stream == 0
            head = dev[:64 << 20].clone()
            dev[:64 << 20].fill_(0x42)
            dev[:64 << 20].copy_(head)
        c.compress_device(dev.data_ptr(), n)
        idx, streams = starch_amd.parse_archive(c.archive())
        assert [m["chromosome"] for m in idx["streams"]] == ["chrY"]
        assert len(streams[0]) == w["stream_bytes"]
        assert hashlib.sha256(streams[0]).hexdigest() == w["sha256"]
    c.use_own_stream()
    c.close()
