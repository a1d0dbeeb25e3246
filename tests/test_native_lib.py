"""CPU-side checks of the native library: it builds, loads, exports every
symbol its headers declare, and its host-only helpers behave."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "starch_amd", "_build", "libstarch_amd.so")


def _declared(header):
    src = open(os.path.join(ROOT, "include", header)).read()
    return sorted(set(re.findall(r"^\s*(?:int|void|const char\*|uint64_t)\s*\**\s*(\w+)\s*\(", src, re.M)))


def _exported():
    out = subprocess.check_output(["nm", "-D", "--defined-only", LIB]).decode()
    return {l.split()[-1] for l in out.splitlines() if " T " in l}


@pytest.mark.parametrize("header", ["starch_amd.h", "starch_bzlib.h"])
def test_library_exports_every_declared_symbol(header):
    assert os.path.exists(LIB)
    names = _declared(header)
    exp = _exported()
    missing = [n for n in names if n not in exp]
    assert not missing, missing


def test_library_loads_and_reports_no_device_here():
    import starch_amd
    L = starch_amd.load()
    assert L.starch_version() == 0x000100
    try:
        import torch
        has_gpu = torch.cuda.is_available()
    except Exception:
        has_gpu = False
    if not has_gpu:
        with pytest.raises(starch_amd.StarchError):
            starch_amd.Starch(0)


def test_gen_bed_deterministic_and_sorted():
    import starch_amd
    a = starch_amd.gen_bed(0, 20000, chroms=[0, 1])
    b = starch_amd.gen_bed(0, 20000, chroms=[0, 1])
    assert a == b
    lines = a.decode().splitlines()
    prev = None
    for ln in lines:
        c, s, e = ln.split("\t")
        s, e = int(s), int(e)
        assert 20 <= e - s < 1000
        if prev and prev[0] == c:
            assert s > prev[1]
        prev = (c, s)
    shard = starch_amd.gen_bed(0, 20000, chroms=[1])
    assert a.endswith(shard)
    pp = starch_amd.gen_bed(2, 0, chroms=[23])
    assert pp.count(b"\n") == 57227415


def test_build_index_roundtrip():
    import json
    import starch_amd
    seg = starch_amd.Segment(line_count=3, text_bytes=10, stream_offset=4, stream_bytes=40, name_len=4,
                             n_blocks=1, combined_crc=7)
    blob = starch_amd.build_index([seg], [b"ch\"1"], 44, note="n")
    assert len(blob) > 32 and blob.endswith(b"\n")
    assert int(blob[-32:-12]) == 44
    j = json.loads(blob[:-32])
    assert j["streams"][0]["chromosome"] == "ch\"1"
    assert j["archive"]["note"] == "n"


def test_gen_perpos_sizes_match_host_generator():
    """starch_gen_perpos_device's byte count (closed-form digit sums, no GPU
    needed to size) equals the host generator's (tests/golden/fullsize_cfg5.json
    holds all 24 input sizes; the GPU test checks those)."""
    import starch_amd
    chroms = [13, 14, 23]                     # chr21, chr22, chrY (the host sizer walks every line)
    host = starch_amd.gen_bed_sizes(2, 0, chroms)
    for c, h in zip(chroms, host):
        assert starch_amd.gen_perpos_device(c) == h, c
    assert starch_amd.gen_perpos_device(0, first=0, count=0) == 0
    # a piece: lines [9, 11) of chr1 = "chr1\t9\t10\n" + "chr1\t10\t11\n"
    assert starch_amd.gen_perpos_device(0, first=9, count=2) == len(b"chr1\t9\t10\nchr1\t10\t11\n")
