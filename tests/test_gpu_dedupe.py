"""GPU parity of exact block reuse (starch_amd/csrc/bz2_dedupe.hip): streams
with byte-identical bzip2 blocks must come out byte-identical to libbz2 whether
blocks are reused (default), reuse is off (STARCH_DEDUPE=0), or candidates are
grouped so loosely that the byte compare rejects most of them
(STARCH_DEDUPE_KEY=n)."""
import bz2 as pybz2
import os
import random

import pytest

from tests import oracle_lib

pytestmark = pytest.mark.gpu

NMAX1 = 100000 * 1 - 19          # nblockMAX at blockSize100k = 1 (bz:bzlib.c:194)


def _ref(text, level):
    if oracle_lib.ref() is not None:
        return oracle_lib.ref_bz2(text, level)
    return oracle_lib.bz2(text, level)


def _no_runs(rng, n):
    """n bytes with no run of 4 equal bytes, so RLE1 is the identity and
    blocks are exactly nblockMAX input bytes."""
    out = bytearray()
    while len(out) < n:
        c = rng.randrange(256)
        if len(out) >= 3 and out[-1] == out[-2] == out[-3] == c:
            continue
        out.append(c)
    return bytes(out)


@pytest.fixture(scope="module")
def ctx():
    import starch_amd
    c = starch_amd.Starch(0)
    yield c
    c.close()


@pytest.fixture
def env():
    saved = {k: os.environ.get(k) for k in ("STARCH_DEDUPE", "STARCH_DEDUPE_KEY")}
    yield os.environ
    for k, v in saved.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v


def _cases():
    rng = random.Random(424242)
    x = _no_runs(rng, NMAX1)
    y = _no_runs(rng, NMAX1)
    if x[-3:] == bytes([x[0]]) * 3 or y[-3:] == bytes([x[0]]) * 3:
        raise AssertionError("generator produced a run across the block joint")
    tail = _no_runs(rng, 12345)
    return {
        "xxxxx+tail": x * 5 + tail,
        "xyxyx": x + y + x + y + x,
        "yx-x-yyy": y + x + x + y + y + y + tail,
        "text-phases": b"p1\n" + b"0\n" * 350_001,           # per-position (cfg5) phases
    }


@pytest.mark.parametrize("name", list(_cases()))
def test_reuse_matches_libbz2(ctx, env, name):
    text = _cases()[name]
    want = _ref(text, 1)
    for mode in ("default", "off", "key_n"):
        env.pop("STARCH_DEDUPE", None)
        env.pop("STARCH_DEDUPE_KEY", None)
        if mode == "off":
            env["STARCH_DEDUPE"] = "0"
        elif mode == "key_n":
            env["STARCH_DEDUPE_KEY"] = "n"
        got = ctx.bz2_compress(text, 1)
        assert got == want, (name, mode)
    assert pybz2.decompress(want) == text


def test_reuse_is_counted(ctx, env):
    import starch_amd
    env.pop("STARCH_DEDUPE", None)
    env.pop("STARCH_DEDUPE_KEY", None)
    # per-position BED of one chromosome slice: interior blocks repeat
    data = starch_amd.gen_bed(2, 0, chroms=[23])[:60_000_000]
    data = data[:data.rfind(b"\n") + 1]
    arch = ctx.compress(data)
    st = ctx.stats()
    assert st["dedup_blocks"] > 0
    _, streams = starch_amd.parse_archive(arch)
    _, osegs = oracle_lib.transform(data)
    assert pybz2.decompress(streams[0]) == osegs[0][2]
    env["STARCH_DEDUPE"] = "0"
    assert ctx.compress(data) == arch
    assert ctx.stats()["dedup_blocks"] == 0
