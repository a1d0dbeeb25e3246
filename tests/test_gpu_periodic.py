"""Periodic full blocks: the one place where bzip2's output depends on its sort's
tie order.  A block that is k exact copies of a period p has k identical copies
of every rotation; bzip2-1.0.6 always sorts such a block with fallbackSort
(mainSort exhausts its budget, bz:blocksort.c:1057-1068) and origPtr is the rank
fallbackQSort3 (bz:blocksort.c:92-180) leaves rotation 0 at among its copies.
The GPU reproduces that order in k_fallback_exact (bz2_bwt.hip); these cases
are single full 900 KB blocks (the block length is a multiple of the period),
from period 2 (no bucket is ever mixed) to period n/2 (every bucket of the
first doubling round is mixed and ~n/alphabet large).  Each is checked
byte-for-byte against the CPU oracle, whose fallbackSort restatement the
reference's own libbz2 pins (test_oracle.py: 25 periodic goldens), and timed;
the times go to gpurun_out/periodic_times.json."""
import json
import os
import random
import time

import pytest

from tests import oracle_lib

pytestmark = pytest.mark.gpu

NBLOCK_MAX = 899981          # bz:bzlib.c:194 at -9


def _periodic(unit, total=NBLOCK_MAX):
    k = total // len(unit)
    return unit * k


def _rand_unit(seed, p, alphabet):
    r = random.Random(seed)
    return bytes(r.choice(alphabet) for _ in range(p))


CASES = [
    ("p2", lambda: _periodic(b"0\n")),
    ("p3", lambda: _periodic(b"ab\n")),
    ("p5_text", lambda: _periodic(b"p1\n0\n")),
    ("p997", lambda: _periodic(_rand_unit(1, 997, b"0123456789\n-p"))),
    ("p12345", lambda: _periodic(_rand_unit(2, 12345, b"0123456789\n-p"))),
    ("p_half_5sym", lambda: _periodic(_rand_unit(3, NBLOCK_MAX // 2, b"ACGTN"))),
    ("p_third_2sym", lambda: _periodic(_rand_unit(4, NBLOCK_MAX // 3, b"ab"))),
]

_times = {}


@pytest.fixture(scope="module")
def ctx():
    import starch_amd
    c = starch_amd.Starch(0)
    yield c
    c.close()
    os.makedirs("gpurun_out", exist_ok=True)
    with open(os.path.join("gpurun_out", "periodic_times.json"), "w") as f:
        json.dump(_times, f, indent=1)


@pytest.mark.parametrize("name,make", CASES, ids=[c[0] for c in CASES])
def test_periodic_full_block(ctx, name, make):
    data = make()
    assert len(data) <= NBLOCK_MAX
    ctx.bz2_compress(data[:4096], 9)                      # warm the context
    t0 = time.perf_counter()
    got = ctx.bz2_compress(data, 9)
    dt = time.perf_counter() - t0
    _times[name] = {"bytes": len(data), "seconds": round(dt, 4)}
    print("%s: %d bytes, %.1f ms" % (name, len(data), dt * 1e3))
    assert got == oracle_lib.bz2(data, 9), name
    assert dt < 0.1, (name, dt)          # measured 11-30 ms per block; catches a serial blow-up


def test_periodic_blocks_batched(ctx):
    """Several periodic blocks in ONE encode (one sort batch): their fallbackSort
    replays run concurrently (one HIP stream each, bz2_bwt.hip launch_fallback);
    every stream still equals the oracle's, and the batch costs about one block's
    replay, not the sum."""
    import torch
    datas = [make() for _, make in CASES] + [_periodic(b"1\n"), _periodic(b"xyz\n")]
    offs, lens, o = [], [], 0
    for d in datas:
        offs.append(o)
        lens.append(len(d))
        o += (len(d) + 255) // 256 * 256
    host = bytearray(o)
    for d, a in zip(datas, offs):
        host[a:a + len(d)] = d
    d_in = torch.frombuffer(host, dtype=torch.uint8).to("cuda")
    cap = o + o // 50 + 4096 * len(datas)
    d_out = torch.empty(cap, dtype=torch.uint8, device="cuda")
    ctx.bz2_compress_many_device(d_in.data_ptr(), offs, lens, 9, d_out.data_ptr(), cap)   # warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    oo, ol = ctx.bz2_compress_many_device(d_in.data_ptr(), offs, lens, 9, d_out.data_ptr(), cap)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    _times["batch_%d" % len(datas)] = {"bytes": sum(lens), "seconds": round(dt, 4)}
    out = d_out.cpu().numpy().tobytes()
    for d, a, n in zip(datas, oo, ol):
        assert out[a:a + n] == oracle_lib.bz2(d, 9)
    assert dt < 0.15, dt                 # the replays overlap: ~one block's time, not len(datas) x
