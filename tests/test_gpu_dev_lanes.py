"""Encoder lanes of the device path (starch_api.hip lane_cuts / encode_units):
after one transform, the segments split into contiguous runs encoded by
separate encoders on their own streams and host threads, then emitted in
order.  The archive must be byte-identical whatever the lane count, and the
stats counters must add up the same.

The lane count and the size floor are read once per process
(STARCH_DEV_LANES, STARCH_DEV_LANES_MIN), so every count runs in a fresh
child process (started before anything touches the GPU in it)."""
import hashlib
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_SRC = r'''
import hashlib, json, sys
import starch_amd
kind, lines = int(sys.argv[1]), int(sys.argv[2])
data = bytes(starch_amd.gen_bed(kind, lines))
c = starch_amd.Starch(0)
out = {}
a = c.compress(data)
st = c.stats()
out["sha"] = hashlib.sha256(a).hexdigest()
out["n_blocks"] = st["n_blocks"]
out["rle_bytes"] = st["rle_bytes"]
out["n_segments"] = st["n_segments"]
# a second encode on the same context (lane encoders and workers reused)
out["sha2"] = hashlib.sha256(c.compress(data)).hexdigest()
c.close()
print(json.dumps(out))
'''


def _run(lanes, kind, lines):
    env = dict(os.environ)
    env["STARCH_DEV_LANES"] = str(lanes)
    env["STARCH_DEV_LANES_MIN"] = "0"
    p = subprocess.run([sys.executable, "-c", _SRC, str(kind), str(lines)], cwd=ROOT, env=env,
                       capture_output=True, timeout=300)
    assert p.returncode == 0, p.stderr.decode(errors="replace")[-3000:]
    return json.loads(p.stdout.decode().strip().splitlines()[-1])


@pytest.mark.parametrize("kind,lines", [(0, 400_000), (1, 150_000)])
def test_lanes_give_the_one_lane_archive(kind, lines):
    one = _run(1, kind, lines)
    assert one["sha"] == one["sha2"]
    assert one["n_segments"] == 24
    for lanes in (2, 3):
        got = _run(lanes, kind, lines)
        assert got["sha"] == one["sha"], (lanes, got, one)
        assert got["sha2"] == one["sha"]
        assert (got["n_blocks"], got["rle_bytes"]) == (one["n_blocks"], one["rle_bytes"])
