"""The RCCL gather across real ranks: one process per GPU, each
encoding its LPT share of the chromosome units -- the unit of independence is
the reference's per-chromosome hand-off process_tf_buffer
(include/starch3api.hpp:393-407) -- then ncclAllGather of the segment records
and grouped ncclSend/ncclRecv of the streams straight into rank 0's archive
(starch_amd/csrc/gather.hip).  Rank 0's archive must equal the one-GPU
archive byte for byte.

The parent counts GPUs the way bench.py does (KFD topology in sysfs, no HIP
call) before starting the ranks as fresh child processes (no exec).  World 1
runs on every GPU box (the same path: a TCP rendezvous, one rank); world 2
runs when two or more GPUs are visible and is skipped otherwise."""
import importlib.util
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LINES = 2_000_000          # a reduced cfg2: 24 chromosomes, ~48 MB of BED3

_RANK_SRC = r'''
import os, sys
rank, world, port, out = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
import starch_amd
data = bytes(starch_amd.gen_bed(0, %d))
units = starch_amd.plan_units(data, 64)
shard_of = starch_amd.assign_shards(units, world)
ids = [k for k in range(len(units)) if shard_of[k] == rank]
ctx = starch_amd.Starch(rank)
comm = starch_amd.Comm.tcp(rank, rank, world, "127.0.0.1", port)
ctx.encode_units_host(data, [units[k] for k in ids], ids)
ctx.gather_archive(comm)
if rank == 0:
    open(out, "wb").write(ctx.archive())
comm.close()
ctx.close()
''' % LINES


def _visible_gpus():
    spec = importlib.util.spec_from_file_location("starch_bench", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)           # (module level: definitions only; no HIP call)
    return bench.visible_gpus()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [1, 2])
def test_rccl_ranks_gather_equals_one_gpu_archive(world, tmp_path):
    have = _visible_gpus()
    if have is None or have < world:
        pytest.skip("%d GPU(s) visible, world %d needs one per rank" % (have or 0, world))
    out = tmp_path / "archive.bin"
    port = _free_port()
    env = dict(os.environ)
    procs = [subprocess.Popen([sys.executable, "-c", _RANK_SRC, str(r), str(world), str(port), str(out)], cwd=ROOT,
                              env=env, stderr=subprocess.PIPE) for r in range(world)]
    errs = []
    for p in procs:
        try:
            _, e = p.communicate(timeout=300)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        errs.append(e.decode(errors="replace")[-2000:])
    assert [p.returncode for p in procs] == [0] * world, errs
    import starch_amd
    data = bytes(starch_amd.gen_bed(0, LINES))
    c = starch_amd.Starch(0)
    want = c.compress(data)
    c.close()
    got = out.read_bytes()
    assert got == want
    idx, streams = starch_amd.parse_archive(got)
    assert len(streams) == 24
