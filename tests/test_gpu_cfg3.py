"""cfg3 (BASELINE.json configs[2]: the 100 M-interval cfg2 input sharded per
chromosome over 8 MI355X, gathered over RCCL/xGMI) exercised on a one-GPU box
at full size, checked stream by stream against the CPU path's goldens
(tests/golden/fullsize_cfg2.json: the oracle transform + the reference's own
libbz2 1.0.6):

* 8 virtual shards in one process (starch_encode_multi_host: LPT over 8
  contexts on device 0, peer/device copies into context 0's archive);
* 8 rank shards, each encoded on the GPU from its units alone
  (starch_encode_units_host), their real GPU streams then gathered by the
  library's C++ gather in a world-8 gloo group (starch_gather_host -- the same
  gather code RCCL drives), archive == the one-GPU archive byte for byte;
* the RCCL transport itself at world 1 (starch_comm_* + starch_gather_archive)
  and bench.py's multi-rank path (--dist-path) at one rank.
The unit of independence is the reference's per-chromosome hand-off
process_tf_buffer (include/starch3api.hpp:393-407)."""
import ctypes
import hashlib
import json
import os
import socket
import subprocess
import sys

import pytest

from tests import corpus

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden", "fullsize_cfg2.json")


def _cfg2_host():
    import torch
    import starch_amd
    g = json.load(open(GOLDEN))
    n = g["input_bytes"]
    host = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    starch_amd.gen_bed(g["kind"], g["total_lines"], seed=g["seed"], into=ctypes.c_void_p(host.data_ptr()))
    return g, host, n


def _check_golden(g, arch):
    import starch_amd
    idx, streams = starch_amd.parse_archive(arch)
    assert len(streams) == 24
    for st, meta, want in zip(streams, idx["streams"], g["streams"]):
        assert meta["chromosome"] == want["chromosome"]
        assert meta["uncompressedLineCount"] == want["lines"]
        assert meta["transformedBytes"] == want["text_bytes"]
        assert len(st) == want["stream_bytes"], want["chromosome"]
        assert hashlib.sha256(st).hexdigest() == want["sha256"], want["chromosome"]


def test_cfg3_eight_virtual_shards_fullsize():
    import starch_amd
    g, host, n = _cfg2_host()
    ctxs = [starch_amd.Starch(0) for _ in range(8)]
    L = starch_amd.load()
    o = ctxs[0]._opts()
    H = (ctypes.c_void_p * 8)(*[c._h.value for c in ctxs])
    starch_amd._check(L.starch_encode_multi_host(H, 8, ctypes.cast(ctypes.c_void_p(host.data_ptr()), ctypes.c_char_p),
                                                 n, ctypes.byref(o)), ctxs[0]._h)
    arch = ctxs[0].archive()
    _check_golden(g, arch)
    # every context encoded a share: LPT over 24 chromosomes on 8 shards
    assert all(c.stats()["n_lines"] > 0 for c in ctxs[1:])
    for c in ctxs:
        c.close()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_cfg3_rank_shards_through_world8_gather(tmp_path):
    """Each of the 8 LPT shards encoded on the GPU from its own units; the
    streams + segment records go to 8 CPU-only gloo ranks that run the
    library's gather; the archive equals the one-GPU archive."""
    import starch_amd
    g, host, n = _cfg2_host()
    whole = starch_amd.Starch(0)
    whole.compress_host_ptr(host.data_ptr(), n)
    ref = whole.archive()
    whole.close()
    _check_golden(g, ref)
    # plan units over the host input (library planner), LPT over 8 ranks
    L = starch_amd.load()
    cap = 64 * 8
    U = (starch_amd.Unit * cap)()
    nu = ctypes.c_uint64()
    starch_amd._check(L.starch_plan_units(ctypes.cast(ctypes.c_void_p(host.data_ptr()), ctypes.c_char_p), n, cap, U,
                                          ctypes.byref(nu)))
    units = [U[k] for k in range(nu.value)]
    assert len(units) >= 24
    shard_of = starch_amd.assign_shards(units, 8)
    ctx = starch_amd.Starch(0)
    for r in range(8):
        ids = [k for k in range(len(units)) if shard_of[k] == r]
        assert ids, r
        ctx.encode_units_host(host.data_ptr(), [units[k] for k in ids], ids)
        segs = ctx.segments()
        blob = ctx.streams()
        recs = [[s.unit, s.stream_offset, s.stream_bytes, s.line_count, s.text_bytes, s.n_blocks, s.combined_crc,
                 s.name_len, s.base_count_unique, s.base_count_nonunique] for _, s in segs]
        (tmp_path / ("r%d.bin" % r)).write_bytes(blob)
        (tmp_path / ("r%d.json" % r)).write_text(json.dumps({"recs": recs, "names": [nm.hex() for nm, _ in segs]}))
    ctx.close()
    port = _free_port()
    procs = [subprocess.Popen([sys.executable, "-c", _RANK_SRC, str(r), "8", str(port), str(tmp_path)], cwd=ROOT,
                              env=dict(os.environ, HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES=""))
             for r in range(8)]
    rcs = [p.wait(timeout=600) for p in procs]
    assert rcs == [0] * 8
    got = (tmp_path / "archive.bin").read_bytes()
    assert got == ref


# a CPU-only gloo rank: reads its shard's GPU streams, runs the C++ gather
_RANK_SRC = r'''
import json, os, sys
rank, world, port, d = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
import torch.distributed as tdist
tdist.init_process_group("gloo", rank=rank, world_size=world)
import starch_amd
from starch_amd import dist
j = json.load(open(os.path.join(d, "r%d.json" % rank)))
blob = open(os.path.join(d, "r%d.bin" % rank), "rb").read()
segs = [starch_amd.Segment(unit=r[0], stream_offset=r[1], stream_bytes=r[2], line_count=r[3], text_bytes=r[4],
                           n_blocks=r[5], combined_crc=r[6], name_len=r[7], base_count_unique=r[8],
                           base_count_nonunique=r[9]) for r in j["recs"]]
arch = dist.gather_archive(dist.TorchHostPrimitives(), segs, [bytes.fromhex(x) for x in j["names"]], blob)
if rank == 0:
    open(os.path.join(d, "archive.bin"), "wb").write(arch)
tdist.barrier()
tdist.destroy_process_group()
'''


def test_rccl_gather_world1_equals_one_call():
    """The RCCL transport (starch_comm_create + starch_gather_archive) at
    world 1: units encoded as one shard, gathered into the archive."""
    import starch_amd
    data = corpus.multi_chrom_bed(6, 2000, seed=4, kind="bed6") + corpus.fuzz_bed(5, 300)
    c = starch_amd.Starch(0)
    ref = c.compress(data)
    units = starch_amd.plan_units(data, 32)
    comm = starch_amd.Comm(0, 0, 1, starch_amd.Comm.new_id())
    c.encode_units_host(data, units, list(range(len(units))))
    c.gather_archive(comm)
    assert c.archive() == ref
    # a subset of the units: their streams, in order
    c.encode_units_host(data, units[1:], list(range(1, len(units))))
    c.gather_archive(comm)
    idx, streams = starch_amd.parse_archive(c.archive())
    ridx, rstreams = starch_amd.parse_archive(ref)
    assert streams == rstreams[len(rstreams) - len(streams):]
    comm.close()
    c.close()


def test_cli_distributed_world1_equals_single(tmp_path):
    import starch_amd
    exe = os.path.join(os.path.dirname(starch_amd.LIB_PATH), "starch3")
    data = starch_amd.gen_bed(0, 400_000)
    f = tmp_path / "in.bed"
    f.write_bytes(data)
    env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
               STARCH_COMM_PORT=str(_free_port()))
    one = subprocess.run([exe, str(f)], capture_output=True, timeout=300)
    dist = subprocess.run([exe, "--distributed", str(f)], capture_output=True, timeout=300, env=env)
    assert one.returncode == 0 and dist.returncode == 0, (one.stderr, dist.stderr)
    assert dist.stdout == one.stdout


def test_bench_dist_path_one_rank():
    """bench.py's N>1 code path (torch.distributed + the library's RCCL
    gather) at one rank on a reduced cfg2: 24 streams verified against the
    oracle for chr21/chr22 (the verify leg) and a well-formed line."""
    env = dict(os.environ, MASTER_PORT=str(_free_port()))
    r = subprocess.run([sys.executable, "bench.py", "--dist-path", "--steps", "2", "--warmup", "1", "--lines",
                        "3000000"], cwd=ROOT, capture_output=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(r.stdout.decode().strip().splitlines()[-1])
    assert line["n_gpus"] == 1 and line["config"]["lines"] == 3_000_000
    assert line["config"]["archive_bytes"] > 0
