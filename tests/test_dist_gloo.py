"""The library's multi-rank gather (starch_amd/csrc/gather.hip, the same C++
that runs over RCCL on GPUs) driven through host primitives over
torch.distributed gloo on the CPU (starch_gather_host), world sizes 2, 3 and
8: every rank holds the bzip2 streams of its LPT share of the chromosome
units (made here by the CPU oracle -- transform with the units' initial
values, then bzip2 -9), rank 0 gathers them and writes the archive, which
must equal the one-rank archive byte for byte."""
import os
import socket

import pytest

from tests import corpus, oracle_lib


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _inputs(world):
    import starch_amd
    from starch_amd import dist
    data = corpus.multi_chrom_bed(7, 250, seed=21, kind="bed6") + corpus.fuzz_bed(3, 200)
    units, shard_of = dist.shard_units(data, world, max_units_per_rank=4)
    parts = []
    for r in range(world):
        recs, names, blob = [], [], b""
        for k, u in enumerate(units):
            if shard_of[k] != r:
                continue
            piece = data[u.offset:u.offset + u.length]
            _, segs = oracle_lib.transform(piece, u.init_start, u.init_stop)
            bcs = oracle_lib.base_counts(piece, u.init_start, u.init_stop)
            for (chr_, lines, text), (bu, bn) in zip(segs, bcs):
                st = oracle_lib.bz2(text, 9)
                recs.append([k, len(blob), len(st), lines, len(text), 1 + len(st) % 5, len(text) * 7919 % (1 << 32),
                             len(chr_), bu, bn])
                names.append(chr_)
                blob += st
        parts.append((recs, names, blob))
    # the one-rank archive: segments in input order
    _, whole = oracle_lib.transform(data)
    segs, names, body = [], [], bytearray(starch_amd.MAGIC)
    flat = sorted((rec[0], r, i) for r, (recs, _, _) in enumerate(parts) for i, rec in enumerate(recs))
    for _, r, i in flat:
        rec, name, blob = parts[r][0][i], parts[r][1][i], parts[r][2]
        segs.append(starch_amd.Segment(line_count=rec[3], text_bytes=rec[4], stream_offset=len(body),
                                       stream_bytes=rec[2], name_len=len(name), n_blocks=rec[5],
                                       combined_crc=rec[6], unit=rec[0], base_count_unique=rec[8],
                                       base_count_nonunique=rec[9]))
        names.append(name)
        body += blob[rec[1]:rec[1] + rec[2]]
    assert [n for n in names] == [c for c, _, _ in whole]
    # base counts of the units, in archive order, are the whole input's
    assert [(s.base_count_unique, s.base_count_nonunique) for s in segs] == oracle_lib.base_counts(data)
    expect = bytes(body) + starch_amd.build_index(segs, names, len(body), note="gloo", base_counts=True)
    return parts, expect


def _rank_main(rank, world, port, parts, out_path):
    import torch
    import torch.distributed as tdist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    tdist.init_process_group("gloo", rank=rank, world_size=world)
    import starch_amd
    from starch_amd import dist
    recs, names, blob = parts[rank]
    segs = [starch_amd.Segment(unit=r[0], stream_offset=r[1], stream_bytes=r[2], line_count=r[3], text_bytes=r[4],
                               n_blocks=r[5], combined_crc=r[6], name_len=r[7], base_count_unique=r[8],
                               base_count_nonunique=r[9]) for r in recs]
    prims = dist.TorchHostPrimitives()
    arch = dist.gather_archive(prims, segs, names, blob, note="gloo", base_counts=True)
    assert (arch is None) == (rank != 0)
    if rank == 0:
        with open(out_path, "wb") as f:
            f.write(arch)
    tdist.barrier()
    tdist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_gloo_gather_equals_one_rank_archive(world, tmp_path):
    import torch.multiprocessing as mp
    parts, expect = _inputs(world)
    if world <= 3:
        assert all(p[0] for p in parts), "every rank should own some units"
    out = str(tmp_path / "arch.bin")
    mp.spawn(_rank_main, args=(world, _free_port(), parts, out), nprocs=world, join=True)
    got = open(out, "rb").read()
    assert got == expect
