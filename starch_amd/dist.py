"""starch_amd.dist -- multi-process (one rank per MI355X) Starch: shard the
per-chromosome units across ranks, encode each rank's units on its own GPU,
and gather the finished bzip2 streams to rank 0, which writes the archive.

The reference has no distributed layer: its unit of independence
is the per-chromosome hand-off process_tf_buffer (include/starch3api.hpp:
393-407), so chromosome streams shard with no data-path exchange and the only
collective is the gather of compressed streams.  The transport is
pluggable: ``TorchTransport`` wraps a torch.distributed process group
(backend "nccl" = RCCL over xGMI on MI355X; "gloo" on CPU for tests).

Planning, LPT assignment, archive layout and the index writer are the
library's host code (starch_plan_units / starch_assign_shards /
starch_archive_layout / starch_build_index); this module only moves bytes.
"""
import starch_amd

# metadata columns exchanged per segment
_COLS = ("unit", "stream_offset", "stream_bytes", "line_count", "text_bytes", "n_blocks", "combined_crc", "name_len",
         "base_count_unique", "base_count_nonunique")


class TorchTransport:
    """torch.distributed process group as the gather transport."""

    def __init__(self, device, group=None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.device = device
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)

    def all_gather(self, t):
        """Same-shape tensors from every rank -> list indexed by rank."""
        import torch
        out = [torch.empty_like(t) for _ in range(self.world)]
        self.dist.all_gather(out, t, group=self.group)
        return out

    def exchange(self, sends, recvs):
        """sends: [(tensor, dst)], recvs: [(tensor, src)]; per peer pair the
        ops match in issue order."""
        ops = [self.dist.P2POp(self.dist.isend, t, p, group=self.group) for t, p in sends]
        ops += [self.dist.P2POp(self.dist.irecv, t, p, group=self.group) for t, p in recvs]
        if ops:
            for w in self.dist.batch_isend_irecv(ops):
                w.wait()


def shard_units(bed: bytes, world: int, max_units_per_rank: int = 64):
    """Plan units over host BED bytes and LPT them over `world` ranks ->
    (units, shard_of)."""
    units = starch_amd.plan_units(bed, max(1, max_units_per_rank * world))
    return units, starch_amd.assign_shards(units, world)


def local_segments(ctx):
    """This rank's segments after Starch.encode_units_device: (records, names)."""
    segs = ctx.segments()
    rec = [[getattr(s, c) for c in _COLS] for _, s in segs]
    return rec, [n for n, _ in segs]


def gather_archive(tr, records, names, streams, note=None, level=9, emit_index=True, base_counts=False):
    """Gather every rank's streams to rank 0 in archive (unit) order.

    records / names: this rank's segments (``local_segments``); streams: a
    uint8 tensor holding this rank's stream bytes (offsets in records are
    relative to it), on the transport's device.  Returns the archive as a
    uint8 tensor on rank 0 (magic + streams + index + footer, byte-identical
    to a one-GPU run) and None on the other ranks.
    """
    import torch
    dev = tr.device
    n = torch.tensor([len(records), sum(len(x) for x in names)], dtype=torch.int64, device=dev)
    counts = [tuple(int(v) for v in x.tolist()) for x in tr.all_gather(n)]
    maxn = max(1, max(c[0] for c in counts))
    maxb = max(1, max(c[1] for c in counts))
    rec = torch.zeros((maxn, len(_COLS)), dtype=torch.int64, device=dev)
    if records:
        rec[:len(records)] = torch.tensor(records, dtype=torch.int64)
    nm = torch.zeros(maxb, dtype=torch.uint8, device=dev)
    blob = b"".join(names)
    if blob:
        nm[:len(blob)] = torch.frombuffer(bytearray(blob), dtype=torch.uint8)
    all_rec = [x.cpu().tolist() for x in tr.all_gather(rec)]
    all_nm = [bytes(x.cpu().numpy().tobytes()) for x in tr.all_gather(nm)]

    # global segment list in (rank, local order); layout is computed on every
    # rank so senders and the receiver agree on the coalesced runs
    segs = []          # (rank, record, name)
    for r in range(tr.world):
        pos = 0
        for row in all_rec[r][:counts[r][0]]:
            ln = row[_COLS.index("name_len")]
            segs.append((r, row, all_nm[r][pos:pos + ln]))
            pos += ln
    unit_of = [row[0] for _, row, _ in segs]
    nbytes = [row[2] for _, row, _ in segs]
    order, offset, end = starch_amd.archive_layout(unit_of, nbytes, base=4)
    runs = []          # (rank, src offset, dst offset, length): adjacent in part and archive
    for g in order:
        r, row, _ = segs[g]
        if runs and runs[-1][0] == r and runs[-1][1] + runs[-1][3] == row[1] and runs[-1][2] + runs[-1][3] == offset[g]:
            runs[-1][3] += row[2]
        else:
            runs.append([r, row[1], offset[g], row[2]])
    runs = [x for x in runs if x[3] > 0]

    if tr.rank != 0:
        tr.exchange([(streams[s:s + ln], 0) for r, s, _, ln in runs if r == tr.rank], [])
        return None
    out_segs, out_names = [], []
    for g in order:
        r, row, name = segs[g]
        d = dict(zip(_COLS, row))
        out_segs.append(starch_amd.Segment(line_count=d["line_count"], text_bytes=d["text_bytes"],
                                           stream_offset=offset[g], stream_bytes=d["stream_bytes"],
                                           name_len=len(name), n_blocks=d["n_blocks"],
                                           combined_crc=d["combined_crc"] & 0xFFFFFFFF, unit=d["unit"],
                                           base_count_unique=d["base_count_unique"],
                                           base_count_nonunique=d["base_count_nonunique"]))
        out_names.append(name)
    idx = (starch_amd.build_index(out_segs, out_names, end, note=note, level=level, base_counts=base_counts)
           if emit_index else b"")
    arch = torch.empty(end + len(idx), dtype=torch.uint8, device=dev)
    arch[0:4] = torch.frombuffer(bytearray(starch_amd.MAGIC), dtype=torch.uint8)
    for r, s, d, ln in runs:
        if r == 0:
            arch[d:d + ln].copy_(streams[s:s + ln])
    tr.exchange([], [(arch[d:d + ln], r) for r, s, d, ln in runs if r != 0])
    if idx:
        arch[end:] = torch.frombuffer(bytearray(idx), dtype=torch.uint8)
    return arch


def encode_rank(ctx, d_base, units, unit_ids, note=None, level=9):
    """Encode this rank's units (resident in HBM at d_base) -> (records, names,
    streams tensor view on the GPU)."""
    ctx.block_size_100k = level
    ctx.set_note(note or "")
    ctx.encode_units_device(d_base, units, unit_ids)
    p, nbytes = ctx.streams_device()
    return local_segments(ctx) + (device_bytes(p, nbytes),)


def device_bytes(ptr, nbytes):
    """A uint8 CUDA tensor view of library-owned HBM (no copy)."""
    import torch

    class _A:
        __cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "data": (ptr or 1, False), "version": 3}
    if nbytes == 0:
        return torch.empty(0, dtype=torch.uint8, device="cuda")
    return torch.as_tensor(_A(), device="cuda")

