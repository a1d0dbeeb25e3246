"""starch_amd.dist -- multi-process (one rank per MI355X) Starch: shard the
per-chromosome units across ranks, encode each rank's units on its own GPU,
and gather the finished bzip2 streams to rank 0, which writes the archive.

The reference has no distributed layer: its unit of independence
is the per-chromosome hand-off process_tf_buffer (include/starch3api.hpp:
393-407), so chromosome streams shard with no data-path exchange and the only
collective is the gather of compressed streams.

The gather itself is the library's C++ (starch_amd/csrc/gather.hip): on GPUs
``Starch.gather_archive(Comm)`` runs it over RCCL (xGMI) with no Python in the
data path; ``gather_archive`` below drives the SAME C++ gather through host
primitives backed by a torch.distributed group (gloo on the CPU tests).
Planning, LPT assignment, archive layout and the index writer are the
library's host code too; this module only adapts transports.
"""
import starch_amd


def shard_units(bed: bytes, world: int, max_units_per_rank: int = 64):
    """Plan units over host BED bytes and LPT them over `world` ranks ->
    (units, shard_of)."""
    units = starch_amd.plan_units(bed, max(1, max_units_per_rank * world))
    return units, starch_amd.assign_shards(units, world)


def comm_from_torch(device, group=None):
    """An RCCL communicator (starch_amd.Comm) for the ranks of a torch
    process group: rank 0's unique id is broadcast over the group."""
    import torch
    import torch.distributed as dist
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    dev = torch.device("cuda", device) if dist.get_backend(group) == "nccl" else torch.device("cpu")
    t = torch.zeros(128, dtype=torch.uint8, device=dev)
    if rank == 0:
        t.copy_(torch.frombuffer(bytearray(starch_amd.Comm.new_id()), dtype=torch.uint8))
    dist.broadcast(t, 0, group=group)
    return starch_amd.Comm(device, rank, world, t.cpu().numpy().tobytes())


class TorchHostPrimitives:
    """The four primitives of starch_gather_host over a torch.distributed group
    (host bytes; gloo on CPU)."""

    def __init__(self, group=None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self._ops = []

    def all_gather(self, data: bytes):
        import torch
        t = torch.frombuffer(bytearray(data), dtype=torch.uint8) if data else torch.empty(0, dtype=torch.uint8)
        out = [torch.empty_like(t) for _ in range(self.world)]
        self.dist.all_gather(out, t, group=self.group)
        return [x.numpy().tobytes() for x in out]

    def send(self, data: bytes, peer):
        import torch
        self._ops.append(("s", torch.frombuffer(bytearray(data), dtype=torch.uint8), peer))

    def recv(self, n, peer):
        import torch
        t = torch.empty(n, dtype=torch.uint8)
        self._ops.append(("r", t, peer))
        return len(self._ops) - 1

    def group_end(self):
        d = self.dist
        ops = [d.P2POp(d.isend if k == "s" else d.irecv, t, p, group=self.group) for k, t, p in self._ops]
        if ops:
            for w in d.batch_isend_irecv(ops):
                w.wait()
        got = {i: t.numpy().tobytes() for i, (k, t, _) in enumerate(self._ops) if k == "r"}
        self._ops = []
        return got


def gather_archive(prims, segments, names, streams: bytes, note=None, level=9, emit_index=True, base_counts=False):
    """The library's gather over host primitives (TorchHostPrimitives):
    segments = this rank's starch_amd.Segment list (stream_offset into
    `streams`, unit = global unit index), names = their chromosome bytes.
    Returns the archive bytes on rank 0 (byte-identical to a one-GPU run),
    None elsewhere."""
    return starch_amd.gather_host(prims.rank, prims.world, prims.all_gather, prims.send, prims.recv,
                                  prims.group_end, segments, names, streams, note=note, level=level,
                                  emit_index=emit_index, base_counts=base_counts)


def encode_rank(ctx, d_base, units, unit_ids, note=None, level=9):
    """Encode this rank's units (resident in HBM at d_base) -> ctx holds the
    streams for ctx.gather_archive / local_segments."""
    ctx.block_size_100k = level
    ctx.set_note(note or "")
    ctx.encode_units_device(d_base, units, unit_ids)


def local_segments(ctx):
    """This rank's segments after encode_units_*: ([Segment], [name bytes])."""
    segs = ctx.segments()
    return [s for _, s in segs], [n for n, _ in segs]
