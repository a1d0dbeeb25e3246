#!/usr/bin/env python3
"""bench.py -- input-BED MB/s of the MI355X Starch compressor (BASELINE.json
metric) on cfg2: 100 M-interval synthetic hg38 24-chromosome BED3, bzip2 -9.

One process per GPU.  N=1: the whole input on one MI355X.  N>1 (cfg3, launched
by torch.distributed.run): chromosomes LPT-partitioned across ranks by size,
each rank encodes its chromosomes' streams, and rank 0 gathers the finished
streams over RCCL (xGMI) and assembles the archive -- magic + streams in input
order + JSON index -- so the timed step is the whole job.  Inputs are
generated (seeded, tools-independent C generator in the library), copied to
HBM before timing; a "step" = one full compression of the resident input.

Prints ONE JSON line on rank 0 (contract in the task statement), with
"roofline" for the dominant kernel (the block sort, k_bwt) measured by HIP
events on the library's stream, and "cpu_baseline": the reference's own
bzip2 (oracle/_ref/libbz2ref.so, built from third-party/bzip2-1.0.6) plus the
C transform restatement, timed on this host on a bounded sample.
"""
import argparse
import ctypes
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8 TB/s HBM3E (spec)
TOTAL_LINES = 100_000_000      # cfg2
SEED = 20261015


WORKLOADS = {
    0: ("cfg2: 100M-interval synthetic hg38 24-chrom BED3, bzip2 -9",
        "synthetic (seeded hg38 BED3 generator, libstarch_amd starch_gen_bed)"),
    1: ("cfg4: 50M-row ENCODE-style narrowPeak BED6+4, bzip2 -9",
        "synthetic (seeded hg38 narrowPeak generator, libstarch_amd starch_gen_bed)"),
    2: ("cfg5: 3.09G-line single-base per-position hg38 BED (73.6 GB), bzip2 -9",
        "synthetic (every position of the 24 hg38 chromosomes, libstarch_amd starch_gen_bed)"),
}


def lpt(sizes, n):
    """Longest-processing-time assignment of items to n bins."""
    bins = [[] for _ in range(n)]
    load = [0] * n
    for i in sorted(range(len(sizes)), key=lambda k: -sizes[k]):
        b = min(range(n), key=lambda k: load[k])
        bins[b].append(i)
        load[b] += sizes[i]
    return [sorted(b) for b in bins]


def cuda_view(ptr, nbytes):
    import torch

    class _A:
        __cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "data": (ptr, False), "version": 3}
    return torch.as_tensor(_A(), device="cuda")


def _chrom_prefixes(data, names, k):
    """First k lines of every chromosome present in `data` (sorted BED)."""
    import numpy as np
    out = []
    for nm in names:
        key = nm.encode() + b"\t"
        start = 0 if data.startswith(key) else data.find(b"\n" + key)
        if start < 0:
            continue
        if start or not data.startswith(key):
            start += 1
        window = np.frombuffer(data, dtype=np.uint8, count=min(len(data) - start, k * 96), offset=start)
        nls = np.flatnonzero(window == 10)
        end = start + (int(nls[k - 1]) + 1 if len(nls) >= k else len(window))
        out.append(data[start:end])
    return out


def _perpos_prefixes(names, k):
    """First k lines of every chromosome of the per-position input (cfg5): the
    generator writes line p of a chromosome as "<chr>\t<p>\t<p+1>\n"."""
    return [b"".join(b"%s\t%d\t%d\n" % (nm.encode(), p, p + 1) for p in range(k)) for nm in names]


def cpu_baseline(pieces, threads, workload):
    """Reference bzip2 (-9, workFactor 30) + the C transform restatement on a
    bounded sample of the same input: the first lines of each chromosome
    (`pieces`), one chromosome per thread (ctypes releases the GIL)."""
    from tests import oracle_lib
    ref = oracle_lib.ref()
    kind = "reference" if ref is not None else "port"
    sample_bytes = sum(len(p) for p in pieces)
    todo = list(pieces)
    lock = threading.Lock()

    def runner():
        while True:
            with lock:
                if not todo:
                    return
                p = todo.pop()
            _, segs = oracle_lib.transform(p)
            for _, _, t in segs:
                if ref is not None:
                    oracle_lib.ref_bz2(t, 9)
                else:
                    oracle_lib.bz2(t, 9)

    t0 = time.perf_counter()
    ths = [threading.Thread(target=runner) for _ in range(threads)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    dt = time.perf_counter() - t0
    return {"value": round(sample_bytes / dt / 1e6, 2), "unit": "MB/s", "cores": threads, "kind": kind,
            "seconds": round(dt, 2),
            "sample": "first %d lines of each of the %d chromosomes of the same %s input (%.1f MB); transform = "
                      "C restatement (oracle/starch_oracle.c), bzip2 -9 = %s; one chromosome per thread"
                      % (pieces[0].count(b"\n") if pieces else 0, len(pieces), workload, sample_bytes / 1e6,
                         "the reference's vendored libbz2 1.0.6 (oracle/_ref/libbz2ref.so)" if ref is not None
                         else "oracle restatement")}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--lines", type=int, default=TOTAL_LINES)
    ap.add_argument("--kind", type=int, default=0,
                    help="0 BED3 (cfg2), 1 narrowPeak (cfg4), 2 per-position 3.09 G lines (cfg5; --lines ignored)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-lines", type=int, default=1_000_000)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--verify", action="store_true", help="check 2 chromosome streams vs the CPU path")
    args = ap.parse_args()

    import torch
    import starch_amd

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)

    shards = lpt(starch_amd.HG38_LEN, world)
    mine = shards[rank]

    t_gen = time.perf_counter()
    L = starch_amd.load()
    C = (ctypes.c_int32 * len(mine))(*mine)
    nb = ctypes.c_uint64()
    L.starch_gen_bed(args.kind, SEED, args.lines, C, len(mine), None, 0, ctypes.byref(nb))
    host = torch.empty(nb.value + 64, dtype=torch.uint8, pin_memory=True)
    L.starch_gen_bed(args.kind, SEED, args.lines, C, len(mine), ctypes.c_void_p(host.data_ptr()), nb.value,
                     ctypes.byref(nb))
    my_bytes = nb.value
    dev_in = host.to("cuda", non_blocking=False)
    t_gen = time.perf_counter() - t_gen

    ctx = starch_amd.Starch(local)
    stream = torch.cuda.current_stream()
    ctx.set_stream(stream.cuda_stream)

    total_bytes = my_bytes
    if dist is not None:
        t = torch.tensor([my_bytes], dtype=torch.int64, device="cuda")
        dist.all_reduce(t)
        total_bytes = int(t.item())

    def step():
        ctx.compress_device(dev_in.data_ptr(), my_bytes, emit_index=(dist is None))
        if dist is None:
            return None
        # ---- RCCL gather of finished streams to rank 0 -------------------------
        segs = ctx.segments()
        n = ctx.archive_size()
        blob = cuda_view(ctx.archive_device_ptr(), n)[4:n]            # this rank's streams
        meta = torch.tensor([blob.numel()], dtype=torch.int64, device="cuda")
        allm = [torch.zeros(1, dtype=torch.int64, device="cuda") for _ in range(world)]
        dist.all_gather(allm, meta)
        lens = [int(x.item()) for x in allm]
        seg_meta = [(s.name_len, s.line_count, s.text_bytes, s.stream_offset - 4, s.stream_bytes, s.n_blocks,
                     s.combined_crc, name) for name, s in segs]
        obj = [None] * world
        dist.all_gather_object(obj, seg_meta)
        if rank == 0:
            stage = torch.empty(sum(lens), dtype=torch.uint8, device="cuda")
            ops, off = [], 0
            for r in range(world):
                if r == 0:
                    stage[0:lens[0]].copy_(blob)
                else:
                    ops.append(dist.P2POp(dist.irecv, stage[off:off + lens[r]], r))
                off += lens[r]
            for w in dist.batch_isend_irecv(ops) if ops else []:
                w.wait()
            # archive: magic + streams in chromosome (input) order + index
            order = []
            base = 0
            for r in range(world):
                for (nl, lc, tb, so, sb, nbk, crc, name), cid in zip(obj[r], shards[r]):
                    order.append((cid, base + so, sb, name, lc, tb, nbk, crc))
                base += lens[r]
            order.sort()
            total = 4 + sum(o[2] for o in order)
            arch = torch.empty(total + 4096 + 256 * len(order), dtype=torch.uint8, device="cuda")
            arch[0:4] = torch.tensor(list(starch_amd.MAGIC), dtype=torch.uint8, device="cuda")
            pos = 4
            out_segs, names = [], []
            for cid, src, sb, name, lc, tb, nbk, crc in order:
                arch[pos:pos + sb].copy_(stage[src:src + sb])
                out_segs.append(starch_amd.Segment(line_count=lc, text_bytes=tb, stream_offset=pos, stream_bytes=sb,
                                                   name_len=len(name), n_blocks=nbk, combined_crc=crc))
                names.append(name)
                pos += sb
            idx = starch_amd.build_index(out_segs, names, pos)
            arch[pos:pos + len(idx)] = torch.frombuffer(bytearray(idx), dtype=torch.uint8).to("cuda")
            return arch[:pos + len(idx)]
        else:
            ops = [dist.P2POp(dist.isend, blob.contiguous(), 0)]
            for w in dist.batch_isend_irecv(ops):
                w.wait()
            return None

    def log(msg):
        if rank == 0:
            print("[bench] %s" % msg, file=sys.stderr, flush=True)

    log("input %.1f MB generated + copied to HBM in %.1f s; warmup %d" % (my_bytes / 1e6, t_gen, args.warmup))
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    stats_acc = []
    for _ in range(args.steps):
        step()
        stats_acc.append(ctx.stats())
        log("step: %.1f ms (device %.1f ms)" % ((time.perf_counter() - t0) * 1e3, stats_acc[-1]["ms_total"]))
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([dt], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    ms_step = dt / args.steps * 1e3
    value = total_bytes / (dt / args.steps) / 1e6

    if rank != 0:
        if dist is not None:
            dist.barrier()
            dist.destroy_process_group()
        return

    st = stats_acc[-1]
    bwt_ms = sum(s["ms_bwt"] for s in stats_acc) / len(stats_acc)
    # algorithmic bytes of the block sort: SURVEY §8(d) BWT work figure,
    # sum over SORTED blocks of (1 + doubling rounds) x n x 16 B (key + index,
    # read + write).  Blocks that reuse a byte-identical block's result
    # (dedup_blocks) are not sorted; their share of rle_bytes is taken as
    # proportional to their count.
    nblk = max(1, st["n_blocks"])
    sorted_blk = max(1, nblk - st["dedup_blocks"])
    rle_sorted = st["rle_bytes"] * sorted_blk / nblk
    bwt_bytes = 16.0 * rle_sorted * (1.0 + st["bwt_rounds"] / sorted_blk)
    achieved = bwt_bytes / (bwt_ms / 1e3) / 1e9 if bwt_ms > 0 else 0.0
    pipe_bytes = st["input_bytes"] + 2 * st["text_bytes"] + st["archive_bytes"]
    pipe_achieved = pipe_bytes / (st["ms_total"] / 1e3) / 1e9 if st["ms_total"] > 0 else 0.0
    traffic = None
    pmc = os.path.join(ROOT, "profiles", "pmc_k_bwt.json")
    # the committed PMC pass was taken on the default workload (cfg2, one GPU)
    if os.path.exists(pmc) and args.kind == 0 and args.lines == TOTAL_LINES and world == 1:
        try:
            traffic = json.load(open(pmc)).get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    cpu = None
    names = [starch_amd.HG38[c] for c in mine]
    if not args.no_cpu_baseline and world == 1:
        if args.kind == 2:
            pieces = _perpos_prefixes(names, args.cpu_sample_lines)
        else:
            pieces = _chrom_prefixes(host[:my_bytes].numpy().tobytes(), names, args.cpu_sample_lines)
        cpu = cpu_baseline(pieces, args.cpu_threads, WORKLOADS[args.kind][0].split(":")[0])

    verify = None
    if args.verify and world == 1:
        # bit-identity of two whole chromosome streams against the CPU path
        from tests import oracle_lib
        arch = ctx.archive()
        idx, streams = starch_amd.parse_archive(arch)
        verify = {}
        if args.kind == 2:
            # per-position text of a chromosome of L positions is "p1\n" + "0\n" * L;
            # check by decompression (libbz2 -9 on 100 MB of it takes minutes)
            import bz2 as pybz2
            for nm in ("chr21", "chrY"):
                k = [m["chromosome"] for m in idx["streams"]].index(nm)
                L = starch_amd.HG38_LEN[starch_amd.HG38.index(nm)]
                verify[nm] = pybz2.decompress(streams[k]) == b"p1\n" + b"0\n" * L
        else:
            data = host[:my_bytes].numpy().tobytes()
            for nm in ("chr21", "chr22"):
                k = [m["chromosome"] for m in idx["streams"]].index(nm)
                piece = _chrom_prefixes(data, [nm], 1 << 40)[0]
                _, segs = oracle_lib.transform(piece)
                ref = oracle_lib.ref_bz2(segs[0][2], 9) if oracle_lib.ref() else oracle_lib.bz2(segs[0][2], 9)
                verify[nm] = (streams[k] == ref)

    workload, data_desc = WORKLOADS[args.kind]
    if args.kind != 2 and args.lines != TOTAL_LINES:
        workload = "kind=%d lines=%d" % (args.kind, args.lines)
    line = {
        "metric": "input BED MB/s (%s, bzip2 -9, archive bit-identical to CPU starch3 path)" % workload.split(":")[0],
        "value": round(value, 2),
        "unit": "MB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "u8",
        "data": data_desc,
        "config": {"workload": workload,
                   "input_bytes": total_bytes, "lines": st["n_lines"] if world == 1 else args.lines,
                   "parallelism": "chromosome-shard x%d" % world,
                   "blocks": st["n_blocks"], "text_bytes": st["text_bytes"], "archive_bytes": st["archive_bytes"]},
        "roofline": {"bound": "hbm", "kernel": "k_bwt (block sort)", "achieved": round(achieved, 1),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic, "alg_bytes_per_launch": bwt_bytes, "ms_per_launch": round(bwt_ms, 3)},
        "pipeline_roofline": {"alg_bytes": pipe_bytes, "achieved": round(pipe_achieved, 1), "unit": "GB/s",
                              "frac": round(pipe_achieved / HBM_PEAK_GBS, 4)},
        "bwt": {k: st[k] for k in ("n_blocks", "dedup_blocks", "bwt_rounds", "bwt_tied", "periodic_blocks")},
        "stage_ms": {k: round(st[k], 3) for k in ("ms_transform", "ms_rle", "ms_bwt", "ms_mtf", "ms_tables",
                                                   "ms_emit", "ms_total")},
        "cpu_baseline": cpu,
        "verify": verify,
        "gen_seconds": round(t_gen, 2),
    }
    print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
