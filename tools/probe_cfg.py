#!/usr/bin/env python3
"""GPU probe: one timed compression of a generated config slice, stats as JSON.

  python tools/probe_cfg.py --kind 1 --lines 50000000            # cfg4
  python tools/probe_cfg.py --kind 2 --chroms 13                 # cfg5, chr21 only
"""
import argparse
import bz2
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kind", type=int, default=1)
    ap.add_argument("--lines", type=int, default=50_000_000)
    ap.add_argument("--chroms", type=str, default="")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--roundtrip", action="store_true", help="bz2-decompress every stream and compare")
    args = ap.parse_args()
    import torch
    import starch_amd
    chroms = [int(x) for x in args.chroms.split(",")] if args.chroms else None
    t0 = time.perf_counter()
    data = starch_amd.gen_bed(args.kind, args.lines, chroms=chroms)
    tg = time.perf_counter() - t0
    host = torch.frombuffer(bytearray(data), dtype=torch.uint8)
    dev = host.to("cuda")
    ctx = starch_amd.Starch(0)
    res = []
    for _ in range(args.reps):
        torch.cuda.synchronize()
        t = time.perf_counter()
        ctx.compress_device(dev.data_ptr(), len(data))
        torch.cuda.synchronize()
        res.append(time.perf_counter() - t)
    st = ctx.stats()
    out = {"kind": args.kind, "lines": args.lines, "chroms": args.chroms, "input_bytes": len(data),
           "gen_s": round(tg, 2), "wall_s": [round(x, 4) for x in res],
           "MBps": round(len(data) / min(res) / 1e6, 1), "stats": st}
    if args.roundtrip:
        arch = ctx.archive()
        idx, streams = starch_amd.parse_archive(arch)
        h = hashlib.sha256()
        for s in streams:
            h.update(bz2.decompress(s))
        out["text_sha256_from_roundtrip"] = h.hexdigest()
        out["archive_sha256"] = hashlib.sha256(arch).hexdigest()
    print(json.dumps(out), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
