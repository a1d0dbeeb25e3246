#!/usr/bin/env python3
"""Per-encode fixed cost on a small input (dev tool): cfg1 (10,000-line
single-chromosome BED3) already in HBM, encoded REPS times with
starch_encode_device; prints wall ms per encode (median, min) and the
library's own stage times.  Run under `rocprofv3 --hip-trace --stats` to count
the HIP calls (synchronisations, copies) per encode.
usage: small_cost.py [REPS] [LINES]"""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    lines = int(sys.argv[2]) if len(sys.argv) > 2 else 10000
    import torch
    import starch_amd
    import corpus
    data = corpus.cfg1_bed(lines)
    dev = torch.frombuffer(bytearray(data), dtype=torch.uint8).to("cuda")
    ctx = starch_amd.Starch(0)
    for _ in range(5):
        ctx.compress_device(dev.data_ptr(), len(data))
    torch.cuda.synchronize()
    wall = []
    for _ in range(reps):
        t = time.perf_counter()
        ctx.compress_device(dev.data_ptr(), len(data))
        wall.append((time.perf_counter() - t) * 1e3)
    st = ctx.stats()
    print(json.dumps({"input_bytes": len(data), "lines": lines, "reps": reps,
                      "wall_ms_median": round(statistics.median(wall), 4), "wall_ms_min": round(min(wall), 4),
                      "stats": st}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
