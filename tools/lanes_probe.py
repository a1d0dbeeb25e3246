#!/usr/bin/env python3
"""Dev probe (GPU box): does one MI355X encode faster with the cfg2 input
split over K contexts (streams) running concurrently?  Each context encodes
an LPT share of the 24 chromosome units (encode_units_device) in its own host
thread; prints the wall time per step for K = 1, 2, 3, 4."""
import ctypes
import os
import sys
import threading
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import starch_amd  # noqa: E402


def main():
    lines = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
    sizes = starch_amd.gen_bed_sizes(0, lines, list(range(24)), seed=20261015)
    n = sum(sizes)
    host = torch.empty(n + 64, dtype=torch.uint8, pin_memory=True)
    starch_amd.gen_bed(0, lines, list(range(24)), seed=20261015, into=ctypes.c_void_p(host.data_ptr()))
    dev = host.to("cuda")
    units, off = [], 0
    for sz in sizes:
        units.append(starch_amd.Unit(off, sz, 0, 0))
        off += sz
    ctxs = [starch_amd.Starch(0) for _ in range(4)]
    for K in (1, 2, 3, 4):
        shard = starch_amd.assign_shards(units, K)
        mine = [[u for u in range(24) if shard[u] == k] for k in range(K)]

        def run(k):
            ctxs[k].encode_units_device(dev.data_ptr(), [units[u] for u in mine[k]], mine[k])

        ts = []
        for rep in range(4):
            torch.cuda.synchronize()
            t = time.perf_counter()
            th = [threading.Thread(target=run, args=(k,)) for k in range(K)]
            for x in th:
                x.start()
            for x in th:
                x.join()
            ts.append(time.perf_counter() - t)
        best = min(ts[1:])
        print("K=%d: %s ms  best %.2f ms = %.1f GB/s" % (K, " ".join("%.1f" % (x * 1e3) for x in ts), best * 1e3,
                                                        n / best / 1e9), flush=True)


if __name__ == "__main__":
    main()
