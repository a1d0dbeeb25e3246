#!/usr/bin/env python3
"""Dev probe (GPU box): does encoding two halves of cfg2 concurrently on two
contexts (two HIP streams, two host threads) beat one context encoding the
whole input?  Prints ms per configuration (median of REPS)."""
import ctypes
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import starch_amd
    lines = int(os.environ.get("LINES", "100000000"))
    reps = int(os.environ.get("REPS", "7"))
    sizes = starch_amd.gen_bed_sizes(0, lines)
    n = sum(sizes)
    host = torch.empty(n + 64, dtype=torch.uint8, pin_memory=True)
    starch_amd.gen_bed(0, lines, into=ctypes.c_void_p(host.data_ptr()))
    dev = host.to("cuda")
    units, off = [], 0
    for sz in sizes:
        units.append(starch_amd.Unit(off, sz, 0, 0))
        off += sz
    ids = list(range(len(units)))
    one = starch_amd.Starch(0)
    res = {}

    def timed(fn):
        ts = []
        for _ in range(reps + 1):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        ts = sorted(ts[1:])
        return round(ts[len(ts) // 2] * 1e3, 3)

    res["one_ctx_units"] = timed(lambda: one.encode_units_device(dev.data_ptr(), units, ids))
    res["one_ctx_device"] = timed(lambda: one.compress_device(dev.data_ptr(), n))
    for k in (2, 3):
        shard = starch_amd.assign_shards(units, k)
        parts = [[i for i in ids if shard[i] == s] for s in range(k)]
        ctxs = [starch_amd.Starch(0) for _ in range(k)]

        def run():
            th = [threading.Thread(target=lambda c=c, p=p: c.encode_units_device(dev.data_ptr(), [units[i] for i in p], p))
                  for c, p in zip(ctxs, parts)]
            for t in th:
                t.start()
            for t in th:
                t.join()
        res["%d_ctx_concurrent" % k] = timed(run)
        for c in ctxs:
            c.close()
    res["input_mb"] = round(n / 1e6, 1)
    print(res, flush=True)


if __name__ == "__main__":
    main()
