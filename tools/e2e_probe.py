#!/usr/bin/env python3
"""Dev probe (GPU box): host -> host encode (starch_encode_host_into) of cfg2
from pinned memory, median of REPS calls after one warmup; the pipelined
path's knobs come from the environment (STARCH_PIPE_BATCHES, STARCH_LANES,
STARCH_PIPE_FIRST).  Prints one line."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import ctypes
    import torch
    import starch_amd
    lines = int(os.environ.get("LINES", "100000000"))
    n = sum(starch_amd.gen_bed_sizes(0, lines))
    host = torch.empty(n + 64, dtype=torch.uint8, pin_memory=True)
    starch_amd.gen_bed(0, lines, into=ctypes.c_void_p(host.data_ptr()))
    t = time.perf_counter()
    c = starch_amd.Starch(0)
    if os.environ.get("COLD"):
        print("create: %.1f ms" % ((time.perf_counter() - t) * 1e3), flush=True)
    out = torch.empty(n // 2 + (16 << 20), dtype=torch.uint8, pin_memory=not os.environ.get("OUT_PAGEABLE"))
    if os.environ.get("COLD"):   # first calls of a fresh context: a small input first (SMALL=lines), then the whole
        small = int(os.environ.get("SMALL", "0"))
        if small:
            ns = sum(starch_amd.gen_bed_sizes(0, small))
            t = time.perf_counter()
            c.compress_host_into(host.data_ptr(), ns, out.data_ptr(), out.numel())
            print("cold small (%d B): %.1f ms" % (ns, (time.perf_counter() - t) * 1e3), flush=True)
        for k in range(3):
            t = time.perf_counter()
            c.compress_host_into(host.data_ptr(), n, out.data_ptr(), out.numel())
            print("call %d: %.1f ms" % (k, (time.perf_counter() - t) * 1e3), flush=True)
        return
    c.compress_host_into(host.data_ptr(), n, out.data_ptr(), out.numel())
    ts = []
    for _ in range(int(os.environ.get("REPS", "5"))):
        t = time.perf_counter()
        c.compress_host_into(host.data_ptr(), n, out.data_ptr(), out.numel())
        ts.append(time.perf_counter() - t)
    ts.sort()
    dt = ts[len(ts) // 2]
    knobs = {k: os.environ[k] for k in ("STARCH_PIPE_BATCHES", "STARCH_LANES", "STARCH_PIPE_FIRST") if k in os.environ}
    print("e2e %s: %.1f ms %.1f GB/s (all %s)" % (knobs, dt * 1e3, n / dt / 1e9, [round(x * 1e3, 1) for x in ts]),
          flush=True)
    c.close()


if __name__ == "__main__":
    main()
