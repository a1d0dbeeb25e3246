#!/usr/bin/env python3
"""Dev probe (GPU box): host timeline of the host-input paths on cfg2 --
one-call compress_host_ptr (pipelined unless STARCH_PIPELINE=0) and the
streaming session -- with STARCH_TRACE=1 set before the library loads, so the
library prints its per-batch timeline on stderr.
    STARCH_TRACE=1 python tools/e2e_trace.py [lines]"""
import ctypes
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import starch_amd  # noqa: E402


def main():
    lines = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
    n_est = lines * 26 + (64 << 20)
    host = torch.empty(n_est, dtype=torch.uint8, pin_memory=True)
    n = starch_amd.gen_bed(0, lines, seed=1, into=ctypes.c_void_p(host.data_ptr()))
    ctx = starch_amd.Starch(0)
    for rep in range(2):
        t = time.perf_counter()
        ctx.compress_host_ptr(host.data_ptr(), n)
        dt = time.perf_counter() - t
        print("one-call rep %d: %.1f ms, %.1f MB/s, stats ms_total %.1f" % (rep, dt * 1e3, n / dt / 1e6,
              ctx.stats()["ms_total"]), file=sys.stderr, flush=True)
    piece = 64 << 20
    for rep in range(2):
        t = time.perf_counter()
        ctx.stream_begin()
        for off in range(0, n, piece):
            ctx.stream_feed(host.data_ptr() + off, min(piece, n - off))
            ctx.stream_read()
        ctx.stream_end()
        ctx.stream_read()
        dt = time.perf_counter() - t
        print("stream rep %d: %.1f ms, %.1f MB/s" % (rep, dt * 1e3, n / dt / 1e6), file=sys.stderr, flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
