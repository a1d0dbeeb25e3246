#!/usr/bin/env python3
"""Transform-stage micro-benchmark on the GPU (dev tool): cfg2/cfg4 input in
HBM, starch_transform_device repeated, HIP-event ms per call; --sha prints the
SHA-256 of the text and of the segment table (compare STARCH_TF=2pass runs)."""
import hashlib
import argparse
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kind", type=int, default=0)
    ap.add_argument("--lines", type=int, default=100_000_000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--sha", action="store_true")
    ap.add_argument("--chroms", default="13,14", help="kind 2: chromosome ids (HG38 order)")
    a = ap.parse_args()
    import torch
    import starch_amd
    if a.kind == 2:   # per-position (cfg5): a few whole chromosomes written by the device generator
        chroms = [int(x) for x in a.chroms.split(",")]
        sizes = [starch_amd.gen_perpos_device(ci) for ci in chroms]
        n = sum(sizes)
        dev = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
        off = 0
        for ci, sz in zip(chroms, sizes):
            starch_amd.gen_perpos_device(ci, dev.data_ptr() + off, n + 64 - off, stream=0)
            off += sz
        torch.cuda.synchronize()
    else:
        n = sum(starch_amd.gen_bed_sizes(a.kind, a.lines))
        host = torch.empty(n + 64, dtype=torch.uint8, pin_memory=True)
        starch_amd.gen_bed(a.kind, a.lines, into=ctypes.c_void_p(host.data_ptr()))
        dev = host.to("cuda")
    c = starch_amd.Starch(0)
    ms = []
    for _ in range(a.reps):
        c.transform_device(dev.data_ptr(), n)
        ms.append(c.stats()["ms_transform"])
    st = c.stats()
    print("kind %d bytes %d lines %d text %d segs %d  ms %s  best %.3f ms = %.1f GB/s" % (
        a.kind, n, st["n_lines"], st["text_bytes"], st["n_segments"], " ".join("%.3f" % x for x in ms), min(ms),
        n / min(ms) / 1e6))
    if a.sha:
        nt = ctypes.c_uint64()
        c._L.starch_text_size(c._h, ctypes.byref(nt))
        out = torch.empty(nt.value + 1, dtype=torch.uint8, pin_memory=True)
        c._L.starch_text_copy(c._h, ctypes.c_void_p(out.data_ptr()), nt.value)
        segs = [(nm, s.line_count, s.stream_offset, s.text_bytes) for nm, s in c.segments()]
        print("text sha256 %s segs sha256 %s" % (hashlib.sha256(out[:nt.value].numpy().tobytes()).hexdigest()[:16],
                                                 hashlib.sha256(repr(segs).encode()).hexdigest()[:16]))


if __name__ == "__main__":
    main()
