#!/usr/bin/env python3
"""Per-stream SHA-256 pins for the full-size configs:

  cfg2  100 M-line 24-chromosome BED3     (kind 0, 100,000,000 lines)
  cfg4  50 M-row narrowPeak BED6+4        (kind 1,  50,000,000 lines)
  cfg5  3.09 G-line per-position BED      (kind 2, every base of hg38)

Run HERE (CPU container), not on the GPU box.  The input comes from the
library's seeded generator (starch_gen_bed, host code); each chromosome's
expected stream is the CPU path: the oracle transform (oracle/starch_oracle.c)
then the reference's own vendored libbz2 1.0.6 at -9 (oracle/_ref/
libbz2ref.so, built from /root/reference by oracle/build_ref.sh).  cfg5's
73.6 GB input is never materialised: the transform of a per-position
chromosome of L bases is exactly b"p1\\n" + b"0\\n" * L (first line cd = 1 ->
"p1", start 0; every later line starts where the previous one stopped), and
that identity is itself checked on a prefix of the generated input.

Writes tests/golden/fullsize_cfg{2,4,5}.json: for every chromosome its name,
input bytes, line count, transformed bytes, stream bytes and stream SHA-256.
"""
import argparse
import hashlib
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import starch_amd  # noqa: E402
from tests import oracle_lib  # noqa: E402

CFGS = {"cfg2": (0, 100_000_000), "cfg4": (1, 50_000_000), "cfg5": (2, 0)}
SEED = 20261015


def bz2_ref(text):
    return oracle_lib.ref_bz2(text, 9) if oracle_lib.ref() is not None else oracle_lib.bz2(text, 9)


def one_chrom(kind, total, c):
    name = starch_amd.HG38[c]
    if kind == 2:
        L = starch_amd.HG38_LEN[c]
        text = b"p1\n" + b"0\n" * L
        inp_bytes = starch_amd.gen_bed_sizes(2, 0, [c])[0]
        lines = L
    else:
        data = starch_amd.gen_bed(kind, total, chroms=[c], seed=SEED)
        _, segs = oracle_lib.transform(data)
        assert len(segs) == 1 and segs[0][0] == name.encode(), name
        text, lines, inp_bytes = segs[0][2], segs[0][1], len(data)
        del data
    st = bz2_ref(text)
    return {"chromosome": name, "input_bytes": inp_bytes, "lines": lines, "text_bytes": len(text),
            "stream_bytes": len(st), "sha256": hashlib.sha256(st).hexdigest()}


def check_perpos_identity():
    """transform(per-position prefix) == p1 + 0\\n * k, on two chromosomes."""
    for c in (13, 23):
        k = 200_000
        name = starch_amd.HG38[c].encode()
        data = b"".join(b"%s\t%d\t%d\n" % (name, p, p + 1) for p in range(k))
        _, segs = oracle_lib.transform(data)
        assert segs[0][2] == b"p1\n" + b"0\n" * k


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("cfgs", nargs="*", default=["cfg2", "cfg4", "cfg5"])
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 8)
    args = ap.parse_args()
    for cfg in args.cfgs:
        kind, total = CFGS[cfg]
        if kind == 2:
            check_perpos_identity()
        t0 = time.time()
        # longest chromosomes first so the pool drains evenly
        order = sorted(range(24), key=lambda c: -starch_amd.HG38_LEN[c])
        with ThreadPoolExecutor(args.threads) as ex:
            res = dict(zip(order, ex.map(lambda c: one_chrom(kind, total, c), order)))
        streams = [res[c] for c in range(24)]
        out = {"config": cfg, "kind": kind, "total_lines": total, "seed": SEED,
               "bzip2": ("reference libbz2 %s (oracle/_ref)" % oracle_lib.ref().ref_bz2_version().decode())
               if oracle_lib.ref() is not None else "oracle restatement",
               "input_bytes": sum(s["input_bytes"] for s in streams),
               "streams": streams}
        path = os.path.join(ROOT, "tests", "golden", "fullsize_%s.json" % cfg)
        with open(path, "w") as f:
            json.dump(out, f, indent=1)
        print("%s: %d streams, %.1f s -> %s" % (cfg, len(streams), time.time() - t0, path), flush=True)


if __name__ == "__main__":
    main()
