#!/usr/bin/env python3
"""HBM traffic of the block-sort stage from rocprofv3 --pmc passes.

Reads gpurun_out/pmc/{fetch,write}/**/run_counter_collection.csv of ONE bench
step (tools/gpu_pmc.sh, PASSES="fetch write", LINES=100000000), sums the
FETCH_SIZE and WRITE_SIZE (KB) of the block-sort kernels (k3_*, k_fallback*,
k_last_col, scan helpers launched by the sort are not separable and are
excluded), applies the gfx950 correction FETCH_SIZE x 2 and writes profiles/pmc_k_bwt.json,
which bench.py reports as roofline.traffic.  The factor 2 is calibrated for
the block sort's own access widths (tools/probes/fetch_calib.hip,
profiles/r04/fetch_calib.json): a 16-B/lane stream reads 0.500 of its bytes in
FETCH_SIZE, and an 8-B or 16-B gather to its own 128-B line reads 64 units --
the whole line fetched, counted at half -- while two gathers to the halves of
one line read 64 per line, so fetched bytes = 2 x FETCH_SIZE for streams and
gathers alike; WRITE_SIZE is exact for streams (1.000) and counts a partial
line write as one 32-B sector.
usage: pmc_bwt_traffic.py [PMC_DIR] [OUT_JSON]
"""
import collections
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import src_stamp  # noqa: E402


def is_bwt(name):
    n = name.replace("(anonymous namespace)::", "")
    return "k3_" in n or "k_fallback" in n or "k_last_col" in n


KSEL = os.environ.get("PMC_KERNELS", "")     # regex over kernel names (default: the block-sort kernels)


def sums(d, counter):
    import re
    tot = collections.Counter()
    for f in glob.glob(os.path.join(d, "**", "run_counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            sel = re.search(KSEL, r["Kernel_Name"]) if KSEL else is_bwt(r["Kernel_Name"])
            if r["Counter_Name"] == counter and sel:
                tot[r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")] += float(r["Counter_Value"])
    return tot


def main():
    pmc = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
    out = sys.argv[2] if len(sys.argv) > 2 else "profiles/pmc_k_bwt.json"
    f = sums(os.path.join(pmc, "fetch"), "FETCH_SIZE")
    w = sums(os.path.join(pmc, "write"), "WRITE_SIZE")
    fetch_b = 2.0 * sum(f.values()) * 1024.0
    write_b = sum(w.values()) * 1024.0
    res = {
        "src_stamp": src_stamp(),
        "lines": int(os.environ.get("LINES", "100000000")),
        "kind": int(os.environ.get("KIND", "0")),
        "block_reuse": os.environ.get("STARCH_DEDUPE") != "0",
        "hbm_bytes_per_launch": fetch_b + write_b,
        "fetch_bytes": fetch_b,
        "write_bytes": write_b,
        "method": "rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE in separate passes over one bench step (kind/lines above); "
                  "FETCH_SIZE doubled (calibrated for 8/16-B gathers and 16-B streams: profiles/r04/fetch_calib.json); "
                  + ("kernels matching %r summed" % KSEL if KSEL else
                     "block-sort kernels k3_*, k_fallback*, k_last_col summed") + "; Infinity-Cache hits are counted",
        "per_kernel_fetch_bytes": {k: 2.0 * v * 1024.0 for k, v in f.most_common()},
        "per_kernel_write_bytes": {k: v * 1024.0 for k, v in w.most_common()},
    }
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: res[k] for k in ("hbm_bytes_per_launch", "fetch_bytes", "write_bytes")}))


if __name__ == "__main__":
    main()
