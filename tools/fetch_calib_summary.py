#!/usr/bin/env python3
"""Summarise tools/probes/fetch_calib.hip under rocprofv3 (FETCH_SIZE and
WRITE_SIZE passes): counter bytes per access of every probe kernel, from the
second repetition (warm code, cold data).  usage: fetch_calib_summary.py DIR OUT"""
import collections
import csv
import glob
import json
import os
import sys

N = 8 << 20           # accesses per gather / scatter kernel
STREAM = 1 << 30      # bytes of stream16


def per_kernel(d, counter):
    rows = collections.defaultdict(list)   # kernel -> values in dispatch order
    for f in glob.glob(os.path.join(d, "**", "run_counter_collection.csv"), recursive=True):
        rs = [r for r in csv.DictReader(open(f)) if r["Counter_Name"] == counter]
        rs.sort(key=lambda r: int(r.get("Dispatch_Id", 0) or 0))
        for r in rs:
            rows[r["Kernel_Name"].split("(")[0].replace("void ", "")].append(float(r["Counter_Value"]) * 1024.0)
    return {k: v[-1] for k, v in rows.items()}


def main():
    d, out = sys.argv[1], sys.argv[2]
    f = per_kernel(os.path.join(d, "fetch"), "FETCH_SIZE")
    w = per_kernel(os.path.join(d, "write"), "WRITE_SIZE")
    res = {"accesses": N, "stream_bytes": STREAM, "fetch_bytes": f, "write_bytes": w,
           "fetch_per_access": {k: v / N for k, v in f.items() if k != "stream16" and k != "stream4w"},
           "write_per_access": {k: v / N for k, v in w.items() if k.startswith("scatter")},
           "stream16_fetch_over_bytes": f.get("stream16", 0) / STREAM,
           "method": "tools/probes/fetch_calib.hip: each gather/scatter kernel touches 8 Mi distinct 128-B lines "
                     "(gpair8: 4 Mi lines, both 64-B halves) of a 4 GiB buffer once, behind a 1 GiB streamed write "
                     "that evicts the Infinity Cache; rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
