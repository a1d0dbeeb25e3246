#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter CSVs per kernel (sum over dispatches).
usage: pmc_summary.py DIR [DIR...]   (each DIR holds run_counter_collection.csv)"""
import collections
import csv
import glob
import re
import sys


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"^void ", "", name)
    return name.split("(")[0][:34]


def main():
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for d in sys.argv[1:]:
        for f in glob.glob(d + "/**/run_counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                agg[short(r["Kernel_Name"])][r["Counter_Name"]] += float(r["Counter_Value"])
    key = lambda kv: -max(kv[1].values())
    for k, v in sorted(agg.items(), key=key):
        print("%-34s " % k + " ".join("%s=%.3g" % (c.replace("SQ_", ""), x) for c, x in sorted(v.items())))


if __name__ == "__main__":
    main()
