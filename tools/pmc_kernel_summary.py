#!/usr/bin/env python3
"""Per-kernel sums of rocprofv3 --pmc counters (tools/gpu_pmc.sh output).

usage: pmc_kernel_summary.py REGEX [PMC_DIR]
For every kernel whose name matches REGEX: the counters of every pass under
PMC_DIR (default gpurun_out/pmc), summed over its dispatches, plus per-wave
instruction counts and the wait / busy ratios the SQ counters give.
"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def main():
    rx = re.compile(sys.argv[1])
    root = sys.argv[2] if len(sys.argv) > 2 else "gpurun_out/pmc"
    tot = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for f in glob.glob(os.path.join(root, "*", "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                name = re.sub(r"\(.*", "", r["Kernel_Name"].replace("(anonymous namespace)", "anon"))
                if not rx.search(r["Kernel_Name"]):
                    continue
                tot[name][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[name].add((f, r["Dispatch_Id"]))
    for name, c in tot.items():
        print("%s  (%d dispatch records)" % (name, len(disp[name])))
        for k in sorted(c):
            print("  %-24s %.4g" % (k, c[k]))
        w = c.get("SQ_WAVES", 0)
        if w:
            for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR",
                      "SQ_INSTS_BRANCH", "SQ_INSTS_SMEM"):
                if k in c:
                    print("  per wave %-16s %.1f" % (k[9:], c[k] / w))
        if c.get("SQ_WAVE_CYCLES"):
            print("  wait_inst_any / wave_cycles %.3f" % (c.get("SQ_WAIT_INST_ANY", 0) / c["SQ_WAVE_CYCLES"]))
        if c.get("SQ_BUSY_CYCLES"):
            for k in ("SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_WAIT_INST_LDS"):
                if k in c:
                    print("  %s / busy %.3f" % (k, c[k] / c["SQ_BUSY_CYCLES"]))


if __name__ == "__main__":
    main()
