#!/usr/bin/env python3
"""Per-kernel time per step from a rocprofv3 --kernel-trace --stats CSV.
usage: kstats.py [CSV] [STEPS] [TOP]   (defaults: gpurun_out/prof/run_kernel_stats.csv 3 22)"""
import csv
import sys


def main():
    path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof/run_kernel_stats.csv"
    steps = float(sys.argv[2]) if len(sys.argv) > 2 else 3.0
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 22
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    tot = sum(float(r["TotalDurationNs"]) for r in rows) / 1e6 / steps
    for r in rows[:top]:
        name = r["Name"].replace("(anonymous namespace)::", "").replace("void ", "")
        print("%-64s %6d %9.3f ms/step" % (name[:64], int(r["Calls"]), float(r["TotalDurationNs"]) / 1e6 / steps))
    print("%-64s %6s %9.3f ms/step" % ("(all kernels)", "", tot))


if __name__ == "__main__":
    main()
