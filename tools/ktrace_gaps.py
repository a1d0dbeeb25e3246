#!/usr/bin/env python3
"""Dev tool: the last encode of a rocprofv3 --kernel-trace CSV in launch
order -- each dispatch's start (us from the step start), duration and the idle
gap before it, so host syncs and small launches show up.
usage: ktrace_gaps.py run_kernel_trace.csv"""
import csv
import sys


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    first = [i for i, r in enumerate(rows) if "k_tf_fused" in r["Kernel_Name"] or "k_tf1" in r["Kernel_Name"]]
    s = first[-1]
    e = [i for i, r in enumerate(rows) if "k_stream_frame" in r["Kernel_Name"] and i > s][0]
    step = rows[s:e + 1]
    t0 = int(step[0]["Start_Timestamp"])
    prev_end = t0
    tot_gap = 0
    for r in step:
        a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = max(0, a - prev_end)
        tot_gap += gap
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:48]
        print("%9.1f  dur %8.1f  gap %7.1f  %-48s grid=%s" % ((a - t0) / 1e3, (b - a) / 1e3, gap / 1e3, k,
                                                         r.get("Grid_Size_X", r.get("Grid_Size", ""))))
        prev_end = max(prev_end, b)
    print("span %.1f us, gaps %.1f us, %d dispatches" % ((prev_end - t0) / 1e3, tot_gap / 1e3, len(step)))


if __name__ == "__main__":
    main()
