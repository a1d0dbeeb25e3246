#!/usr/bin/env python3
"""Per-kernel time inside the last encode of a rocprofv3 --kernel-trace CSV
(dev tool): the span from the last k_tf_fused/k_tf1 launch to the next
k_stream_frame, kernel busy time, idle gaps, top kernels.
usage: ktrace_step.py run_kernel_trace.csv [TOP]"""
import collections
import csv
import sys


def name(r):
    k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
    return k.split("(")[0][:56]


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
    first = [i for i, r in enumerate(rows) if "k_tf_fused" in r["Kernel_Name"] or "k_tf1" in r["Kernel_Name"]]
    s = first[-1]
    e = [i for i, r in enumerate(rows) if "k_stream_frame" in r["Kernel_Name"] and i > s][0]
    step = rows[s:e + 1]
    t0 = int(step[0]["Start_Timestamp"])
    span = (int(step[-1]["End_Timestamp"]) - t0) / 1e6
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in step) / 1e6
    gaps = sum(max(0, int(step[i]["Start_Timestamp"]) - int(step[i - 1]["End_Timestamp"])) for i in range(1, len(step)))
    print("encode span %.3f ms, %d kernels, busy %.3f ms, idle gaps %.3f ms" % (span, len(step), busy, gaps / 1e6))
    d, n = collections.Counter(), collections.Counter()
    for r in step:
        d[name(r)] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        n[name(r)] += 1
    for k, v in d.most_common(top):
        print("%-58s %3d  %7.3f ms" % (k, n[k], v / 1e6))


if __name__ == "__main__":
    main()
