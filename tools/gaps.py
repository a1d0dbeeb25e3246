#!/usr/bin/env python3
"""GPU idle time inside each encode of a rocprofv3 kernel trace (dev tool):
per encode (k_tf_fused .. k_stream_frame) the span, the busy time and the
largest idle gaps with the kernels around them.
usage: gaps.py [run_kernel_trace.csv] [min_gap_us]"""
import csv
import sys


def main():
    path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof/run_kernel_trace.csv"
    mg = float(sys.argv[2]) if len(sys.argv) > 2 else 15.0
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    short = lambda n: n.replace("bz::", "").replace("(anonymous namespace)::", "").replace("void ", "")[:38]
    starts = [i for i, r in enumerate(rows) if "k_tf_fused" in r["Kernel_Name"] or "k_tf1" in r["Kernel_Name"]]
    for n, i in enumerate(starts):
        seg = rows[i:starts[n + 1] if n + 1 < len(starts) else len(rows)]
        ends = [q for q, r in enumerate(seg) if "k_stream_frame" in r["Kernel_Name"]]
        if not ends:
            continue
        seg = seg[:ends[-1] + 1]
        t0 = int(seg[0]["Start_Timestamp"])
        end, busy, prev, gaps = t0, 0, "start", []
        for r in seg:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            if s - end > mg * 1000:
                gaps.append(((s - t0) / 1e6, (s - end) / 1e3, short(prev), short(r["Kernel_Name"])))
            busy += max(0, e - max(s, end))
            end = max(end, e)
            prev = r["Kernel_Name"]
        print("encode %d: span %.2f ms, busy %.2f ms, idle %.2f ms" % (n, (end - t0) / 1e6, busy / 1e6,
                                                                      (end - t0 - busy) / 1e6))
        for g in gaps:
            print("   at %7.2f ms: %6.1f us idle after %-38s before %s" % g)


if __name__ == "__main__":
    main()
