#!/usr/bin/env python3
"""Per-step kernel timeline from a rocprofv3 kernel_trace.csv (tools only):
average duration of each kernel and of the gaps between consecutive kernels
over the last N steps (a step starts at each `start_kernel` dispatch)."""
import collections
import csv
import sys


def main(path, start_kernel="movegen_lds_kernel", last=200):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    steps, cur = [], None
    for r in rows:
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        if start_kernel in name and (cur is None or any(start_kernel in n for n, _, _ in cur)):
            if cur:
                steps.append(cur)
            cur = []
        if cur is not None:
            cur.append((name, int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    steps = steps[-last:]
    dur = collections.defaultdict(list)
    gap = collections.defaultdict(list)
    span = []
    for s in steps:
        for i, (n, a, b) in enumerate(s):
            dur[f"{i:02d} {n}"].append(b - a)
            if i:
                gap[f"{i:02d} before {n}"].append(a - s[i - 1][2])
        span.append(s[-1][2] - s[0][1])
    print(f"{len(steps)} steps; mean span {sum(span) / len(span) / 1e3:.1f} us")
    for k in sorted(dur):
        g = gap.get(k[:3] + "before " + k[3:], [0])
        print(f"{k:60s} dur {sum(dur[k]) / len(dur[k]) / 1e3:8.2f} us   gap-before {sum(g) / len(g) / 1e3:6.2f} us")


if __name__ == "__main__":
    main(sys.argv[1], *(sys.argv[2:3] or []))
