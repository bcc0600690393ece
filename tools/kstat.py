#!/usr/bin/env python3
"""Print average durations of kernels matching a substring from a rocprofv3 kernel_stats.csv (tools only)."""
import csv
import sys

for r in csv.DictReader(open(sys.argv[1])):
    if sys.argv[2] in r["Name"]:
        print(sys.argv[3] if len(sys.argv) > 3 else "", r["Name"][:44], "calls", r["Calls"],
              "avg_us", round(float(r["AverageNs"]) / 1e3, 1))
