#!/usr/bin/env python3
"""Split a rocprofv3 kernel trace of tools/window_probe.py into its windows
(gaps > 5 ms) and print, per window, each kernel's duration and the idle
gaps between them (us). Tools only."""
import csv
import glob
import json
import os
import sys

rows = list(csv.DictReader(open(glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True)[0])))
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][-40:]) for r in rows)
wins, cur = [], [ks[0]]
for k in ks[1:]:
    if k[0] - cur[-1][1] > 5_000_000:
        wins.append(cur)
        cur = [k]
    else:
        cur.append(k)
wins.append(cur)
out = []
for wv in wins[-10:]:
    seq, prev = [], None
    for s, e, n in wv:
        if prev is not None:
            seq.append(["gap", round((s - prev) / 1e3, 1)])
        seq.append([n, round((e - s) / 1e3, 1)])
        prev = e
    out.append({"span_us": round((wv[-1][1] - wv[0][0]) / 1e3, 1), "seq": seq})
print(json.dumps(out, indent=1))
