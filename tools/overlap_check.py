#!/usr/bin/env python3
"""Span check of a rocprofv3 --kernel-trace --memory-copy-trace run of
tools/overlap_probe.py: for every device-to-host copy, the fused launch (if
any) whose [start, end] contains it. Prints a JSON summary. Tools only."""
import csv
import glob
import json
import os
import sys


def rows(d, pat):
    f = glob.glob(os.path.join(d, "**", pat), recursive=True)
    return list(csv.DictReader(open(f[0]))) if f else []


def main(d):
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows(d, "*kernel_trace.csv")]
    fused = [(s, e) for s, e, n in ks if "fused_step" in n]
    cps = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Direction", r.get("Operation", "")),
            int(r.get("Size", r.get("Bytes", 0)) or 0)) for r in rows(d, "*memory_copy_trace.csv")]
    out = {"fused_launches": len(fused), "copies": []}
    for s, e, kind, size in cps:
        inside = [i for i, (fs, fe) in enumerate(fused) if fs <= s and e <= fe]
        out["copies"].append({"kind": kind, "bytes": size, "us": (e - s) / 1e3,
                              "inside_fused_launch": inside[0] if inside else None})
    sized = any(c["bytes"] for c in out["copies"])
    big = [c for c in out["copies"] if c["bytes"] >= 1 << 20] if sized else out["copies"]
    out["columns"] = list(rows(d, "*memory_copy_trace.csv")[0].keys()) if cps else []
    out["large_copies"] = len(big)
    out["large_copies_inside_a_fused_launch"] = sum(c["inside_fused_launch"] is not None for c in big)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
