#!/usr/bin/env python3
"""Value and ms/step of bench.py JSON lines (tools only): one line per file,
then the mean per library tag (file names <prefix>_<lib>_<rep>.json)."""
import collections
import json
import os
import sys

per = collections.defaultdict(list)
for f in sys.argv[1:]:
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except (OSError, ValueError, IndexError):
        print(f"{f}: no JSON line")
        continue
    name = os.path.basename(f)[:-5]
    lib = name.rsplit("_", 1)[0]
    per[lib].append(d["value"] / 1e6)
    print(f"{name:32s} {d['value'] / 1e6:8.2f} M  {d['ms_per_step']:.4f} ms/step")
for lib, v in per.items():
    print(f"mean {lib:27s} {sum(v) / len(v):8.2f} M  (n={len(v)})")
