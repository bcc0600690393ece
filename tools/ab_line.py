#!/usr/bin/env python3
"""One summary line of a bench.py JSON output (tools only): value, ms/step and
the movegen / MLP / fused launch averages of the main leg and the 2-ply legs."""
import json
import sys

d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])


def leg(x):
    k = x.get("kernels", {})
    parts = [f"{x['value'] / 1e6:.3f}M", f"{x['ms_per_step']:.4f}ms/step"]
    for name in ("movegen", "mlp", "fused_step"):
        if name in k:
            parts.append(f"{name} {k[name]['avg_launch_ms']:.4f}ms")
    return " ".join(parts)


out = [sys.argv[1], "main:", leg(d)]
for key in ("two_ply_k4", "two_ply_kall"):
    if key in d:
        out += [f"| {key}:", leg(d[key])]
if d.get("cpu_baseline"):
    out.append(f"| cpu {d['cpu_baseline']['value']:.0f}/s")
print(" ".join(out))
