#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (tools only) into
per-launch HBM bytes per leg and kernel group, with the gfx950 correction of
MI355X_MICROARCH.md (HBM section): FETCH_SIZE reads 1/2 of wide coalesced
streaming reads, so hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.
A bench "movegen launch" is tier 1 + tier 2 (movegen_few/lds + movegen_block);
the 2-ply leg has two movegen launches and two MLP launches per step. The
fused 1-ply leg is one bgx::fused_step_kernel dispatch per 300 steps; its
bytes are also given per step (bench.py scales them to its own launches)."""
FUSED_STEPS_PER_DISPATCH = 300
import collections
import csv
import glob
import json
import os
import sys


def per_kernel(path):
    f = glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        return {}
    acc = collections.defaultdict(lambda: [0.0, set()])
    for r in csv.DictReader(open(f[0])):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        acc[name][0] += float(r["Counter_Value"])
        acc[name][1].add(r["Dispatch_Id"])
    return {k: (v[0], len(v[1])) for k, v in acc.items()}


def group(name):
    if "fused_step" in name:
        return "fused"
    return "mlp" if "mlp_kernel" in name else "movegen"


def main(out):
    res = {"round": os.path.basename(os.path.normpath(out)),
           "workload": "bench.py defaults: 8,192 lanes per GPU (l<n>_ legs: n lanes), seeded xavier weights, T=1.5",
           "source": "tools/profile_round.sh: rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), "
                     "fused 1-ply leg (--kernel-include-regex fused_step, 300 steps per dispatch) and 2-ply K=4 leg "
                     "(--kernel-include-regex 'movegen|mlp_kernel', 60 steps); SQ busy ratios from "
                     "tools/sq_counters.sh (sq_<leg>.json)",
           "correction": "hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950: FETCH_SIZE counts 1/2 of wide "
                         "coalesced reads; narrow movegen reads are uncalibrated, the raw value is kept beside it)"}
    # legs at another lane count (tools/profile_round.sh <dir> <lanes>) are l<lanes>_<leg>
    pre = sorted({os.path.basename(d).split("_")[1] + "_" for d in glob.glob(os.path.join(out, "pmc_l*_*"))
                  if os.path.isdir(d)})
    for leg in [p + b for p in [""] + pre for b in ("1ply_fused", "2ply_k4", "2ply_kall")]:
        f = per_kernel(os.path.join(out, f"pmc_{leg}_FETCH_SIZE"))
        w = per_kernel(os.path.join(out, f"pmc_{leg}_WRITE_SIZE"))
        if not f and not w:
            continue
        legd = {"kernels": {}}
        for name in sorted(set(f) | set(w)):
            fk, nf = f.get(name, (0.0, 0))
            wk, nw = w.get(name, (0.0, 0))
            n = max(nf, nw, 1)
            legd["kernels"][name] = {"dispatches": n, "fetch_size_kb_per_dispatch": fk / max(nf, 1),
                                     "write_size_kb_per_dispatch": wk / max(nw, 1)}
        for g in ("movegen", "mlp", "fused"):
            names = [k for k in legd["kernels"] if group(k) == g]
            if not names:
                continue
            # every movegen call ends with one movegen_block_kernel dispatch; every
            # MLP call is one mlp_kernel dispatch
            if g == "movegen":
                n_launch = sum(legd["kernels"][k]["dispatches"] for k in names if "movegen_block" in k)
            elif g == "fused":
                n_launch = sum(legd["kernels"][k]["dispatches"] for k in names)
            else:
                n_launch = sum(legd["kernels"][k]["dispatches"] for k in names)
            fk = sum(legd["kernels"][k]["fetch_size_kb_per_dispatch"] * legd["kernels"][k]["dispatches"] for k in names)
            wk = sum(legd["kernels"][k]["write_size_kb_per_dispatch"] * legd["kernels"][k]["dispatches"] for k in names)
            legd[g] = {"kernels": names, "launches": n_launch,
                       "hbm_bytes_per_launch": (2 * fk + wk) * 1024 / n_launch,
                       "hbm_bytes_per_launch_uncorrected": (fk + wk) * 1024 / n_launch}
            if g == "fused":
                legd[g]["steps_per_launch"] = FUSED_STEPS_PER_DISPATCH
                legd[g]["hbm_bytes_per_step"] = legd[g]["hbm_bytes_per_launch"] / FUSED_STEPS_PER_DISPATCH
        # SQ counter ratios of the same leg's kernels (tools/sq_summary.py)
        sq_leg = leg[:-len("_fused")] if leg.endswith("1ply_fused") else leg
        try:
            sq = json.load(open(os.path.join(out, f"sq_{sq_leg}.json")))["kernels"]
            for g in ("movegen", "mlp", "fused"):
                if g in legd:
                    # the 2-ply tier-1 reply kernel (board-major since round 4; the pool kernel before)
                    ks = [k for k in sq if group(k) == g and (g != "movegen" or "movegen_reply" in k or "movegen_pool" in k)]
                    if ks:
                        k = ks[0]
                        for r in ("valu_busy", "mfma_busy", "lds_busy", "salu_busy", "wait_frac", "issue_stall_frac",
                                  "waves_per_cu"):
                            if sq[k].get(r) is not None:
                                legd[g][r] = sq[k][r]
                        legd[g]["sq_kernel"] = k
        except (OSError, ValueError, KeyError):
            pass
        if leg.startswith("l"):
            legd["lanes"] = int(leg[1:leg.index("_")])
        res[leg] = legd
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
