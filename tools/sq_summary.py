#!/usr/bin/env python3
"""Per-kernel SQ / GRBM counter summary of tools/sq_counters.sh passes
(tools only). Derived ratios, per dispatch (MI355X_MICROARCH.md: SQ_WAVE_CYCLES
/ SQ_ACTIVE_INST_* / SQ_WAIT_* count quad-cycles, SQ_VALU_MFMA_BUSY_CYCLES and
GRBM_GUI_ACTIVE count cycles, GRBM_GUI_ACTIVE summed over the 8 XCDs):
  cycles        = GRBM_GUI_ACTIVE / 8 (the dispatch's GPU-busy cycles)
  valu_busy     = 4 * SQ_ACTIVE_INST_VALU / (cycles * 1024 SIMDs)
  salu_busy     = SQ_INST_CYCLES_SALU / (cycles * 256 CUs)   (rocprofv3's SALUBusy expression; one
                  scalar unit per CU; null when the counter is not collected)
  sca_active_per_cu = 4 * SQ_ACTIVE_INST_SCA / (cycles * 256 CUs)   (waves' SALU + SMEM issue cycles per CU)
  lds_busy      = 4 * SQ_ACTIVE_INST_LDS / (cycles * 256 CUs)
  mfma_busy     = SQ_VALU_MFMA_BUSY_CYCLES / (cycles * 1024 SIMDs)
  wait_frac     = SQ_WAIT_ANY / SQ_WAVE_CYCLES, issue_stall_frac = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES,
  active_frac   = SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES
  waves_per_cu  = SQ_WAVE_CYCLES / (cycles / 4) / 256 (mean resident waves per CU)"""
import collections
import csv
import glob
import json
import os
import sys


def main(out, leg):
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(lambda: collections.defaultdict(set))
    for d in sorted(glob.glob(os.path.join(out, f"sq_{leg}_*"))):
        if not os.path.isdir(d):
            continue
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"].split("(")[0].replace("void ", "")
                tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[k][r["Counter_Name"]].add(r["Dispatch_Id"])
    res = {"leg": leg, "formulas": __doc__.split("per dispatch", 1)[1].strip(), "kernels": {}}
    for k, c in tot.items():
        per = {n: v / max(1, len(disp[k][n])) for n, v in c.items()}
        cyc = per.get("GRBM_GUI_ACTIVE", 0) / 8
        dv = {"dispatches": max(len(s) for s in disp[k].values()), "counters_per_dispatch": per}
        # a ratio whose counter was not collected is null, never 0
        def ratio(name, scale):
            return scale * per[name] if name in per else None
        if cyc > 0:
            dv["cycles"] = cyc
            dv["valu_busy"] = ratio("SQ_ACTIVE_INST_VALU", 4 / (cyc * 1024))
            # rocprofv3's own SALUBusy: SQ_INST_CYCLES_SALU / CU_NUM / GRBM_GUI_ACTIVE (per XCD);
            # SQ_ACTIVE_INST_SCA (quad-cycles of SALU + SMEM per wave) beside it
            dv["salu_busy"] = ratio("SQ_INST_CYCLES_SALU", 1 / (cyc * 256))
            dv["sca_active_per_cu"] = ratio("SQ_ACTIVE_INST_SCA", 4 / (cyc * 256))
            dv["lds_busy"] = ratio("SQ_ACTIVE_INST_LDS", 4 / (cyc * 256))
            dv["mfma_busy"] = ratio("SQ_VALU_MFMA_BUSY_CYCLES", 1 / (cyc * 1024))
            dv["waves_per_cu"] = ratio("SQ_WAVE_CYCLES", 1 / (cyc / 4) / 256)
        wc = per.get("SQ_WAVE_CYCLES", 0)
        if wc:
            dv["wait_frac"] = ratio("SQ_WAIT_ANY", 1 / wc)
            dv["issue_stall_frac"] = ratio("SQ_WAIT_INST_ANY", 1 / wc)
            dv["lds_issue_stall_frac"] = ratio("SQ_WAIT_INST_LDS", 1 / wc)
            dv["active_frac"] = ratio("SQ_ACTIVE_INST_ANY", 1 / wc)
        res["kernels"][k] = dv
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "2ply_k4")
