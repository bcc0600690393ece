#!/bin/bash
# round 4: instruction counts of the reply launch's non-doubles work -- board-major
# on covered roots only (0x81) vs every root as per-roll jobs (0x101) -- one PMC pass each
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4i; mkdir -p $O
for cfg in "cov:0x81" "unc:0x101" "dbl:0x7e"; do
  tag=${cfg%%:*}; g=${cfg#*:}
  rm -rf $O/pmc_$tag
  BGX_REPLY_GROUPS=$g BGX_MG_FEW=0 timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-include-regex movegen_reply -d $O/pmc_$tag -o run --output-format csv -- python tools/reply_micro.py 32768 child > $O/pmc_$tag.log 2>&1 || { tail -5 $O/pmc_$tag.log; exit 1; }
  python - $O/pmc_$tag $tag <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(float); disp = set()
for r in csv.DictReader(open(f)):
    disp.add(r.get("Dispatch_Id")); acc[r["Counter_Name"]] += float(r["Counter_Value"])
n = len(disp)
print(sys.argv[2], "dispatches", n, {k: round(v / n / 32768, 1) for k, v in sorted(acc.items())}, "(per board)")
PY
done
