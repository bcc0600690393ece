# instruction counts per movegen job kind (pool kernel, mg_micro job sets): one PMC pass per kind
set -o pipefail
export TMPDIR=/tmp; OUT=gpurun_out/${1:-mgk}; mkdir -p $OUT
for kind in nondoubles doubles; do
  rm -rf $OUT/pmc_$kind
  timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES --kernel-include-regex movegen_pool -d $OUT/pmc_$kind -o run --output-format csv -- python tools/mg_micro.py 300000 $kind > $OUT/pmc_$kind.log 2>&1 || { tail -5 $OUT/pmc_$kind.log; exit 1; }
  python - $OUT/pmc_$kind $kind <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(float); disp = set()
for r in csv.DictReader(open(f)):
    disp.add(r.get("Dispatch_Id")); acc[r["Counter_Name"]] += float(r["Counter_Value"])
n = len(disp)
print(sys.argv[2], "dispatches", n, {k: round(v / n / 300000, 1) for k, v in sorted(acc.items())})
PY
done
