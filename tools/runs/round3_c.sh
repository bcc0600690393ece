# Round-3 session, GPU call 3: which device -> host copy path runs on the DMA engines.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5c; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 120 python tools/copy_probe.py > $OUT/copy_plain.log 2>&1 || { tail $OUT/copy_plain.log; exit 1; }
tail -1 $OUT/copy_plain.log
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d $OUT/copy -o run --output-format csv -- python tools/copy_probe.py > $OUT/copy.log 2>&1 || { tail $OUT/copy.log; exit 1; }
python - <<'PY'
import csv, glob, collections
k = list(csv.DictReader(open(glob.glob("gpurun_out/r5c/copy/*kernel_trace.csv")[0])))
mf = glob.glob("gpurun_out/r5c/copy/*memory_copy_trace.csv")
m = list(csv.DictReader(open(mf[0]))) if mf else []
print("kernels:", collections.Counter(x["Kernel_Name"][:40] for x in k))
print("copies:", collections.Counter((x["Direction"] if "Direction" in x else "", x["Kind"]) for x in m))
for x in m:
    print(x["Kind"], x.get("Direction"), (int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e3, "us")
for x in k:
    if "copy" in x["Kernel_Name"].lower():
        print("blit", (int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e3, "us")
PY
