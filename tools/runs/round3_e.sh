# Round-3 session, GPU call 5: do the ROCclr blit-engine knobs route device ->
# host copies to the DMA engines? (copy_probe under kernel + memory-copy trace)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5e; rm -rf $OUT; mkdir -p $OUT
for v in "GPU_BLIT_ENGINE_TYPE=2" "HSA_ENABLE_SDMA=1" "GPU_FORCE_BLIT_COPY_SIZE=0"; do
  n=$(echo $v | cut -d= -f1)
  env $v timeout -k 10 120 python tools/copy_probe.py > $OUT/$n.log 2>&1 || { tail $OUT/$n.log; exit 1; }
  echo "$v: $(tail -1 $OUT/$n.log)"
done
export GPU_BLIT_ENGINE_TYPE=2
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d $OUT/copy -o run --output-format csv -- python tools/copy_probe.py > $OUT/copy.log 2>&1 || { tail $OUT/copy.log; exit 1; }
python - <<'PY'
import csv, glob, collections
k = list(csv.DictReader(open(glob.glob("gpurun_out/r5e/copy/*kernel_trace.csv")[0])))
mf = glob.glob("gpurun_out/r5e/copy/*memory_copy_trace.csv")
m = list(csv.DictReader(open(mf[0]))) if mf else []
print("GPU_BLIT_ENGINE_TYPE=2 kernels:", collections.Counter(x["Kernel_Name"][:40] for x in k))
print("dma copies:", collections.Counter((x.get("Direction", ""), x["Kind"]) for x in m))
for x in m[:12]:
    print(x["Kind"], x.get("Direction"), (int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e3, "us")
PY
