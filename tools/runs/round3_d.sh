# Round-3 session, GPU call 4: DMA-engine copy kinds; the one-thread-per-lane
# choice phase (default build) vs round 2's half-wave rounds (libbgx_half.so,
# -DBGX_CHOICE_HALF): engine parity tests, then A/B at 20 and 300 steps.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5d; rm -rf $OUT; mkdir -p $OUT
echo "[1] copy kinds"
timeout -k 10 120 python tools/copy_probe.py > $OUT/copy_plain.log 2>&1 || { tail $OUT/copy_plain.log; exit 1; }
tail -1 $OUT/copy_plain.log
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d $OUT/copy -o run --output-format csv -- python tools/copy_probe.py > $OUT/copy.log 2>&1 || { tail $OUT/copy.log; exit 1; }
python - <<'PY'
import csv, glob, collections
k = list(csv.DictReader(open(glob.glob("gpurun_out/r5d/copy/*kernel_trace.csv")[0])))
mf = glob.glob("gpurun_out/r5d/copy/*memory_copy_trace.csv")
m = list(csv.DictReader(open(mf[0]))) if mf else []
print("kernels:", collections.Counter(x["Kernel_Name"][:40] for x in k))
print("dma copies:", collections.Counter((x.get("Direction", ""), x["Kind"]) for x in m))
PY
echo "[2] engine tests"
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_replay.py -x -q --timeout 120 --timeout-method thread > $OUT/engine_tests.log 2>&1 || { tail -40 $OUT/engine_tests.log; exit 1; }
tail -2 $OUT/engine_tests.log
echo "[3] A/B"
for lib in libbgx libbgx_half libbgx libbgx_half; do
  BGX_LIB=$PWD/mlp-ppo-2ply-multi_amd/bgx/$lib.so timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --two-ply-steps 0 --kall-steps 0 --config1-steps 0 > $OUT/${lib}_20.json 2> $OUT/${lib}_20.err || { tail $OUT/${lib}_20.err; exit 1; }
  BGX_LIB=$PWD/mlp-ppo-2ply-multi_amd/bgx/$lib.so timeout -k 10 200 python bench.py --steps 600 --warmup 5 --no-cpu-baseline --two-ply-steps 0 --kall-steps 0 --config1-steps 0 > $OUT/${lib}_600.json 2> $OUT/${lib}_600.err || { tail $OUT/${lib}_600.err; exit 1; }
  python -c "
import json
a=json.load(open('$OUT/${lib}_20.json')); b=json.load(open('$OUT/${lib}_600.json'))
print('$lib', '20:', round(a['value']/1e6,2), '600:', round(b['value']/1e6,2), 'launch600 ms', round(b['kernels']['fused_step']['avg_launch_ms'],3))"
done
echo "[4] prof (default build)"
BGX_FUSED_PROF=1 timeout -k 10 200 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --two-ply-steps 0 --kall-steps 0 --config1-steps 0 > $OUT/prof.json 2> $OUT/prof.err || { tail $OUT/prof.err; exit 1; }
grep "fused prof" $OUT/prof.err | head -8
