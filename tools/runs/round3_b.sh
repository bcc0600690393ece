# Round-3 session, GPU call 2: the GPU suite (pipelined harvest, host gather,
# late tickets), the driver's bench command, launch costs with per-workgroup
# spans, and the copy-engine overlap trace.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5b; rm -rf $OUT; mkdir -p $OUT
echo "[1] gpu tests"
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
echo "[2] bench (driver command)"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench20.json 2> $OUT/bench20.err || { tail $OUT/bench20.err; exit 1; }
echo "[3] bench 300"
timeout -k 10 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --two-ply-steps 0 --kall-steps 0 --config1-steps 0 > $OUT/bench300.json 2> $OUT/bench300.err || { tail $OUT/bench300.err; exit 1; }
echo "[4] launch cost (balanced, per-workgroup spans)"
BALANCE=1 BGX_FUSED_PROF=1 timeout -k 10 200 python tools/launch_cost.py > $OUT/launch_cost_bal.txt 2>&1 || { tail $OUT/launch_cost_bal.txt; exit 1; }
echo "[5] overlap trace"
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d $OUT/overlap -o run --output-format csv -- python tools/overlap_probe.py > $OUT/overlap.log 2>&1 || { tail $OUT/overlap.log; exit 1; }
python tools/overlap_check.py $OUT/overlap > $OUT/overlap.json; grep -E "fused_launches|large_copies" $OUT/overlap.json
python - <<'PY'
import json
for f in ("bench20", "bench300"):
    j = json.load(open(f"gpurun_out/r5b/{f}.json"))
    print(f, round(j["value"] / 1e6, 2), "M", "eps/s", round(j["episodes_per_s"]), "ms/step", round(j["ms_per_step"] * 1e3, 2), "us",
          "launch", round(j["kernels"]["fused_step"]["avg_launch_ms"] * 1e3, 1), "k4", round(j.get("two_ply_k4", {}).get("value", 0) / 1e6, 3),
          "kall", round(j.get("two_ply_kall", {}).get("value", 0) / 1e6, 3))
PY
grep -E "k=|fit|last launch" $OUT/launch_cost_bal.txt
