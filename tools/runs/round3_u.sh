# Round-3 session, GPU call 22: the cleaned pipelined kernel: the whole GPU
# suite, smoke, the driver's bench command and a 600-step run.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5u; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $OUT/bench20.json 2> $OUT/bench20.err || { tail $OUT/bench20.err; exit 1; }
timeout -k 10 200 python bench.py --steps 600 --warmup 5 --no-cpu-baseline --two-ply-steps 0 --kall-steps 0 --config1-steps 0 > $OUT/bench600.json 2> $OUT/bench600.err || { tail $OUT/bench600.err; exit 1; }
python - <<'PY'
import json
a = json.load(open("gpurun_out/r5u/bench20.json")); b = json.load(open("gpurun_out/r5u/bench600.json"))
print("bench20", round(a["value"] / 1e6, 2), "M; episodes/s", round(a.get("episodes_per_s", 0)), "k4", round(a.get("two_ply_k4", {}).get("value", 0) / 1e6, 3),
      "kall", round(a.get("two_ply_kall", {}).get("value", 0) / 1e6, 3), "cpu", a.get("cpu_baseline", {}).get("value"), "roofline", json.dumps(a.get("roofline"))[:300])
print("bench600", round(b["value"] / 1e6, 2))
PY
