# Round-3 session, GPU call 1: counters available, the GPU suite, the driver's
# bench command (balanced vs lockstep) and the launch-cost fit.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5a; rm -rf $OUT; mkdir -p $OUT
echo "[1] counters"
timeout -k 10 60 rocprofv3 -L > $OUT/counters_all.txt 2>&1 || echo "list failed"
grep -iE "SQ_ACTIVE_INST|SQ_INST_CYCLES|SALU|SCA" $OUT/counters_all.txt | head -40 > $OUT/counters_sq.txt || true
echo "[2] gpu tests"
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -3 $OUT/gpu_tests.log
echo "[3] bench (driver command), balanced"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench20.json 2> $OUT/bench20.err || { tail $OUT/bench20.err; exit 1; }
echo "[4] bench 20 lockstep"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-balance --two-ply-steps 0 --kall-steps 0 > $OUT/bench20_lockstep.json 2> $OUT/bench20l.err || { tail $OUT/bench20l.err; exit 1; }
echo "[5] bench 300 balanced"
timeout -k 10 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --two-ply-steps 0 --kall-steps 0 --config1-steps 0 > $OUT/bench300.json 2> $OUT/bench300.err || { tail $OUT/bench300.err; exit 1; }
echo "[6] launch cost"
BALANCE=1 timeout -k 10 200 python tools/launch_cost.py > $OUT/launch_cost_bal.txt 2>&1 || { tail $OUT/launch_cost_bal.txt; exit 1; }
BALANCE=0 timeout -k 10 200 python tools/launch_cost.py > $OUT/launch_cost_lock.txt 2>&1 || { tail $OUT/launch_cost_lock.txt; exit 1; }
python - <<'PY'
import json
for f in ("bench20", "bench20_lockstep", "bench300"):
    j = json.load(open(f"gpurun_out/r5a/{f}.json"))
    print(f, round(j["value"] / 1e6, 2), "M", "eps/s", round(j["episodes_per_s"]), j["roofline"]["bound"],
          "k4", round(j.get("two_ply_k4", {}).get("value", 0) / 1e6, 3), "kall", round(j.get("two_ply_kall", {}).get("value", 0) / 1e6, 3))
PY
tail -2 gpurun_out/r5a/launch_cost_bal.txt gpurun_out/r5a/launch_cost_lock.txt
