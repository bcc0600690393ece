# GPU check used during development: parity tests, movegen micro-benchmarks, bench.
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -2 gpurun_out/t.log
timeout -k 10 200 python tools/mg_micro.py 200000 > gpurun_out/mg.log 2>&1 && cat gpurun_out/mg.log
timeout -k 10 200 python tools/mg_latency.py 2>&1 | grep -v amdgpu.ids
for sm in default; do
  timeout -k 10 300 python bench.py --steps 300 --warmup 100 --no-cpu-baseline > gpurun_out/b$sm.log 2>&1 || exit 1
  python - $sm <<'PY'
import json,sys
d=json.loads(open(f"gpurun_out/b{sys.argv[1]}.log").read().strip().splitlines()[-1])
t=d["two_ply_k4"]
print("run="+sys.argv[1], "1ply", round(d["value"]), round(d["ms_per_step"],4), "mg", round(d["kernels"]["movegen"]["avg_launch_ms"],4), "mlp", round(d["kernels"]["mlp"]["avg_launch_ms"],4), "fb", d["fallback_jobs"], "| 2ply", round(t["value"]), round(t["ms_per_step"],3), "mg", round(t["kernels"]["movegen"]["avg_launch_ms"],4), "mlp", round(t["kernels"]["mlp"]["avg_launch_ms"],4))
PY
done
