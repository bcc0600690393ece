# parameter sweep helper (development): 1-ply bench under different env settings
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
for kv in "$@"; do
  env $kv timeout -k 10 300 python bench.py --steps 300 --warmup 100 --two-ply-steps 0 --no-cpu-baseline > gpurun_out/sw.log 2>&1 || exit 1
  python - "$kv" <<'PY'
import json,sys
d=json.loads(open("gpurun_out/sw.log").read().strip().splitlines()[-1])
print(sys.argv[1], "1ply", round(d["value"]), round(d["ms_per_step"],4), "mg", round(d["kernels"]["movegen"]["avg_launch_ms"],4), "mlp", round(d["kernels"]["mlp"]["avg_launch_ms"],4), "fb", d["fallback_jobs"])
PY
done
