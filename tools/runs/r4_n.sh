#!/bin/bash
# round 4: reply row-chunk size A/B (BGX_FLAT_CHUNK 512 / 1024 / 2048): 2-ply legs, rows per step
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4n; mkdir -p $O
A="--no-cpu-baseline --config1-steps 0 --timing-steps 20 --steps 20 --warmup 5 --two-ply-steps 50 --kall-steps 10"
for rep in 1 2; do for ch in 512 1024 2048; do
  BGX_FLAT_CHUNK=$ch timeout -k 10 300 python bench.py $A > $O/b_${ch}_$rep.json 2> $O/b_${ch}_$rep.err || { tail -20 $O/b_${ch}_$rep.err; exit 1; }
  python tools/ab_line.py chunk${ch}_$rep $O/b_${ch}_$rep.json
  python - $O/b_${ch}_$rep.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("  rows/step", {leg: round(d[leg]["value_rows_per_s"] * d[leg]["ms_per_step"] / 1e9, 3) for leg in ("two_ply_k4", "two_ply_kall")}, "M")
PY
done; done
