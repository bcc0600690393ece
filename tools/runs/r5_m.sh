#!/bin/bash
# round 5: K=4 reply launch, board-major doubles with the per-roll tail
# fraction around r5_l's best (16/64)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5m; mkdir -p $O
K4="--ply 2 --steps 100 --warmup 20 --kall-steps 0 --config1-steps 0 --two-ply-steps 0 --no-cpu-baseline --timing-steps 50"
for rep in 1 2; do
  for t in 6 10 13 16 20 24; do
    BGX_REPLY_DBL=1 BGX_REPLY_DBL_TAIL=$t timeout -k 10 180 python bench.py $K4 > $O/k4_t${t}_$rep.json 2> $O/e.err || { tail -5 $O/e.err; exit 1; }
  done
done
python tools/ab_vals.py $O/k4_*.json
for f in $O/k4_*.json; do python tools/ab_line.py $(basename $f .json) $f; done
