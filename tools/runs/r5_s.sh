#!/bin/bash
# round 5: the per-roll tail fraction again, now with workgroup row chunks
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5s; mkdir -p $O
K4="--ply 2 --steps 100 --warmup 20 --kall-steps 0 --config1-steps 0 --two-ply-steps 0 --no-cpu-baseline --timing-steps 50"
KA="--ply 2 --k-top 0 --steps 20 --warmup 5 --kall-steps 0 --config1-steps 0 --two-ply-steps 0 --no-cpu-baseline --timing-steps 10"
for rep in 1 2; do
  for t in 4 8 12 16 24; do
    BGX_REPLY_DBL_TAIL=$t timeout -k 10 180 python bench.py $K4 > $O/k4_t${t}_$rep.json 2> $O/e.err || { tail -5 $O/e.err; exit 1; }
  done
  for t in 0 12 24; do
    BGX_REPLY_DBL_TAIL=$t timeout -k 10 180 python bench.py $KA > $O/ka_t${t}_$rep.json 2> $O/e.err || { tail -5 $O/e.err; exit 1; }
  done
done
python tools/ab_vals.py $O/k4_*.json $O/ka_*.json
