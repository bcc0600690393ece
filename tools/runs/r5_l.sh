#!/bin/bash
# round 5: the board-major doubles reply launch with its last rows in per-roll
# items (BGX_REPLY_DBL_TAIL, 64ths of the rows): reply tests on the mixed form,
# then K=4 / K=all legs over the tail fraction against the per-roll launch
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5l; mkdir -p $O
echo "[1] reply tests, mixed form"
BGX_REPLY_DBL_TAIL=16 timeout -k 10 300 python -u -m pytest tests/test_gpu_reply.py -x -q --timeout 240 --timeout-method thread > $O/t1.log 2>&1 || { tail -30 $O/t1.log; exit 1; }
tail -1 $O/t1.log
BGX_REPLY_DBL=1 BGX_REPLY_DBL_TAIL=16 timeout -k 10 300 python -u -m pytest tests/test_gpu_reply.py -k agree -x -q --timeout 240 --timeout-method thread > $O/t2.log 2>&1 || { tail -30 $O/t2.log; exit 1; }
tail -1 $O/t2.log
K4="--ply 2 --steps 100 --warmup 20 --kall-steps 0 --config1-steps 0 --two-ply-steps 0 --no-cpu-baseline --timing-steps 50"
KA="--ply 2 --k-top 0 --steps 20 --warmup 5 --kall-steps 0 --config1-steps 0 --two-ply-steps 0 --no-cpu-baseline --timing-steps 10"
echo "[2] A/B"
for rep in 1 2; do
  BGX_REPLY_DBL=0 timeout -k 10 180 python bench.py $K4 > $O/k4_roll_$rep.json 2> $O/e.err || { tail -5 $O/e.err; exit 1; }
  for t in 0 16 32 48; do
    BGX_REPLY_DBL=1 BGX_REPLY_DBL_TAIL=$t timeout -k 10 180 python bench.py $K4 > $O/k4_t${t}_$rep.json 2> $O/e.err || { tail -5 $O/e.err; exit 1; }
  done
  for t in 0 8 16; do
    BGX_REPLY_DBL=1 BGX_REPLY_DBL_TAIL=$t timeout -k 10 180 python bench.py $KA > $O/ka_t${t}_$rep.json 2> $O/e.err || { tail -5 $O/e.err; exit 1; }
  done
done
python tools/ab_vals.py $O/k4_*.json $O/ka_*.json
for f in $O/k4_*.json $O/ka_*.json; do python tools/ab_line.py $(basename $f .json) $f; done
