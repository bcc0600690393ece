#!/bin/bash
# round 5: reply launch items in doubles-first order (libbgx_hf) vs row-major
# (in-tree), K=4 with per-roll and board-major doubles, K=all
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5h; mkdir -p $O
B=$PWD/mlp-ppo-2ply-multi_amd/bgx
echo "[1] reply tests on libbgx_hf"
BGX_LIB=$B/libbgx_hf.so timeout -k 10 300 python -u -m pytest tests/test_gpu_reply.py -x -q --timeout 240 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
K4="--ply 2 --steps 100 --warmup 20 --kall-steps 0 --config1-steps 0 --two-ply-steps 0 --no-cpu-baseline --timing-steps 50"
KA="--ply 2 --k-top 0 --steps 20 --warmup 5 --kall-steps 0 --config1-steps 0 --two-ply-steps 0 --no-cpu-baseline --timing-steps 10"
echo "[2] A/B"
for rep in 1 2; do for lib in libbgx libbgx_hf; do
  BGX_LIB=$B/$lib.so timeout -k 10 180 python bench.py $K4 > $O/k4_${lib}_$rep.json 2> $O/e.err || { tail -5 $O/e.err; exit 1; }
  BGX_REPLY_DBL=1 BGX_LIB=$B/$lib.so timeout -k 10 180 python bench.py $K4 > $O/k4dbl_${lib}_$rep.json 2> $O/e.err || { tail -5 $O/e.err; exit 1; }
  BGX_LIB=$B/$lib.so timeout -k 10 180 python bench.py $KA > $O/ka_${lib}_$rep.json 2> $O/e.err || { tail -5 $O/e.err; exit 1; }
done; done
for f in $O/k4_*.json $O/k4dbl_*.json $O/ka_*.json; do python tools/ab_line.py $(basename $f .json) $f; done
