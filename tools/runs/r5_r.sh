#!/bin/bash
# round 5: top5_kernel lanes per job (BGX_T5_GL 4 in-tree, 2, 8): the 2-ply
# engine tests on each build, then K=4 / K=all legs A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5r; mkdir -p $O
B=$PWD/mlp-ppo-2ply-multi_amd/bgx
echo "[1] 2-ply tests per build"
for lib in libbgx_gl2 libbgx_gl8; do
  BGX_LIB=$B/$lib.so timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_scale.py -k "2ply or two_ply or k4 or kall" -x -q --timeout 240 --timeout-method thread > $O/t_$lib.log 2>&1 || { tail -30 $O/t_$lib.log; exit 1; }
  tail -1 $O/t_$lib.log
done
echo "[2] legs"
K4="--ply 2 --steps 100 --warmup 20 --kall-steps 0 --config1-steps 0 --two-ply-steps 0 --no-cpu-baseline --timing-steps 50"
KA="--ply 2 --k-top 0 --steps 20 --warmup 5 --kall-steps 0 --config1-steps 0 --two-ply-steps 0 --no-cpu-baseline --timing-steps 10"
for rep in 1 2; do for lib in libbgx libbgx_gl2 libbgx_gl8; do
  BGX_LIB=$B/$lib.so timeout -k 10 180 python bench.py $K4 > $O/k4_${lib}_$rep.json 2> $O/e.err || { tail -5 $O/e.err; exit 1; }
  BGX_LIB=$B/$lib.so timeout -k 10 180 python bench.py $KA > $O/ka_${lib}_$rep.json 2> $O/e.err || { tail -5 $O/e.err; exit 1; }
done; done
python tools/ab_vals.py $O/k4_*.json $O/ka_*.json
