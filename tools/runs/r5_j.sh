#!/bin/bash
# round 5: mlp_tile4 in 8 waves per 32-lane workgroup (256 registers, no spills), with the two-half tile
# half's MFMAs, libbgx_hv) vs in-tree: fused == phased on it, then 600 / 20-step A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5j; mkdir -p $O
B=$PWD/mlp-ppo-2ply-multi_amd/bgx
echo "[1] parity on libbgx_nw8hv"
BGX_LIB=$B/libbgx_nw8hv.so timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py -k "fused" -x -q --timeout 240 --timeout-method thread > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
LIBS="libbgx libbgx_nw8 libbgx_nw8hv libbgx_nw8hv2"
A600="--steps 600 --warmup 300 --kall-steps 0 --config1-steps 0 --two-ply-steps 0 --no-cpu-baseline --timing-steps 0"
A20="--steps 20 --warmup 5 --kall-steps 0 --config1-steps 0 --two-ply-steps 0 --no-cpu-baseline --timing-steps 20"
echo "[2] 600 steps"
for rep in 1 2; do for lib in $LIBS; do
  BGX_LIB=$B/$lib.so timeout -k 10 180 python bench.py $A600 > $O/b600_${lib}_$rep.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
done; done
python tools/ab_vals.py $O/b600_*.json
echo "[3] 20 steps"
for rep in 1 2 3; do for lib in $LIBS; do
  BGX_LIB=$B/$lib.so timeout -k 10 180 python bench.py $A20 > $O/b20_${lib}_$rep.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
done; done
python tools/ab_vals.py $O/b20_*.json
