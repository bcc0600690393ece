#!/bin/bash
# round 5: 16-lane workgroups (configs[1]: 4,096 lanes) on 12 waves instead of 8
# (libbgx_nw16) vs in-tree: fused == phased on it, then 4,096-lane A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5k; mkdir -p $O
B=$PWD/mlp-ppo-2ply-multi_amd/bgx
echo "[1] parity on libbgx_nw16"
BGX_LIB=$B/libbgx_nw16.so timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py -k "fused" -x -q --timeout 240 --timeout-method thread > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
LIBS="libbgx libbgx_nw16"
A600="--lanes 4096 --steps 600 --warmup 300 --kall-steps 0 --config1-steps 0 --two-ply-steps 0 --no-cpu-baseline --timing-steps 0"
A300="--lanes 4096 --steps 300 --warmup 100 --kall-steps 0 --config1-steps 0 --two-ply-steps 0 --no-cpu-baseline --timing-steps 0"
echo "[2] 4,096 lanes, 600 steps"
for rep in 1 2; do for lib in $LIBS; do
  BGX_LIB=$B/$lib.so timeout -k 10 180 python bench.py $A600 > $O/b600_${lib}_$rep.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
done; done
python tools/ab_vals.py $O/b600_*.json
echo "[3] 4,096 lanes, 300 steps (bench.py's configs[1] leg shape)"
for rep in 1 2; do for lib in $LIBS; do
  BGX_LIB=$B/$lib.so timeout -k 10 180 python bench.py $A300 > $O/b300_${lib}_$rep.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
done; done
python tools/ab_vals.py $O/b300_*.json
