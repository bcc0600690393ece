#!/bin/bash
# round 5: mlp_tile4 with software-pipelined fragment reads (BGX_TILE_PF, in-tree = 2)
# vs the compiler's schedule (pf0) and a 1-deep ring (pf1): fused == phased
# and the bench-shape replay on the new default, then 600- and 20-step A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5b; mkdir -p $O
echo "[1] parity of the in-tree build"
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py -k "fused" tests/test_gpu_scale.py::test_bench_shape_1ply_matches_oracle -x -q --timeout 240 --timeout-method thread > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
B=mlp-ppo-2ply-multi_amd/bgx
echo "[2] 600 steps"
A600="--steps 600 --warmup 300 --kall-steps 0 --config1-steps 0 --two-ply-steps 0 --no-cpu-baseline --timing-steps 0"
for rep in 1 2; do for lib in libbgx libbgx_pf0 libbgx_pf1; do
  BGX_LIB=$B/$lib.so timeout -k 10 180 python bench.py $A600 > $O/b600_${lib}_$rep.json 2> $O/b600.err || { tail -5 $O/b600.err; exit 1; }
  python tools/ab_line.py b600_${lib}_$rep $O/b600_${lib}_$rep.json
done; done
echo "[3] 20 steps (driver flags, 1-ply leg only)"
A20="--steps 20 --warmup 5 --kall-steps 0 --config1-steps 0 --two-ply-steps 0 --no-cpu-baseline --timing-steps 0"
for rep in 1 2 3; do for lib in libbgx libbgx_pf0 libbgx_pf1; do
  BGX_LIB=$B/$lib.so timeout -k 10 180 python bench.py $A20 > $O/b20_${lib}_$rep.json 2> $O/b20.err || { tail -5 $O/b20.err; exit 1; }
  python tools/ab_line.py b20_${lib}_$rep $O/b20_${lib}_$rep.json
done; done
echo "[4] phase clocks of the in-tree build, 600 steps"
BGX_FUSED_PROF=1 timeout -k 10 300 python bench.py $A600 > $O/prof600.json 2> $O/prof600.err || { tail -20 $O/prof600.err; exit 1; }
grep "fused prof" $O/prof600.err
