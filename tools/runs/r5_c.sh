#!/bin/bash
# round 5: half-lane tickets in the balanced launch's last round + mlp_tile4
# prefetch (in-tree) vs whole-group tickets (nohalf) and the MFMA chain at
# priority 1 / 3 (p1, p3): parity of the in-tree build, then 600 / 20-step A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5c; mkdir -p $O
echo "[1] parity of the in-tree build"
timeout -k 10 500 python -u -m pytest tests/test_gpu_engine.py -k "fused or balanced" tests/test_gpu_scale.py::test_bench_shape_1ply_matches_oracle -x -q --timeout 240 --timeout-method thread > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
B=mlp-ppo-2ply-multi_amd/bgx
LIBS="libbgx libbgx_nohalf libbgx_p1 libbgx_p3"
A600="--steps 600 --warmup 300 --kall-steps 0 --config1-steps 0 --two-ply-steps 0 --no-cpu-baseline --timing-steps 0"
A20="--steps 20 --warmup 5 --kall-steps 0 --config1-steps 0 --two-ply-steps 0 --no-cpu-baseline --timing-steps 0"
echo "[2] 600 steps"
for rep in 1 2; do for lib in $LIBS; do
  BGX_LIB=$B/$lib.so timeout -k 10 180 python bench.py $A600 > $O/b600_${lib}_$rep.json 2> $O/b600.err || { tail -5 $O/b600.err; exit 1; }
done; done
python tools/ab_vals.py $O/b600_*.json
echo "[3] 20 steps"
for rep in 1 2 3 4; do for lib in $LIBS; do
  BGX_LIB=$B/$lib.so timeout -k 10 180 python bench.py $A20 > $O/b20_${lib}_$rep.json 2> $O/b20.err || { tail -5 $O/b20.err; exit 1; }
done; done
python tools/ab_vals.py $O/b20_*.json
