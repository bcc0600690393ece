#!/bin/bash
# round 5: top5_kernel with the next iteration's values loaded ahead (in-tree,
# BGX_T5_PF=1) vs without (libbgx_t5n): 2-ply GPU tests, then K=4 / K=all A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5w; mkdir -p $O
B=$PWD/mlp-ppo-2ply-multi_amd/bgx
timeout -k 10 900 python -u -m pytest tests/test_gpu_reply.py tests/test_gpu_engine.py tests/test_gpu_replay.py tests/test_gpu_scale.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
K4="--ply 2 --steps 100 --warmup 20 --kall-steps 0 --config1-steps 0 --two-ply-steps 0 --no-cpu-baseline --timing-steps 50"
KA="--ply 2 --k-top 0 --steps 20 --warmup 5 --kall-steps 0 --config1-steps 0 --two-ply-steps 0 --no-cpu-baseline --timing-steps 10"
for rep in 1 2 3; do for lib in libbgx libbgx_t5n; do
  BGX_LIB=$B/$lib.so timeout -k 10 180 python bench.py $K4 > $O/k4_${lib}_$rep.json 2> $O/e.err || { tail -5 $O/e.err; exit 1; }
  BGX_LIB=$B/$lib.so timeout -k 10 180 python bench.py $KA > $O/ka_${lib}_$rep.json 2> $O/e.err || { tail -5 $O/e.err; exit 1; }
done; done
python tools/ab_vals.py $O/k4_*.json $O/ka_*.json
