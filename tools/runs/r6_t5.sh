#!/bin/bash
# round 6: top5_kernel with 16-byte block loads (BGX_T5_VB=2 / 4 builds,
# bgx/libbgx_t5v2.so, libbgx_t5v4.so) against the scalar-load default:
# 2-ply oracle tests on each block build, kernel traces of one K=4 + K=all
# bench run per build, then the interleaved bench legs.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6t5; mkdir -p $O
B=$PWD/mlp-ppo-2ply-multi_amd/bgx
timeout -k 10 120 python tools/probe/t5_debug.py $O/base.npz > $O/dbg.log 2>&1 || { tail $O/dbg.log; exit 1; }
for v in t5v2 t5v4; do
  BGX_LIB=$B/libbgx_$v.so timeout -k 10 120 python tools/probe/t5_debug.py $O/$v.npz >> $O/dbg.log 2>&1 || { tail $O/dbg.log; exit 1; }
  python -c "import numpy as np; a=np.load('$O/base.npz'); b=np.load('$O/$v.npz'); print('$v', {k: bool((a[k][0] == b[k]).all()) for k in ('exact', 'samp')})"
done
for v in t5v2 t5v4; do
  BGX_LIB=$B/libbgx_$v.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_scale.py tests/test_gpu_engine.py tests/test_gpu_replay.py -k "configs2 or same_seed or k4_8192_lanes_w or kall_8192 or two_ply or 2ply" > $O/t_$v.log 2>&1 || { tail -30 $O/t_$v.log; exit 1; }
  echo "$v tests: $(tail -1 $O/t_$v.log)"
done
A="--ply 2 --steps 40 --warmup 10 --timing-steps 1 --two-ply-steps 0 --kall-steps 20 --config1-steps 0 --config2-steps 0 --no-cpu-baseline"
for v in libbgx libbgx_t5v2 libbgx_t5v4; do
  BGX_LIB=$B/$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_$v -o run --output-format csv -- python bench.py $A > $O/kt_$v.json 2> $O/kt_$v.err || { tail $O/kt_$v.err; exit 1; }
  f=$(find $O/kt_$v -name "*kernel_stats.csv" | head -1); echo "$v: $(grep top5 $f | cut -d, -f1-4)"
done
bash tools/runs/ab_legs.sh r6t5/ab 3 "k4 kall" base t5v2::libbgx_t5v2 t5v4::libbgx_t5v4
