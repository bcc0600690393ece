#!/bin/bash
# round 4: fused 1-ply A/B -- in-tree vs mlp_tile4 without zero-k-step branches
# (libbgx_noskip.so) vs tier-1 leaf streaming (libbgx_fleaf.so): fused == phased
# on each build, driver windows (3 reps, interleaved) and 600-step runs
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4l; mkdir -p $O
for lib in tools/diag/libbgx_noskip.so tools/diag/libbgx_fleaf.so; do
  BGX_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -x -q --timeout 240 --timeout-method thread -k "fused_step_matches or fused_greedy or balanced" > $O/t_$(basename $lib .so).log 2>&1 || { tail -30 $O/t_$(basename $lib .so).log; exit 1; }
  tail -1 $O/t_$(basename $lib .so).log
done
B="--no-cpu-baseline --two-ply-steps 0 --kall-steps 0 --config1-steps 0 --timing-steps 20"
for rep in 1 2 3; do for lib in mlp-ppo-2ply-multi_amd/bgx/libbgx.so tools/diag/libbgx_noskip.so tools/diag/libbgx_fleaf.so; do
  tag=$(basename $lib .so)_$rep
  BGX_LIB=$lib timeout -k 10 200 python bench.py --steps 20 --warmup 5 $B > $O/b20_$tag.json 2>> $O/b.err || { tail -20 $O/b.err; exit 1; }
  python tools/ab_line.py b20_$tag $O/b20_$tag.json
done; done
for lib in mlp-ppo-2ply-multi_amd/bgx/libbgx.so tools/diag/libbgx_noskip.so tools/diag/libbgx_fleaf.so; do
  tag=$(basename $lib .so)
  BGX_LIB=$lib timeout -k 10 200 python bench.py --steps 600 --warmup 300 $B > $O/b600_$tag.json 2>> $O/b.err || { tail -20 $O/b.err; exit 1; }
  python tools/ab_line.py b600_$tag $O/b600_$tag.json
done
