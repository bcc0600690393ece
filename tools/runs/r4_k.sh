#!/bin/bash
# round 4: fused 1-ply with tier-1 leaf streaming for path doubles (libbgx_fleaf.so):
# fused == phased and replay tests on that build, then driver-window and 600-step A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4k; mkdir -p $O
BGX_LIB=tools/diag/libbgx_fleaf.so timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_replay.py tests/test_gpu_scale.py -x -q --timeout 240 --timeout-method thread -k "fused or replay or bench_shape or transitions" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
B="--no-cpu-baseline --two-ply-steps 0 --kall-steps 0 --config1-steps 0 --timing-steps 20"
for rep in 1 2 3; do for lib in mlp-ppo-2ply-multi_amd/bgx/libbgx.so tools/diag/libbgx_fleaf.so; do
  tag=$(basename $lib .so)_$rep
  BGX_LIB=$lib timeout -k 10 200 python bench.py --steps 20 --warmup 5 $B > $O/b20_$tag.json 2>> $O/b.err || { tail -20 $O/b.err; exit 1; }
  python tools/ab_line.py b20_$tag $O/b20_$tag.json
done; done
for lib in mlp-ppo-2ply-multi_amd/bgx/libbgx.so tools/diag/libbgx_fleaf.so; do
  tag=$(basename $lib .so)
  BGX_LIB=$lib BGX_FUSED_PROF=1 timeout -k 10 200 python bench.py --steps 600 --warmup 300 $B > $O/b600_$tag.json 2> $O/prof_$tag.err || { tail -20 $O/prof_$tag.err; exit 1; }
  python tools/ab_line.py b600prof_$tag $O/b600_$tag.json; grep "tier-2\|last launch" $O/prof_$tag.err | tail -3
done
