# Round-3 session, GPU call 9: whole-tile MLP items (mlp_tile4) in the fused
# kernel vs the (tile pair, m-tile) items (libbgx_prev.so = commit b177f90):
# fused == phased tests, then A/B at 20 and 600 steps, then the prof split.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5h; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread -k "fused or balanced or greedy or pipelined" > $OUT/engine_tests.log 2>&1 || { tail -40 $OUT/engine_tests.log; exit 1; }
tail -1 $OUT/engine_tests.log
for lib in libbgx libbgx_prev libbgx libbgx_prev; do
  BGX_LIB=$PWD/mlp-ppo-2ply-multi_amd/bgx/$lib.so timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --two-ply-steps 0 --kall-steps 0 --config1-steps 0 > $OUT/${lib}_20.json 2> $OUT/${lib}_20.err || { tail $OUT/${lib}_20.err; exit 1; }
  BGX_LIB=$PWD/mlp-ppo-2ply-multi_amd/bgx/$lib.so timeout -k 10 200 python bench.py --steps 600 --warmup 5 --no-cpu-baseline --two-ply-steps 0 --kall-steps 0 --config1-steps 0 > $OUT/${lib}_600.json 2> $OUT/${lib}_600.err || { tail $OUT/${lib}_600.err; exit 1; }
  python -c "
import json
a=json.load(open('$OUT/${lib}_20.json')); b=json.load(open('$OUT/${lib}_600.json'))
print('$lib', '20:', round(a['value']/1e6,2), '600:', round(b['value']/1e6,2), 'launch600 ms', round(b['kernels']['fused_step']['avg_launch_ms'],3))"
done
BGX_FUSED_PROF=1 timeout -k 10 200 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --two-ply-steps 0 --kall-steps 0 --config1-steps 0 > $OUT/prof.json 2> $OUT/prof.err || { tail $OUT/prof.err; exit 1; }
grep "fused prof" $OUT/prof.err | head -5
