# Round-3 session 2: in the budget's last round a workgroup whose next step
# needs a tier-2 redo yields the remaining tickets (libbgx_y.so, -DBGX_YIELD_TAIL)
# vs the committed kernel (libbgx.so); engine / replay tests with the variant first.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r7aj; rm -rf $OUT; mkdir -p $OUT
BGX_LIB=$PWD/mlp-ppo-2ply-multi_amd/bgx/libbgx_y.so timeout -k 10 500 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_replay.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for k in 1 2 3; do for lib in libbgx_y libbgx; do
  BGX_LIB=$PWD/mlp-ppo-2ply-multi_amd/bgx/$lib.so timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --two-ply-steps 0 --kall-steps 0 --config1-steps 0 > $OUT/${lib}_20_$k.json 2> $OUT/${lib}_20_$k.err || { tail $OUT/${lib}_20_$k.err; exit 1; }
  python -c "
import json
a=json.load(open('$OUT/${lib}_20_$k.json'))
print('$lib', '20:', round(a['value']/1e6,2), 'M, env steps', a['env_steps_per_rank'])"
done; done
for lib in libbgx_y libbgx; do
  BGX_LIB=$PWD/mlp-ppo-2ply-multi_amd/bgx/$lib.so timeout -k 10 200 python bench.py --steps 600 --warmup 5 --no-cpu-baseline --two-ply-steps 0 --kall-steps 0 --config1-steps 0 > $OUT/${lib}_600.json 2> $OUT/${lib}_600.err || { tail $OUT/${lib}_600.err; exit 1; }
  python -c "import json; b=json.load(open('$OUT/${lib}_600.json')); print('$lib 600:', round(b['value']/1e6,2))"
done
BGX_LIB=$PWD/mlp-ppo-2ply-multi_amd/bgx/libbgx_y.so BGX_FUSED_PROF=1 BGX_FUSED_PROF_DUMP=$OUT/wg_y.csv timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --two-ply-steps 0 --kall-steps 0 --config1-steps 0 --timing-steps 20 > $OUT/prof_y.json 2> $OUT/prof_y.err || { tail $OUT/prof_y.err; exit 1; }
grep "last launch" $OUT/prof_y.err
