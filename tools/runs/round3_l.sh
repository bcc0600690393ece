# Round-3 session, GPU call 13: mlp_tile4 with two laundered LDS bases (no per-read
# address adds) in the fused kernel vs the previous
# mlp_tile4 (libbgx_v1.so, -DBGX_TILE4_V1); LDS-staged reply MLP + 16-deep
# top-5 loads with a max/min insert network for 2-ply. Parity first (fused == phased, replays, 2-ply).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5l; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_replay.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for lib in libbgx libbgx_v1 libbgx libbgx_v1; do
  BGX_LIB=$PWD/mlp-ppo-2ply-multi_amd/bgx/$lib.so timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --two-ply-steps 0 --kall-steps 0 --config1-steps 0 > $OUT/${lib}_20.json 2> $OUT/${lib}_20.err || { tail $OUT/${lib}_20.err; exit 1; }
  BGX_LIB=$PWD/mlp-ppo-2ply-multi_amd/bgx/$lib.so timeout -k 10 200 python bench.py --steps 600 --warmup 5 --no-cpu-baseline --two-ply-steps 0 --kall-steps 0 --config1-steps 0 > $OUT/${lib}_600.json 2> $OUT/${lib}_600.err || { tail $OUT/${lib}_600.err; exit 1; }
  python -c "
import json
a=json.load(open('$OUT/${lib}_20.json')); b=json.load(open('$OUT/${lib}_600.json'))
print('$lib', '20:', round(a['value']/1e6,2), '600:', round(b['value']/1e6,2), 'launch600 ms', round(b['kernels']['fused_step']['avg_launch_ms'],3))"
done
BGX_FUSED_PROF=1 timeout -k 10 200 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --two-ply-steps 0 --kall-steps 0 --config1-steps 0 > $OUT/prof.json 2> $OUT/prof.err || { tail $OUT/prof.err; exit 1; }
grep "fused prof" $OUT/prof.err | head -5
ARGS="--ply 2 --k-top 4 --steps 100 --warmup 20 --timing-steps 1 --two-ply-steps 0 --kall-steps 0 --config1-steps 0 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python bench.py $ARGS > $OUT/kt.json 2> $OUT/kt.err || { tail $OUT/kt.err; exit 1; }
python tools/kstat.py $(find $OUT/kt -name "*kernel_stats.csv" | head -1) ""
python -c "import json; j=json.load(open('$OUT/kt.json')); print('k4 traced', round(j['value']/1e6,3), 'M', round(j['ms_per_step']*1e3,1), 'us/step')"
