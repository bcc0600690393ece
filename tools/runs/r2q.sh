# fused: 16 lanes / 8 waves below 32 x CUs lanes, 32 lanes / 12 waves above; slice split variant (128-slot table)
set -o pipefail
export TMPDIR=/tmp; OUT=gpurun_out/r2q; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_replay.py -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
BGX_LIB=tools/diag/libbgx_s128.so timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py -x -q --timeout 200 --timeout-method thread -k fused > $OUT/tests_s128.log 2>&1 || { tail -40 $OUT/tests_s128.log; exit 1; }
tail -1 $OUT/tests_s128.log
for lib in mlp-ppo-2ply-multi_amd/bgx/libbgx.so tools/diag/libbgx_s128.so; do
tag=$(basename $lib .so)
BGX_LIB=$lib BGX_FUSED_PROF=1 timeout -k 10 200 python bench.py --steps 300 --warmup 100 --two-ply-steps 0 --kall-steps 0 --config1-steps 0 --no-cpu-baseline --timing-steps 100 > $OUT/prof_$tag.json 2> $OUT/prof_$tag.err || exit 1
grep "fused prof" $OUT/prof_$tag.err
done
AB_ARGS="--steps 600 --warmup 300 --kall-steps 0 --two-ply-steps 0 --no-cpu-baseline --timing-steps 300 --config1-steps 300" bash tools/ab_multi.sh r2q/ab tools/diag/libbgx_s128.so tools/diag/libbgx_prev.so
for f in $OUT/ab/*.json; do python -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$f', round(d['value']/1e6,2), round(d['configs1_4096_lanes']['value']/1e6,2))"; done
