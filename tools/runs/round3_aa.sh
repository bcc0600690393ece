# Round-3 session 2, GPU call 4: the next step's MLP tiles run at the end of a
# step's queue (rows allocated per lane as its tier-1 job finishes; libbgx.so)
# vs the committed tree 8b530a0 (libbgx_prev.so). Engine / replay tests first.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r6aa; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_replay.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for lib in libbgx libbgx_prev libbgx libbgx_prev; do
  BGX_LIB=$PWD/mlp-ppo-2ply-multi_amd/bgx/$lib.so timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --two-ply-steps 0 --kall-steps 0 --config1-steps 0 > $OUT/${lib}_20.json 2> $OUT/${lib}_20.err || { tail $OUT/${lib}_20.err; exit 1; }
  BGX_LIB=$PWD/mlp-ppo-2ply-multi_amd/bgx/$lib.so timeout -k 10 200 python bench.py --steps 600 --warmup 5 --no-cpu-baseline --two-ply-steps 0 --kall-steps 0 --config1-steps 0 > $OUT/${lib}_600.json 2> $OUT/${lib}_600.err || { tail $OUT/${lib}_600.err; exit 1; }
  python -c "
import json
a=json.load(open('$OUT/${lib}_20.json')); b=json.load(open('$OUT/${lib}_600.json'))
print('$lib', '20:', round(a['value']/1e6,2), 'M  600:', round(b['value']/1e6,2), 'launch600 ms', round(b['kernels']['fused_step']['avg_launch_ms'],3))"
done
BGX_FUSED_PROF=1 timeout -k 10 200 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --two-ply-steps 0 --kall-steps 0 --config1-steps 0 > $OUT/prof.json 2> $OUT/prof.err || { tail $OUT/prof.err; exit 1; }
grep "fused prof" $OUT/prof.err
