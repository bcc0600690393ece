# Round-3 session, GPU call 19: W fragments by LDS-DMA during the first tier 1
# (libbgx.so) vs the register copy in the prologue (libbgx_wcopy.so); the
# host-side composition of the driver's 20-step window.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5r; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_replay.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for lib in libbgx libbgx_wcopy libbgx libbgx_wcopy libbgx libbgx_wcopy; do
  BGX_LIB=$PWD/mlp-ppo-2ply-multi_amd/bgx/$lib.so timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --two-ply-steps 0 --kall-steps 0 --config1-steps 0 > $OUT/${lib}_20.json 2> $OUT/${lib}_20.err || { tail $OUT/${lib}_20.err; exit 1; }
  python -c "
import json
a=json.load(open('$OUT/${lib}_20.json'))
print('$lib', '20:', round(a['value']/1e6,2))"
done
timeout -k 10 200 python bench.py --steps 600 --warmup 5 --no-cpu-baseline --two-ply-steps 0 --kall-steps 0 --config1-steps 0 > $OUT/libbgx_600.json 2> $OUT/libbgx_600.err || { tail $OUT/libbgx_600.err; exit 1; }
python -c "import json; b=json.load(open('$OUT/libbgx_600.json')); print('600:', round(b['value']/1e6,2))"
timeout -k 10 120 python tools/probe/host_overhead.py > $OUT/host.json 2> $OUT/host.err || { tail $OUT/host.err; exit 1; }
cat $OUT/host.json
