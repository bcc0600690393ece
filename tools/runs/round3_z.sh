# Round-3 session 2, GPU call 3: in-kernel harvest (each fused workgroup harvests
# its own lanes at the end of a launch; libbgx.so) + LDS-DMA W prologue, vs the
# DMA prologue alone (libbgx_dma.so) and the committed tree (libbgx_prev.so).
# Whole GPU suite first.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r6z; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for lib in libbgx libbgx_dma libbgx_prev libbgx libbgx_dma libbgx_prev; do
  BGX_LIB=$PWD/mlp-ppo-2ply-multi_amd/bgx/$lib.so timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --two-ply-steps 0 --kall-steps 0 --config1-steps 0 > $OUT/${lib}_20.json 2> $OUT/${lib}_20.err || { tail $OUT/${lib}_20.err; exit 1; }
  BGX_LIB=$PWD/mlp-ppo-2ply-multi_amd/bgx/$lib.so timeout -k 10 200 python bench.py --steps 600 --warmup 5 --no-cpu-baseline --two-ply-steps 0 --kall-steps 0 --config1-steps 0 > $OUT/${lib}_600.json 2> $OUT/${lib}_600.err || { tail $OUT/${lib}_600.err; exit 1; }
  python -c "
import json
a=json.load(open('$OUT/${lib}_20.json')); b=json.load(open('$OUT/${lib}_600.json'))
print('$lib', '20:', round(a['value']/1e6,2), 'eps/s', round(a['episodes_per_s']/1e6,2), 'M  600:', round(b['value']/1e6,2), 'launch600 ms', round(b['kernels']['fused_step']['avg_launch_ms'],3))"
done
timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/trace -o run --output-format csv -- python tools/window_probe.py > $OUT/window_traced.json 2> $OUT/trace.err || { tail $OUT/trace.err; exit 1; }
python tools/window_check.py $OUT/trace > $OUT/window_split.json
python -c "
import json; j=json.load(open('$OUT/window_split.json'))
for w in j[-3:]: print(w['span_us'], w['seq'])"
BGX_FUSED_PROF=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --two-ply-steps 0 --kall-steps 0 --config1-steps 0 --timing-steps 20 > $OUT/prof_20.json 2> $OUT/prof_20.err || { tail $OUT/prof_20.err; exit 1; }
grep "last launch" $OUT/prof_20.err
