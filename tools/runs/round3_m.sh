# Round-3 session, GPU call 14: LDS-DMA staged top-5 (16 jobs' values per wave
# in one memory latency); the 2-ply suite, then K=4 traced and K=all.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5m; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
ARGS="--ply 2 --k-top 4 --steps 100 --warmup 20 --timing-steps 1 --two-ply-steps 0 --kall-steps 0 --config1-steps 0 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python bench.py $ARGS > $OUT/kt.json 2> $OUT/kt.err || { tail $OUT/kt.err; exit 1; }
python tools/kstat.py $(find $OUT/kt -name "*kernel_stats.csv" | head -1) "" | head -9
timeout -k 10 200 python bench.py $ARGS > $OUT/k4.json 2> $OUT/k4.err || { tail $OUT/k4.err; exit 1; }
python -c "import json; j=json.load(open('$OUT/k4.json')); print('k4', round(j['value']/1e6,3), 'M', round(j['ms_per_step']*1e3,1), 'us/step')"
timeout -k 10 300 python bench.py --ply 2 --k-top 0 --steps 20 --warmup 5 --timing-steps 1 --two-ply-steps 0 --kall-steps 0 --config1-steps 0 --no-cpu-baseline > $OUT/kall.json 2> $OUT/kall.err || { tail $OUT/kall.err; exit 1; }
python -c "import json; j=json.load(open('$OUT/kall.json')); print('kall', round(j['value']/1e6,3), 'M', round(j['ms_per_step']*1e3,1), 'us/step')"
