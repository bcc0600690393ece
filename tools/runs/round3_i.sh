# Round-3 session, GPU call 10: the driver's 20-step window, host-timed and traced.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5i; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_replay.py -x -q --timeout 120 --timeout-method thread -k "pipelined or bulk or transitions or replay" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 120 python tools/window_probe.py > $OUT/window.json 2> $OUT/window.err || { tail $OUT/window.err; exit 1; }
python -c "import json; j=json.load(open('$OUT/window.json')); print('host median us', round(j['median_us'],1), [round(o['us']) for o in j['windows']])"
timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/trace -o run --output-format csv -- python tools/window_probe.py > $OUT/window_traced.json 2> $OUT/trace.err || { tail $OUT/trace.err; exit 1; }
python tools/window_check.py $OUT/trace > $OUT/window_split.json
python -c "
import json; j=json.load(open('$OUT/window_split.json'))
for w in j[-3:]: print(w['span_us'], w['seq'])"
