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
echo "[icache]"
ARGS="--steps 300 --warmup 100 --timing-steps 1 --two-ply-steps 0 --kall-steps 0 --config1-steps 0 --no-cpu-baseline"
timeout -s KILL 200 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ --kernel-include-regex "fused_step" -d $OUT/icache -o run --output-format csv -- python bench.py $ARGS > $OUT/icache.log 2>&1 || { tail -5 $OUT/icache.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAVE_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE --kernel-include-regex "fused_step" -d $OUT/ifetch -o run --output-format csv -- python bench.py $ARGS > $OUT/ifetch.log 2>&1 || { tail -5 $OUT/ifetch.log; exit 1; }
python - <<'PY'
import csv, glob, collections
for d in ("icache", "ifetch"):
    f = glob.glob(f"gpurun_out/r5i/{d}/**/*counter_collection.csv", recursive=True)
    acc = collections.defaultdict(float); n = collections.defaultdict(set)
    for r in csv.DictReader(open(f[0])):
        acc[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]].add(r["Dispatch_Id"])
    print(d, {k: round(v / max(1, len(n[k]))) for k, v in acc.items()})
PY
