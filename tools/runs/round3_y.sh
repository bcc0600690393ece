# Round-3 session 2, GPU call 2: the shape of a short fused launch (prof build:
# prologue / step loop / epilogue per workgroup, shader clock) at 20 and 300
# steps, and the host-timed 20-step window with and without an idle gap before it.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r6y; rm -rf $OUT; mkdir -p $OUT
for n in 20 300; do
  BGX_FUSED_PROF=1 timeout -k 10 200 python bench.py --steps $n --warmup 5 --no-cpu-baseline --two-ply-steps 0 --kall-steps 0 --config1-steps 0 --timing-steps $n > $OUT/prof_$n.json 2> $OUT/prof_$n.err || { tail $OUT/prof_$n.err; exit 1; }
  echo "== prof $n steps"; grep "fused prof" $OUT/prof_$n.err
done
for sl in 20 0; do
  SLEEP_MS=$sl timeout -k 10 120 python tools/window_probe.py > $OUT/window_sleep$sl.json 2> $OUT/window_sleep$sl.err || { tail $OUT/window_sleep$sl.err; exit 1; }
  python -c "import json; j=json.load(open('$OUT/window_sleep$sl.json')); print('sleep', $sl, 'median us', round(j['median_us'],1), sorted(round(o['us']) for o in j['windows']))"
done
timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/trace -o run --output-format csv -- python tools/window_probe.py > $OUT/window_traced.json 2> $OUT/trace.err || { tail $OUT/trace.err; exit 1; }
python tools/window_check.py $OUT/trace > $OUT/window_split.json
python -c "
import json; j=json.load(open('$OUT/window_split.json'))
for w in j[-4:]: print(w['span_us'], w['seq'])"
for k in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/driver_$k.json 2> $OUT/driver_$k.err || { tail $OUT/driver_$k.err; exit 1; }
  python -c "import json; j=json.load(open('$OUT/driver_$k.json')); print('driver cmd', round(j['value']/1e6,1), 'M', round(j['ms_per_step']*1e3,1), 'us/step; K=4', round(j['two_ply_k4']['value']/1e6,2), 'K=all', round(j['two_ply_kall']['value']/1e6,3))"
done
