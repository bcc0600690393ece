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
