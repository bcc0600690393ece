# Round-3 session 2, GPU call 5: how an idle gap before the 20-step window
# changes it (host-timed windows after 0, 0.3, 1, 3, 20 ms of idle GPU), and
# what bench.py's own gap before t0 is (stats() + barrier, timed).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r6ab; rm -rf $OUT; mkdir -p $OUT
for sl in 0 0.3 1 3 20; do
  SLEEP_MS=$sl timeout -k 10 120 python tools/window_probe.py > $OUT/window_sleep$sl.json 2> $OUT/window_sleep$sl.err || { tail $OUT/window_sleep$sl.err; exit 1; }
  python -c "import json; j=json.load(open('$OUT/window_sleep$sl.json')); print('idle ms', $sl, 'median us', round(j['median_us'],1), sorted(round(o['us']) for o in j['windows']))"
done
timeout -k 10 120 python tools/gap_probe.py > $OUT/gap.json 2> $OUT/gap.err || { tail $OUT/gap.err; exit 1; }
cat $OUT/gap.json
