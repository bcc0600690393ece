# Round-3 session, GPU call 24: the driver's 20-step window, host-timed, median
# of 10 windows after 300 desync steps (tools/window_probe.py), carried next-
# position expansion (libbgx.so) vs not (libbgx_prev.so), twice each.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5w; rm -rf $OUT; mkdir -p $OUT
for lib in libbgx libbgx_prev libbgx libbgx_prev; do
  BGX_LIB=$PWD/mlp-ppo-2ply-multi_amd/bgx/$lib.so timeout -k 10 120 python tools/window_probe.py > $OUT/${lib}.json 2> $OUT/${lib}.err || { tail $OUT/${lib}.err; exit 1; }
  python -c "import json; j=json.load(open('$OUT/${lib}.json')); print('$lib', 'median us', round(j['median_us'],1), sorted(round(o['us']) for o in j['windows']))"
done
