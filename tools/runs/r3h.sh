# harvest waits by polling a host-mapped sequence word: GPU suite + A/B vs the previous build
set -o pipefail
export TMPDIR=/tmp; OUT=gpurun_out/r3h; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 120 python tools/short_breakdown.py > $OUT/breakdown.json 2> $OUT/breakdown.err || { tail $OUT/breakdown.err; exit 1; }
python -c "import json;r=json.load(open('$OUT/breakdown.json'));[print({k:round(v,1) for k,v in x.items()}) for x in r]"
AB_ARGS="--steps 20 --warmup 5 --kall-steps 0 --config1-steps 0 --two-ply-steps 20 --no-cpu-baseline" timeout -k 10 400 bash tools/ab_multi.sh r3h_short tools/diag/libbgx_prev.so &&
timeout -k 10 600 bash tools/ab_multi.sh r3h_long tools/diag/libbgx_prev.so
