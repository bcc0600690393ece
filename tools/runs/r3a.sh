# cooperative tier 2 for doubles path jobs in the fused kernel: GPU engine tests,
# short-run host breakdown, A/B (prev = before the exact frontier check; coopin = inline coop; in-tree = out-of-line coop)
set -o pipefail
export TMPDIR=/tmp; OUT=gpurun_out/r3a; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
timeout -k 10 120 python tools/short_breakdown.py > $OUT/breakdown.json 2> $OUT/breakdown.err || { tail $OUT/breakdown.err; exit 1; }
python -c "import json;r=json.load(open('$OUT/breakdown.json'));[print({k:round(v,1) for k,v in x.items()}) for x in r]"
timeout -k 10 600 bash tools/ab_multi.sh r3a_long tools/diag/libbgx_prev.so tools/diag/libbgx_coopin.so &&
AB_ARGS="--steps 20 --warmup 5 --kall-steps 0 --config1-steps 0 --two-ply-steps 20 --no-cpu-baseline" timeout -k 10 400 bash tools/ab_multi.sh r3a_short tools/diag/libbgx_prev.so tools/diag/libbgx_coopin.so
