# fused MLP items over (tile pair, m-tile pair) (mlp_item4): engine tests + A/B vs the previous build
set -o pipefail
export TMPDIR=/tmp; OUT=gpurun_out/r3b; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py -x -q -m gpu -k fused --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 600 bash tools/ab_multi.sh r3b_long tools/diag/libbgx_prev.so &&
AB_ARGS="--steps 20 --warmup 5 --kall-steps 0 --config1-steps 0 --two-ply-steps 20 --no-cpu-baseline" timeout -k 10 400 bash tools/ab_multi.sh r3b_short tools/diag/libbgx_prev.so
