# half_last by v_readlane + one scan less in the softmax (m <= 32): GPU suite + A/B vs the previous build
set -o pipefail
export TMPDIR=/tmp; OUT=gpurun_out/r3g; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
AB_ARGS="--steps 20 --warmup 5 --kall-steps 0 --config1-steps 0 --two-ply-steps 20 --no-cpu-baseline" timeout -k 10 400 bash tools/ab_multi.sh r3g_short tools/diag/libbgx_prev.so &&
timeout -k 10 600 bash tools/ab_multi.sh r3g_long tools/diag/libbgx_prev.so
