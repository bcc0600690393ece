# MLP kernels built with the memory-clause scheduling strategy: GPU suite, then A/B vs the previous build
set -o pipefail
export TMPDIR=/tmp; OUT=gpurun_out/r4g; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
AB_ARGS="--steps 300 --warmup 100 --kall-steps 3 --config1-steps 0 --two-ply-steps 100 --no-cpu-baseline --timing-steps 100" timeout -k 10 500 bash tools/ab_multi.sh r4g_ab tools/diag/libbgx_prev.so
