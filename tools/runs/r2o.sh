# few-jobs movegen kernel with 4 KB slices, two blocks per CU, specialised for the root launch: suite, A/B, timelines
set -o pipefail
export TMPDIR=/tmp; OUT=gpurun_out/r2o; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
bash tools/ab_multi.sh r2o/ab tools/diag/libbgx_prev.so || exit 1
bash tools/timeline_ab.sh r2o/tl tools/diag/libbgx_prev.so
