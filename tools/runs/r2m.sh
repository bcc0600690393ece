# pool kernel specialised for the 2-ply reply launch (IN_TWOPLY / OUT_PACKED_FLAT): GPU suite, A/B, timelines
set -o pipefail
export TMPDIR=/tmp; OUT=gpurun_out/r2m; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
bash tools/ab_multi.sh r2m/ab tools/diag/libbgx_prev.so || exit 1
bash tools/timeline_ab.sh r2m/tl tools/diag/libbgx_prev.so
