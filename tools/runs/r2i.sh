# branch-free move helpers + one-register job prefetch: GPU suite, then A/B (wpe8 in-tree, wpe7, previous)
set -o pipefail
export TMPDIR=/tmp; OUT=gpurun_out/r2i; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
bash tools/ab_multi.sh r2i/ab tools/diag/libbgx_wpe7.so tools/diag/libbgx_prev.so
