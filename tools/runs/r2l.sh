# top-5 via DPP row max + MLP epilogue spread over all k-steps: GPU suite, A/B, K=4 timelines
set -o pipefail
export TMPDIR=/tmp; OUT=gpurun_out/r2l; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
bash tools/ab_multi.sh r2l/ab tools/diag/libbgx_prev.so || exit 1
bash tools/timeline_ab.sh r2l/tl tools/diag/libbgx_prev.so
