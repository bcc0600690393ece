# pool slice 4 KB: GPU suite on the in-tree build, then A/B against the 8 KB build and PW variants
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out/r2e
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r2e/tests.log 2>&1 || { tail -40 gpurun_out/r2e/tests.log; exit 1; }
tail -2 gpurun_out/r2e/tests.log
bash tools/ab_multi.sh r2e/ab tools/diag/libbgx_prev.so tools/diag/libbgx_pw7.so tools/diag/libbgx_pw16.so
