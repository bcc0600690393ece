# 12-wave reply MLP (mlp_kernel_il3) A/B: 2-ply parity tests on the variant, A/B, timelines
set -o pipefail
export TMPDIR=/tmp; OUT=gpurun_out/r2n; mkdir -p $OUT
BGX_LIB=tools/diag/libbgx_il3.so timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "2ply or two_ply" > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
bash tools/ab_multi.sh r2n/ab tools/diag/libbgx_il3.so || exit 1
bash tools/timeline_ab.sh r2n/tl tools/diag/libbgx_il3.so
