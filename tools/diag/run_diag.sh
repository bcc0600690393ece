set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out/diag
timeout -k 10 200 python -u tools/diag/two_ply_diag.py 2>&1 | tee gpurun_out/diag/new.log || exit 1
BGX_LIB=tools/diag/libbgx_prev.so timeout -k 10 200 python -u tools/diag/two_ply_diag.py 2>&1 | tee gpurun_out/diag/prev.log || exit 1
BGX_MG_TEST_TIER=2 timeout -k 10 200 python -u tools/diag/two_ply_diag.py 2>&1 | tee gpurun_out/diag/tier2.log || exit 1
