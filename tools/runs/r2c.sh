set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out/r2c
timeout -k 10 600 python -u -m pytest tests/test_gpu_replay.py -v --timeout 300 --timeout-method thread > gpurun_out/r2c/replay.log 2>&1
rc=$?
tail -15 gpurun_out/r2c/replay.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/sq_counters.sh r2c 2ply_k4 "movegen_pool|mlp_kernel_il" || exit 1
