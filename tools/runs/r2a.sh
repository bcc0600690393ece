set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out/r2a
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r2a/gpu_tests.log 2>&1 || { tail -40 gpurun_out/r2a/gpu_tests.log; exit 1; }
tail -2 gpurun_out/r2a/gpu_tests.log
timeout -k 10 300 python bench.py > gpurun_out/r2a/bench.json 2> gpurun_out/r2a/bench.err || { tail -20 gpurun_out/r2a/bench.err; exit 1; }
tail -c 600 gpurun_out/r2a/bench.json
