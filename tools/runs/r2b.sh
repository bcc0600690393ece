set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out/r2b
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r2b/gpu_tests.log 2>&1
rc=$?
tail -30 gpurun_out/r2b/gpu_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 240 python bench.py > gpurun_out/r2b/bench.json 2> gpurun_out/r2b/bench.err || { tail -20 gpurun_out/r2b/bench.err; exit 1; }
tail -c 400 gpurun_out/r2b/bench.json
