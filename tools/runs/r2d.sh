# Re-entry check: full GPU suite, then the default bench line.
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out/r2d
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r2d/tests.log 2>&1 || { tail -40 gpurun_out/r2d/tests.log; exit 1; }
tail -2 gpurun_out/r2d/tests.log
timeout -k 10 300 python bench.py > gpurun_out/r2d/bench.json 2> gpurun_out/r2d/bench.err || { tail -20 gpurun_out/r2d/bench.err; exit 1; }
tail -c 400 gpurun_out/r2d/bench.json
