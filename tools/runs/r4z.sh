# final-tree rehearsal: GPU suite, smoke(), the driver bench command, the default bench
set -o pipefail
export TMPDIR=/tmp; OUT=gpurun_out/r4z; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err || { tail $OUT/bench_driver.err; exit 1; }
python tools/ab_line.py driver $OUT/bench_driver.json
timeout -k 10 300 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail $OUT/bench_default.err; exit 1; }
python tools/ab_line.py default $OUT/bench_default.json
