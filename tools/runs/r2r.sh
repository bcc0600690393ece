# round checkpoint: full GPU suite + smoke + the default bench line
set -o pipefail
export TMPDIR=/tmp; OUT=gpurun_out/r2r; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { tail $OUT/smoke.txt; exit 1; }
tail -1 $OUT/smoke.txt
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python tools/ab_line.py bench $OUT/bench.json
