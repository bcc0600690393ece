#!/bin/bash
# round 6 closing run: the GPU suite, smoke(), the driver's command twice (the
# round profile ran before it: tools/profile_round.sh r6prof)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6final; mkdir -p $O
echo "[1] gpu suite"
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/suite.log 2>&1 || { tail -40 $O/suite.log; exit 1; }
tail -2 $O/suite.log
echo "[2] smoke"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
echo "[3] driver command"
for i in 1 2; do timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench20_$i.json 2>> $O/bench.err || { tail -20 $O/bench.err; exit 1; }; python tools/ab_line.py bench20_$i $O/bench20_$i.json; done
