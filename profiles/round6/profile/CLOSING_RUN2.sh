#!/bin/bash
# round 6 closing check on the final tree: the GPU suite, smoke(), the driver's command
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6final2; mkdir -p $O
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/suite.log 2>&1 || { tail -40 $O/suite.log; exit 1; }
tail -2 $O/suite.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python tools/ab_line.py bench20 $O/bench20.json
