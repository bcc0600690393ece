#!/bin/bash
# round 5, first GPU call: the GPU suite with the wave-uniform sub-queue exit,
# the driver's command, and the fused kernel's phase clocks (MLP tile split)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5a; mkdir -p $O
echo "[1] gpu suite"
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/suite.log 2>&1 || { tail -40 $O/suite.log; exit 1; }
tail -2 $O/suite.log
echo "[2] driver command"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python tools/ab_line.py bench20 $O/bench20.json
echo "[3] phase clocks, 600 steps"
BGX_FUSED_PROF=1 timeout -k 10 300 python bench.py --steps 600 --warmup 300 --timing-steps 0 --two-ply-steps 0 --kall-steps 0 --config1-steps 0 --no-cpu-baseline > $O/prof600.json 2> $O/prof600.err || { tail -20 $O/prof600.err; exit 1; }
grep "fused prof" $O/prof600.err
echo "[4] phase clocks, 20-step window"
BGX_FUSED_PROF=1 BGX_FUSED_PROF_DUMP=$O/wg20.csv timeout -k 10 300 python bench.py --steps 20 --warmup 5 --timing-steps 0 --two-ply-steps 0 --kall-steps 0 --config1-steps 0 --no-cpu-baseline > $O/prof20.json 2> $O/prof20.err || { tail -20 $O/prof20.err; exit 1; }
grep "fused prof" $O/prof20.err
