#!/bin/bash
# round 5: step durations by index within a launch (prof build) for the
# driver's 20-step window and a 600-step run; then the guarded board-major
# doubles reply test (tools/runs/dbl_guard.sh; last: nothing follows it)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5e; mkdir -p $O
A20="--steps 20 --warmup 5 --kall-steps 0 --config1-steps 0 --two-ply-steps 0 --no-cpu-baseline --timing-steps 0"
A600="--steps 600 --warmup 300 --kall-steps 0 --config1-steps 0 --two-ply-steps 0 --no-cpu-baseline --timing-steps 0"
echo "[1] prof, 20-step window"
BGX_FUSED_PROF=1 timeout -k 10 180 python bench.py $A20 --desync-steps 0 > $O/p20_nodesync.json 2> $O/p20_nodesync.err || { tail -5 $O/p20_nodesync.err; exit 1; }
grep "fused prof" $O/p20_nodesync.err | grep -E "index|queue|last launch"
BGX_FUSED_PROF=1 timeout -k 10 180 python bench.py $A20 > $O/p20.json 2> $O/p20.err || { tail -5 $O/p20.err; exit 1; }
grep "fused prof" $O/p20.err | grep -E "index|queue|last launch"
echo "[2] prof, 600 steps"
BGX_FUSED_PROF=1 timeout -k 10 300 python bench.py $A600 > $O/p600.json 2> $O/p600.err || { tail -5 $O/p600.err; exit 1; }
grep "fused prof" $O/p600.err | grep -E "index|queue|last launch|MLP"
echo "[3] guarded board-major doubles"
bash tools/runs/dbl_guard.sh
