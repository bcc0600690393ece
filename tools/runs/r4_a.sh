#!/bin/bash
# round 4: new scale / flag tests, the full GPU suite, A/B against the HEAD build
# (tools/diag/libbgx_base.so: no bar rule), driver-shaped lines, a prof run
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4a; mkdir -p $O
B="--no-cpu-baseline --two-ply-steps 0 --kall-steps 0 --config1-steps 0"
echo "[1] new tests"
timeout -k 10 420 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_engine.py -x -v --timeout 200 --timeout-method thread \
  -k "scale or flags or capacity or bench_shape or kall_4096 or same_seed or pipelined" > $O/t1.log 2>&1 || { tail -40 $O/t1.log; exit 1; }
tail -3 $O/t1.log
echo "[2] full gpu suite"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/t2.log 2>&1 || { tail -40 $O/t2.log; exit 1; }
tail -3 $O/t2.log
echo "[3] A/B vs base"
AB_ARGS="--steps 600 --warmup 300 --kall-steps 10 --config1-steps 0 --two-ply-steps 100 --no-cpu-baseline --timing-steps 300" \
  bash tools/ab_multi.sh r4a/ab tools/diag/libbgx_base.so tools/diag/libbgx_pf.so || exit 1
echo "[4] driver-shaped 20 steps"
for i in 1 2; do timeout -k 10 200 python bench.py --steps 20 --warmup 5 $B > $O/b20_$i.json 2>> $O/b20.err || exit 1; python tools/ab_line.py b20_$i $O/b20_$i.json; done
echo "[5] prof"
BGX_FUSED_PROF=1 timeout -k 10 200 python bench.py --steps 300 --warmup 0 --timing-steps 1 $B > $O/prof.json 2> $O/prof.err || { tail $O/prof.err; exit 1; }
grep "fused prof" $O/prof.err | tail -14
