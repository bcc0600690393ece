#!/bin/bash
# round 4 (re-entry): the new reply-kernel parity tests, the scale / flag /
# determinism tests, the full GPU suite, smoke(), the driver-shaped bench line
# and a 2-ply A/B of the reply kernels (BGX_REPLY_BM=0: per-roll jobs)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4b; mkdir -p $O
B="--no-cpu-baseline --config1-steps 0 --timing-steps 20"
echo "[1] new tests"
timeout -k 10 480 python -u -m pytest tests/test_gpu_reply.py tests/test_gpu_scale.py tests/test_gpu_engine.py -x -v --timeout 240 --timeout-method thread \
  -k "reply or scale or flags or capacity or bench_shape or kall_4096 or same_seed or pipelined" > $O/t1.log 2>&1 || { tail -60 $O/t1.log; exit 1; }
tail -3 $O/t1.log
echo "[2] 2-ply A/B"
for bm in 1 0; do BGX_REPLY_BM=$bm timeout -k 10 300 python bench.py --steps 20 --warmup 5 --two-ply-steps 50 --kall-steps 10 $B > $O/ab_bm$bm.json 2> $O/ab_bm$bm.err || { tail -30 $O/ab_bm$bm.err; exit 1; }; python tools/ab_line.py bm$bm $O/ab_bm$bm.json; done
echo "[3] full gpu suite"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/t2.log 2>&1 || { tail -60 $O/t2.log; exit 1; }
tail -3 $O/t2.log
echo "[4] smoke"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
echo "[5] driver-shaped 20 steps"
for i in 1 2; do timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/b20_$i.json 2>> $O/b20.err || { tail -30 $O/b20.err; exit 1; }; python tools/ab_line.py b20_$i $O/b20_$i.json; done
