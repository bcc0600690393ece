#!/bin/bash
# round 5: per-roll tail 4/64 as the default: 2-ply GPU tests, the driver's command
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5u; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_reply.py tests/test_gpu_engine.py tests/test_gpu_replay.py tests/test_gpu_scale.py -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python tools/ab_line.py bench20 $O/bench20.json
