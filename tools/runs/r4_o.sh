#!/bin/bash
# round 4: path_state + DMA-staged worker -- movegen / fused / replay / reply /
# drop-in tests, the worker's producer rate, the driver command, the reply
# row-chunk A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4o; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_engine.py tests/test_gpu_replay.py tests/test_gpu_reply.py tests/test_gpu_main.py -x -q --timeout 240 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 300 python tools/queue_bench.py --modes producer > $O/queue_producer.json 2> $O/queue.err || { tail -20 $O/queue.err; exit 1; }
tail -1 $O/queue_producer.json
for i in 1 2; do timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench20_$i.json 2>> $O/bench.err || { tail -20 $O/bench.err; exit 1; }; python tools/ab_line.py bench20_$i $O/bench20_$i.json; done
bash tools/runs/r4_n.sh
