#!/bin/bash
# round 4: the reply launch by item group (rocprofv3 kernel stats of
# tools/reply_micro.py children), the two-cursor row reservation A/B in the
# bench's 2-ply legs, and the reply parity tests
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4d; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_reply.py tests/test_gpu_engine.py tests/test_gpu_scale.py -x -q --timeout 240 --timeout-method thread -k "reply or fused or flags or capacity or pipelined or bench_shape" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
B="--no-cpu-baseline --two-ply-steps 0 --kall-steps 0 --config1-steps 0 --timing-steps 20"
for i in 1 2; do timeout -k 10 200 python bench.py --steps 20 --warmup 5 $B > $O/b20_$i.json 2>> $O/b20.err || { tail -20 $O/b20.err; exit 1; }; python tools/ab_line.py b20_$i $O/b20_$i.json; done
timeout -k 10 200 python bench.py --steps 600 --warmup 300 $B > $O/b600.json 2>> $O/b20.err || { tail -20 $O/b20.err; exit 1; }; python tools/ab_line.py b600 $O/b600.json
for cfg in "bm:" "perroll:BGX_REPLY_BM=0" "nd:BGX_REPLY_GROUPS=0x1" "dbl:BGX_REPLY_GROUPS=0x7e"; do
  tag=${cfg%%:*}; envs=${cfg#*:}
  rm -rf $O/prof_$tag
  env $envs BGX_MG_FEW=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$tag -o run --output-format csv -- python tools/reply_micro.py 32768 child > $O/micro_$tag.log 2>&1 || { tail -10 $O/micro_$tag.log; exit 1; }
  f=$(find $O/prof_$tag -name "*kernel_stats.csv" | head -1)
  python tools/kstat.py $f movegen $tag
done
A="--no-cpu-baseline --config1-steps 0 --timing-steps 20 --steps 20 --warmup 5 --two-ply-steps 50 --kall-steps 10"
timeout -k 10 300 python bench.py $A > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
python tools/ab_line.py bm2cursor $O/b.json
