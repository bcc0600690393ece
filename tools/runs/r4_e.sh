#!/bin/bash
# round 4: deferred uncovered-root jobs + direct leaf emission for path doubles
# in the reply launch: parity tests, reply micro by group, 2-ply bench legs
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4e; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_reply.py tests/test_gpu_engine.py tests/test_gpu_replay.py tests/test_gpu_scale.py tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread -k "reply or two_ply or 2ply or kall or same_seed or movegen" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for cfg in "bm:" "nd:BGX_REPLY_GROUPS=0x1" "dbl:BGX_REPLY_GROUPS=0x7e"; do
  tag=${cfg%%:*}; envs=${cfg#*:}
  rm -rf $O/prof_$tag
  env $envs BGX_MG_FEW=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$tag -o run --output-format csv -- python tools/reply_micro.py 32768 child > $O/micro_$tag.log 2>&1 || { tail -10 $O/micro_$tag.log; exit 1; }
  f=$(find $O/prof_$tag -name "*kernel_stats.csv" | head -1)
  python tools/kstat.py $f movegen $tag
done
A="--no-cpu-baseline --config1-steps 0 --timing-steps 20 --steps 20 --warmup 5 --two-ply-steps 50 --kall-steps 10"
timeout -k 10 300 python bench.py $A > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
python tools/ab_line.py defer_leaf $O/b.json
