#!/bin/bash
# round 4: workgroup sub-queue for uncovered roots + direct leaf emission (parity, reply micro,
# 2-ply legs), then the spin-then-block harvest wait A/B on the driver window
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4g; mkdir -p $O
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
python tools/ab_line.py subq_leaf $O/b.json
B="--no-cpu-baseline --two-ply-steps 0 --kall-steps 0 --config1-steps 0 --timing-steps 20"
for rep in 1 2 3; do for sp in 1 0; do
  BGX_SPIN_WAIT=$sp timeout -k 10 200 python bench.py --steps 20 --warmup 5 $B > $O/f_b20_s${sp}_$rep.json 2>> $O/f_b.err || { tail -20 $O/f_b.err; exit 1; }
  python tools/ab_line.py b20_s${sp}_$rep $O/f_b20_s${sp}_$rep.json
done; done
