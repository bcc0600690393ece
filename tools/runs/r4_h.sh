#!/bin/bash
# round 4: reply-launch A/B of the leaf streaming (L) and the sub-queue (Q):
# libbgx_abLQ.so builds, reply micro kernel stats and 2-ply bench legs per build;
# plus, on the in-tree build, the non-doubles group split into covered roots
# only (0x81) and every root as per-roll jobs (0x101)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4h; mkdir -p $O
A="--no-cpu-baseline --config1-steps 0 --timing-steps 20 --steps 20 --warmup 5 --two-ply-steps 50 --kall-steps 10"
for cfg in "nd:0x1" "cov:0x81" "unc:0x101"; do
  tag=${cfg%%:*}; g=${cfg#*:}
  rm -rf $O/prof_$tag
  BGX_REPLY_GROUPS=$g BGX_MG_FEW=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$tag -o run --output-format csv -- python tools/reply_micro.py 32768 child > $O/micro_$tag.log 2>&1 || { tail -10 $O/micro_$tag.log; exit 1; }
  python tools/kstat.py $(find $O/prof_$tag -name "*kernel_stats.csv" | head -1) movegen $tag
done
for rep in 1 2; do
  for lib in tools/diag/libbgx_ab00.so tools/diag/libbgx_ab10.so tools/diag/libbgx_ab01.so tools/diag/libbgx_ab11.so; do
    tag=$(basename $lib .so)
    if [ $rep = 1 ]; then
      rm -rf $O/prof_$tag
      BGX_LIB=$lib BGX_MG_FEW=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$tag -o run --output-format csv -- python tools/reply_micro.py 32768 child > $O/micro_$tag.log 2>&1 || { tail -10 $O/micro_$tag.log; exit 1; }
      python tools/kstat.py $(find $O/prof_$tag -name "*kernel_stats.csv" | head -1) movegen $tag
    fi
    BGX_LIB=$lib timeout -k 10 300 python bench.py $A > $O/b_${tag}_$rep.json 2> $O/b_${tag}_$rep.err || { tail -20 $O/b_${tag}_$rep.err; exit 1; }
    python tools/ab_line.py ${tag}_$rep $O/b_${tag}_$rep.json
  done
done
