#!/bin/bash
# round 4: board-major doubles (BGX_DBL_BM=1 build, bgx/libbgx_dbl.so) -- reply
# parity + 2-ply engine tests on that build, reply micro by group with
# instruction counts (both builds), 2-ply legs A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4p; mkdir -p $O
DBL=$PWD/mlp-ppo-2ply-multi_amd/bgx/libbgx_dbl.so
BGX_LIB=$DBL timeout -k 10 400 python -u -m pytest tests/test_gpu_reply.py tests/test_gpu_engine.py tests/test_gpu_scale.py -x -q --timeout 240 --timeout-method thread -k "reply or 2ply or two_ply or kall or same_seed" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for lib in base dbl; do
  if [ $lib = dbl ]; then export BGX_LIB=$DBL; else unset BGX_LIB; fi
  for cfg in "bm:0x0" "dbl:0x7e"; do
    tag=${lib}_${cfg%%:*}; g=${cfg#*:}
    rm -rf $O/prof_$tag $O/pmc_$tag
    BGX_REPLY_GROUPS=$g BGX_MG_FEW=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$tag -o run --output-format csv -- python tools/reply_micro.py 32768 child > $O/micro_$tag.log 2>&1 || { tail -10 $O/micro_$tag.log; exit 1; }
    python tools/kstat.py $(find $O/prof_$tag -name "*kernel_stats.csv" | head -1) movegen $tag
    BGX_REPLY_GROUPS=$g BGX_MG_FEW=0 timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-include-regex movegen_reply -d $O/pmc_$tag -o run --output-format csv -- python tools/reply_micro.py 32768 child > $O/pmc_$tag.log 2>&1 || { tail -5 $O/pmc_$tag.log; exit 1; }
    python - $O/pmc_$tag $tag <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(float); disp = set()
for r in csv.DictReader(open(f)):
    disp.add(r.get("Dispatch_Id")); acc[r["Counter_Name"]] += float(r["Counter_Value"])
n = len(disp)
print(sys.argv[2], "dispatches", n, {k: round(v / n / 32768, 1) for k, v in sorted(acc.items())}, "(per candidate)")
PY
  done
done
unset BGX_LIB
A="--no-cpu-baseline --config1-steps 0 --timing-steps 20 --steps 20 --warmup 5 --two-ply-steps 50 --kall-steps 10"
for rep in 1 2; do for lib in base dbl; do
  if [ $lib = dbl ]; then L="BGX_LIB=$DBL"; else L=""; fi
  env $L timeout -k 10 300 python bench.py $A > $O/b_${lib}_$rep.json 2> $O/b_${lib}_$rep.err || { tail -20 $O/b_${lib}_$rep.err; exit 1; }
  python tools/ab_line.py ${lib}_$rep $O/b_${lib}_$rep.json
done; done
