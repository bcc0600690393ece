# trainer kernel timing: micro-benchmark + rocprof kernel stats
set -o pipefail
export TMPDIR=/tmp; OUT=gpurun_out/r2w; mkdir -p $OUT
timeout -k 10 300 python tools/train_micro.py 10 > $OUT/micro.json 2> $OUT/micro.err || { tail $OUT/micro.err; exit 1; }
cat $OUT/micro.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python tools/train_micro.py 10 > $OUT/kt.json 2> $OUT/kt.err || { tail $OUT/kt.err; exit 1; }
f=$(find $OUT/kt -name "*kernel_stats.csv" | head -1); cut -d, -f1-4 $f > $OUT/kstats.txt; head -4 $OUT/kstats.txt
