# 16-wave pool default: K=4 step timeline (kernel trace) + movegen split by dice kind
set -o pipefail
export TMPDIR=/tmp; OUT=gpurun_out/r2f; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/k4 -o run --output-format csv -- python bench.py --ply 2 --k-top 4 --steps 60 --warmup 20 --timing-steps 1 --two-ply-steps 0 --kall-steps 0 --config1-steps 0 --no-cpu-baseline > $OUT/k4.json 2> $OUT/k4.err || { tail $OUT/k4.err; exit 1; }
f=$(find $OUT/k4 -name "*kernel_trace.csv" | head -1); python tools/step_timeline.py $f movegen_few_kernel 40 > $OUT/timeline.txt; cat $OUT/timeline.txt
timeout -k 10 200 python tools/mg_micro.py 300000 > $OUT/micro.json 2> $OUT/micro.err || { tail $OUT/micro.err; exit 1; }
cat $OUT/micro.json
