set -o pipefail
export TMPDIR=/tmp; OUT=gpurun_out/${1:-kt2}; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/k4 -o run --output-format csv -- python bench.py --ply 2 --k-top 4 --steps 100 --warmup 20 --timing-steps 1 --two-ply-steps 0 --kall-steps 0 --config1-steps 0 --no-cpu-baseline > $OUT/k4.json 2> $OUT/k4.err || { tail $OUT/k4.err; exit 1; }
f=$(find $OUT/k4 -name "*kernel_stats.csv" | head -1); cut -d, -f1-4 $f | head -14
