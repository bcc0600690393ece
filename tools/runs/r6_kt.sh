# per-kernel durations of the 2-ply K=4 bench leg, delta (default) and full reply MLP
set -o pipefail
export TMPDIR=/tmp; OUT=gpurun_out/r6kt; mkdir -p $OUT
for d in 1 0; do
  BGX_REPLY_DELTA=$d timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/k4_$d -o run --output-format csv -- python bench.py --ply 2 --k-top 4 --steps 60 --warmup 10 --timing-steps 1 --two-ply-steps 0 --kall-steps 0 --config1-steps 0 --config2-steps 0 --no-cpu-baseline > $OUT/k4_$d.json 2> $OUT/k4_$d.err || { tail $OUT/k4_$d.err; exit 1; }
  f=$(find $OUT/k4_$d -name "*kernel_stats.csv" | head -1); echo "== delta=$d"; cut -d, -f1-5 $f | head -14
done
