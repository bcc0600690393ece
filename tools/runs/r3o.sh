# 2-ply K=4 and K=all at 4,096 lanes (round-1 comparison point: 1.185 ms per K=4 step)
set -o pipefail
export TMPDIR=/tmp; OUT=gpurun_out/r3o; mkdir -p $OUT
timeout -k 10 300 python bench.py --lanes 4096 --steps 100 --warmup 50 --kall-steps 20 --config1-steps 0 --two-ply-steps 100 --no-cpu-baseline > $OUT/bench_4096.json 2> $OUT/bench_4096.err || { tail $OUT/bench_4096.err; exit 1; }
python tools/ab_line.py lanes4096 $OUT/bench_4096.json
