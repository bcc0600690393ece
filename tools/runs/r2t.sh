# driver-like short bench (--steps 20 --warmup 5) and the 2-ply legs at configs[2]'s 4,096 lanes
set -o pipefail
export TMPDIR=/tmp; OUT=gpurun_out/r2t; mkdir -p $OUT
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/short.json 2> $OUT/short.err || { tail $OUT/short.err; exit 1; }
python tools/ab_line.py short $OUT/short.json
timeout -k 10 300 python bench.py --lanes 4096 --steps 300 --warmup 100 --two-ply-steps 100 --kall-steps 20 --config1-steps 0 --no-cpu-baseline > $OUT/l4096.json 2> $OUT/l4096.err || { tail $OUT/l4096.err; exit 1; }
python tools/ab_line.py l4096 $OUT/l4096.json
