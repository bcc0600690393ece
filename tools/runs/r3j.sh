# fused phase clocks with the tier-1 queue-pop overhead
set -o pipefail
export TMPDIR=/tmp; OUT=gpurun_out/r3j; mkdir -p $OUT
BGX_FUSED_PROF=1 timeout -k 10 200 python bench.py --steps 600 --warmup 300 --kall-steps 0 --config1-steps 0 --two-ply-steps 0 --no-cpu-baseline --timing-steps 50 > $OUT/prof_bench.json 2> $OUT/prof.txt && grep "fused prof" $OUT/prof.txt
