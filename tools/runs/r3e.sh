# fused phase clocks (BGX_FUSED_PROF) at 8,192 lanes, 600 steps
set -o pipefail
export TMPDIR=/tmp; OUT=gpurun_out/r3e; mkdir -p $OUT
BGX_FUSED_PROF=1 timeout -k 10 200 python bench.py --steps 600 --warmup 300 --kall-steps 0 --config1-steps 0 --two-ply-steps 0 --no-cpu-baseline --timing-steps 50 > $OUT/bench.json 2> $OUT/prof.txt || { tail $OUT/prof.txt; exit 1; }
grep "fused prof" $OUT/prof.txt
