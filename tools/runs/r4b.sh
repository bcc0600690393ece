# why a 20-step launch runs slower per step than a 600-step one: per-workgroup
# durations of the last fused launch (BGX_FUSED_PROF), 20- and 300-step launches
set -o pipefail
export TMPDIR=/tmp; OUT=gpurun_out/r4b; mkdir -p $OUT
A="--two-ply-steps 0 --kall-steps 0 --config1-steps 0 --no-cpu-baseline"
BGX_FUSED_PROF=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --timing-steps 20 $A > $OUT/prof20.json 2> $OUT/prof20.txt && grep "fused prof" $OUT/prof20.txt &&
BGX_FUSED_PROF=1 timeout -k 10 200 python bench.py --steps 300 --warmup 5 --timing-steps 300 $A > $OUT/prof300.json 2> $OUT/prof300.txt && grep "fused prof" $OUT/prof300.txt
