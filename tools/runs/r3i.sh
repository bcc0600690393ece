# cooperative tier 2 at 12 waves only: A/B at 4,096 lanes (16-lane workgroups, 8 waves) and 8,192, then phase clocks with the last-round wait
set -o pipefail
export TMPDIR=/tmp; OUT=gpurun_out/r3i; mkdir -p $OUT
AB_ARGS="--lanes 4096 --steps 600 --warmup 300 --kall-steps 0 --config1-steps 0 --two-ply-steps 0 --no-cpu-baseline --timing-steps 100" timeout -k 10 500 bash tools/ab_multi.sh r3i_4096 tools/diag/libbgx_prev.so &&
AB_ARGS="--steps 600 --warmup 300 --kall-steps 0 --config1-steps 0 --two-ply-steps 0 --no-cpu-baseline --timing-steps 100" timeout -k 10 500 bash tools/ab_multi.sh r3i_8192 tools/diag/libbgx_prev.so &&
BGX_FUSED_PROF=1 timeout -k 10 200 python bench.py --steps 600 --warmup 300 --kall-steps 0 --config1-steps 0 --two-ply-steps 0 --no-cpu-baseline --timing-steps 50 > $OUT/prof_bench.json 2> $OUT/prof.txt && grep "fused prof" $OUT/prof.txt
