# fused prologue: W fragment loads batched (in-tree) / + tier-1 queue pop read at the
# end of the job (libbgx_poplate) vs the previous build; long, short, launch cost
set -o pipefail
export TMPDIR=/tmp; OUT=gpurun_out/r4e; mkdir -p $OUT
AB_ARGS="--steps 600 --warmup 300 --kall-steps 0 --config1-steps 0 --two-ply-steps 0 --no-cpu-baseline --timing-steps 100" timeout -k 10 500 bash tools/ab_multi.sh r4e_long tools/diag/libbgx_poplate.so tools/diag/libbgx_prev.so &&
AB_ARGS="--steps 20 --warmup 5 --kall-steps 0 --config1-steps 0 --two-ply-steps 0 --no-cpu-baseline --timing-steps 20" timeout -k 10 400 bash tools/ab_multi.sh r4e_short tools/diag/libbgx_poplate.so tools/diag/libbgx_prev.so &&
timeout -k 10 200 python tools/launch_cost.py > $OUT/cost.txt 2> $OUT/cost.err && cat $OUT/cost.txt
