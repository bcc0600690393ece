# compiler scheduling strategy for every kernel: max-ilp / max-memory-clause builds vs the
# in-tree default build; 1-ply 600 steps + 2-ply K=4 100 steps, and the driver's 20-step shape
set -o pipefail
export TMPDIR=/tmp
AB_ARGS="--steps 600 --warmup 300 --kall-steps 0 --config1-steps 0 --two-ply-steps 100 --no-cpu-baseline --timing-steps 100" timeout -k 10 600 bash tools/ab_multi.sh r4f_long tools/diag/libbgx_ilp.so tools/diag/libbgx_mc.so &&
AB_ARGS="--steps 20 --warmup 5 --kall-steps 0 --config1-steps 0 --two-ply-steps 0 --no-cpu-baseline --timing-steps 20" timeout -k 10 400 bash tools/ab_multi.sh r4f_short tools/diag/libbgx_ilp.so tools/diag/libbgx_mc.so
