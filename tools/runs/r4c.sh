# packed-fp32 epilogue in the fused kernel's MLP items (in-tree) vs the previous build
set -o pipefail
export TMPDIR=/tmp
AB_ARGS="--steps 600 --warmup 300 --kall-steps 0 --config1-steps 0 --two-ply-steps 0 --no-cpu-baseline --timing-steps 100" timeout -k 10 500 bash tools/ab_multi.sh r4c_long tools/diag/libbgx_prev.so &&
AB_ARGS="--steps 20 --warmup 5 --kall-steps 0 --config1-steps 0 --two-ply-steps 0 --no-cpu-baseline --timing-steps 20" timeout -k 10 400 bash tools/ab_multi.sh r4c_short tools/diag/libbgx_prev.so
