# exact frontier check in expand_flat: overflow counts + A/B vs the previous build (long and driver-like runs)
set -o pipefail
export TMPDIR=/tmp; OUT=gpurun_out/r2z; mkdir -p $OUT
BGX_LIB=tools/diag/libbgx_stamp.so timeout -k 10 200 python tools/stamp_fused.py 8192 > $OUT/stamps.json 2> $OUT/stamps.err || { tail $OUT/stamps.err; exit 1; }
grep overflow $OUT/stamps.json
timeout -k 10 600 bash tools/ab_multi.sh r2z_long tools/diag/libbgx_prev.so &&
AB_ARGS="--steps 20 --warmup 5 --kall-steps 0 --config1-steps 0 --two-ply-steps 20 --no-cpu-baseline" timeout -k 10 400 bash tools/ab_multi.sh r2z_short tools/diag/libbgx_prev.so
