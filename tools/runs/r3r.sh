# fused MLP item pairs with fragments 3 k-steps ahead: fused tests, A/B, phase clocks
set -o pipefail
export TMPDIR=/tmp; OUT=gpurun_out/r3r; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -x -q -m gpu -k fused --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
AB_ARGS="--steps 600 --warmup 300 --kall-steps 0 --config1-steps 0 --two-ply-steps 0 --no-cpu-baseline --timing-steps 100" timeout -k 10 500 bash tools/ab_multi.sh r3r_long tools/diag/libbgx_prev.so &&
AB_ARGS="--steps 20 --warmup 5 --kall-steps 0 --config1-steps 0 --two-ply-steps 0 --no-cpu-baseline --timing-steps 20" timeout -k 10 400 bash tools/ab_multi.sh r3r_short tools/diag/libbgx_prev.so &&
AB_ARGS="--lanes 4096 --steps 600 --warmup 300 --kall-steps 0 --config1-steps 0 --two-ply-steps 0 --no-cpu-baseline --timing-steps 100" timeout -k 10 500 bash tools/ab_multi.sh r3r_4096 tools/diag/libbgx_prev.so &&
BGX_FUSED_PROF=1 timeout -k 10 200 python bench.py --steps 600 --warmup 300 --kall-steps 0 --config1-steps 0 --two-ply-steps 0 --no-cpu-baseline --timing-steps 50 > $OUT/prof_bench.json 2> $OUT/prof.txt && grep "fused prof" $OUT/prof.txt
