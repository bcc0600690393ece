# fused 1-ply with 32 lanes per workgroup: fused == phased tests, phase profile, A/B vs the 16-lane build
set -o pipefail
export TMPDIR=/tmp; OUT=gpurun_out/r2g; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py -x -q --timeout 200 --timeout-method thread -k "fused" > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for fl in 16 32; do
BGX_FUSED_LANES=$fl BGX_FUSED_PROF=1 timeout -k 10 200 python bench.py --steps 300 --warmup 100 --two-ply-steps 0 --kall-steps 0 --config1-steps 0 --no-cpu-baseline --timing-steps 100 > $OUT/prof_$fl.json 2> $OUT/prof_$fl.err || exit 1
grep "fused prof" $OUT/prof_$fl.err
done
AB_ARGS="--steps 600 --warmup 300 --kall-steps 0 --two-ply-steps 0 --no-cpu-baseline --timing-steps 300 --config1-steps 300" bash tools/ab_multi.sh r2g/ab tools/diag/libbgx_prev.so
