# fused 1-ply with 12 waves per workgroup (3 per SIMD, 168 registers, 3.5 KB slices): fused tests on the variant, phase profile, A/B
set -o pipefail
export TMPDIR=/tmp; OUT=gpurun_out/r2p; mkdir -p $OUT
BGX_LIB=tools/diag/libbgx_nw12.so timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_replay.py -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for lib in mlp-ppo-2ply-multi_amd/bgx/libbgx.so tools/diag/libbgx_nw12.so; do
tag=$(basename $lib .so)
BGX_LIB=$lib BGX_FUSED_PROF=1 timeout -k 10 200 python bench.py --steps 300 --warmup 100 --two-ply-steps 0 --kall-steps 0 --config1-steps 0 --no-cpu-baseline --timing-steps 100 > $OUT/prof_$tag.json 2> $OUT/prof_$tag.err || exit 1
grep "fused prof" $OUT/prof_$tag.err
done
AB_ARGS="--steps 600 --warmup 300 --kall-steps 0 --two-ply-steps 0 --no-cpu-baseline --timing-steps 300 --config1-steps 300" bash tools/ab_multi.sh r2p/ab tools/diag/libbgx_nw12.so
