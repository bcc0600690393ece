# Round-3 session, GPU call 8: choice-phase breakdown (prof build timers).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5g; rm -rf $OUT; mkdir -p $OUT
BGX_FUSED_PROF=1 timeout -k 10 200 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --two-ply-steps 0 --kall-steps 0 --config1-steps 0 > $OUT/prof.json 2> $OUT/prof.err || { tail $OUT/prof.err; exit 1; }
grep "fused prof" $OUT/prof.err | head -12
