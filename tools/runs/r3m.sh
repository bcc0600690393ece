# features from a 16-entry nibble table (two conflict-free 8-byte reads) in the fused and MLP kernels:
# GPU suite, A/B (1-ply + 2-ply K=4 long, 20-step short, 4,096 lanes), phase clocks
set -o pipefail
export TMPDIR=/tmp; OUT=gpurun_out/r3m; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 600 bash tools/ab_multi.sh r3m_long tools/diag/libbgx_prev.so &&
AB_ARGS="--steps 20 --warmup 5 --kall-steps 0 --config1-steps 0 --two-ply-steps 0 --no-cpu-baseline --timing-steps 20" timeout -k 10 400 bash tools/ab_multi.sh r3m_short tools/diag/libbgx_prev.so &&
AB_ARGS="--lanes 4096 --steps 600 --warmup 300 --kall-steps 0 --config1-steps 0 --two-ply-steps 0 --no-cpu-baseline --timing-steps 100" timeout -k 10 500 bash tools/ab_multi.sh r3m_4096 tools/diag/libbgx_prev.so &&
BGX_FUSED_PROF=1 timeout -k 10 200 python bench.py --steps 600 --warmup 300 --kall-steps 0 --config1-steps 0 --two-ply-steps 0 --no-cpu-baseline --timing-steps 50 > $OUT/prof_bench.json 2> $OUT/prof.txt && grep "fused prof" $OUT/prof.txt
