# rule-mode child move lists: GPU suite, A/B vs previous; then the 2-rank gloo rehearsal on one GPU
set -o pipefail
export TMPDIR=/tmp; OUT=gpurun_out/r2k; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
bash tools/ab_multi.sh r2k/ab tools/diag/libbgx_prev.so || exit 1
R="--steps 600 --warmup 300 --two-ply-steps 0 --kall-steps 0 --config1-steps 0 --no-cpu-baseline --timing-steps 100"
timeout -k 10 300 python bench.py $R --lanes 8192 > $OUT/rank1_8192.json 2> $OUT/rank1.err || { tail $OUT/rank1.err; exit 1; }
BGX_DIST_BACKEND=gloo timeout -k 10 400 python bench.py $R --gpus 2 --lanes 4096 > $OUT/rank2_4096.json 2> $OUT/rank2.err || { tail $OUT/rank2.err; exit 1; }
tail -c 600 $OUT/rank2_4096.json
