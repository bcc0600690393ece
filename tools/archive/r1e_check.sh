# GPU check: the GPU test suite, the movegen split micro-benchmark, a 2-ply
# A/B of the tier-1 (pool) and reply-MLP (prefetch, zero-k-step skip)
# variants, and the default bench line. Output under gpurun_out/r1e/.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r1e
rm -rf $OUT; mkdir -p $OUT
echo "[1/4] gpu tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.txt 2>&1 || { tail -40 $OUT/tests.txt; exit 1; }
tail -3 $OUT/tests.txt
echo "[2/4] movegen split"
timeout -k 10 200 python tools/mg_micro.py 200000 > $OUT/mg.txt 2>&1 || { tail -20 $OUT/mg.txt; exit 1; }
cat $OUT/mg.txt
echo "[3/4] 2-ply A/B (pool pref skip)"
for v in "0 0 0" "1 0 0"; do
  set -- $v
  BGX_MG_POOL=$1 BGX_MLP_PREF=$2 BGX_MLP_SKIP=$3 timeout -k 10 300 python bench.py --ply 2 --steps 200 --warmup 50 \
    --two-ply-steps 0 --kall-steps 0 --no-cpu-baseline > $OUT/ab_$1$2$3.json 2> $OUT/ab_$1$2$3.err || { tail -20 $OUT/ab_$1$2$3.err; exit 1; }
  python tools/ab_line.py "pool=$1 pref=$2 skip=$3" $OUT/ab_$1$2$3.json
done
for p in 0 1; do
  BGX_MG_POOL=$p timeout -k 10 300 python bench.py --ply 2 --k-top 0 --steps 20 --warmup 5 --timing-steps 10 \
    --two-ply-steps 0 --kall-steps 0 --no-cpu-baseline > $OUT/kall_$p.json 2> $OUT/kall_$p.err || { tail -20 $OUT/kall_$p.err; exit 1; }
  python tools/ab_line.py "K=all pool=$p" $OUT/kall_$p.json
done
echo "[4/4] bench (default command)"
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python tools/ab_line.py default $OUT/bench.json
