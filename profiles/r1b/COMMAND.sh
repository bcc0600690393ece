# Round profile (GPU box): bench line, rocprofv3 kernel stats of the same
# command, FETCH_SIZE / WRITE_SIZE passes per leg. Output: gpurun_out/$1/
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-prof}
rm -rf $OUT; mkdir -p $OUT
echo "[1/6] bench (default command)"
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
tail -1 $OUT/bench.json
echo "[2/6] kernel trace + stats of the bench command"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/ktrace -o run --output-format csv -- python bench.py --no-cpu-baseline > $OUT/bench_under_rocprof.json 2> $OUT/ktrace.err || exit 1
for leg in 1 2; do
  if [ $leg = 1 ]; then ARGS="--steps 200 --warmup 50 --two-ply-steps 0 --timing-steps 1 --no-cpu-baseline"; else ARGS="--ply 2 --steps 60 --warmup 20 --two-ply-steps 0 --timing-steps 1 --no-cpu-baseline"; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    echo "[pmc] leg ${leg}-ply $c"
    timeout -k 10 600 rocprofv3 --pmc $c --kernel-include-regex "movegen|mlp_kernel" -d $OUT/pmc_${leg}_$c -o run --output-format csv -- python bench.py $ARGS > $OUT/pmc_${leg}_$c.log 2>&1 || exit 1
  done
done
echo "[6/6] summarise"
python tools/pmc_summary.py $OUT > $OUT/pmc_traffic.json && cat $OUT/pmc_traffic.json
