# Round profile (GPU box): the default bench line, rocprofv3 kernel trace +
# stats of the same command, FETCH_SIZE / WRITE_SIZE passes per leg and the SQ
# counter passes (never combined with tracing; one counter group per pass).
# Legs: "1ply_fused" = the fused step kernel (300 steps per dispatch, 8,192 lanes),
#       "2ply_k4" = the phased 2-ply K=4 step (movegen + MLP kernels, 8,192 lanes),
#       "2ply_kall" = the phased 2-ply K=all step (same kernels, every candidate).
# $2 = a lane count other than 8,192 (4096: configs[1] / configs[2]): only the
# PMC and SQ passes, at that lane count, legs named l<lanes>_<leg> (bench.py
# reads them for its legs at that lane count); the output dir is kept.
# Output: gpurun_out/$1/
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-prof}
LANES=${2:-8192}
if [ $LANES = 8192 ]; then
  P=""; LA=""
  rm -rf $OUT; mkdir -p $OUT
  echo "[1/4] bench (the driver command: --steps 20 --warmup 5)"
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
  tail -c 300 $OUT/bench.json
  echo "[2/4] kernel trace + stats of the bench command"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/ktrace -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_under_rocprof.json 2> $OUT/ktrace.err || { tail $OUT/ktrace.err; exit 1; }
else
  P="l${LANES}_"; LA="--lanes $LANES"
  mkdir -p $OUT
fi
echo "[3/4] PMC traffic passes ($LANES lanes)"
for leg in 1ply_fused 2ply_k4 2ply_kall; do
  if [ $leg = 1ply_fused ]; then
    ARGS="--steps 600 --warmup 300 --timing-steps 300 --two-ply-steps 0 --kall-steps 0 --config1-steps 0 --config2-steps 0 --no-cpu-baseline"; RX="fused_step"
  elif [ $leg = 2ply_k4 ]; then
    ARGS="--ply 2 --steps 60 --warmup 20 --timing-steps 1 --two-ply-steps 0 --kall-steps 0 --config1-steps 0 --config2-steps 0 --no-cpu-baseline"; RX="movegen|mlp_kernel"
  else
    ARGS="--ply 2 --k-top 0 --steps 10 --warmup 2 --desync-steps 60 --timing-steps 1 --two-ply-steps 0 --kall-steps 0 --config1-steps 0 --config2-steps 0 --no-cpu-baseline"; RX="movegen|mlp_kernel"
  fi
  for c in FETCH_SIZE WRITE_SIZE; do
    echo "[pmc] $P$leg $c"
    timeout -s KILL 300 rocprofv3 --pmc $c --kernel-include-regex "$RX" -d $OUT/pmc_$P${leg}_$c -o run --output-format csv -- python bench.py $ARGS $LA > $OUT/pmc_$P${leg}_$c.log 2>&1 || { tail -5 $OUT/pmc_$P${leg}_$c.log; exit 1; }
  done
done
echo "[4/4] SQ counter passes"
bash tools/sq_counters.sh ${1:-prof} 2ply_k4 "movegen_reply|mlp_kernel_il" $LANES > /dev/null || exit 1
bash tools/sq_counters.sh ${1:-prof} 1ply "fused_step" $LANES > /dev/null || exit 1
bash tools/sq_counters.sh ${1:-prof} 2ply_kall "movegen_reply|mlp_kernel_il" $LANES > /dev/null || exit 1
python tools/pmc_summary.py $OUT > $OUT/pmc_traffic.json && cat $OUT/pmc_traffic.json | head -30
