# why the driver-like short run is slower: warmup vs steps, phase split at 20 steps after 5
set -o pipefail
export TMPDIR=/tmp; OUT=gpurun_out/r2u; mkdir -p $OUT
A="--two-ply-steps 0 --kall-steps 0 --config1-steps 0 --no-cpu-baseline"
for sw in "20 300" "300 5" "20 5" "100 5" "20 50"; do
  set -- $sw
  timeout -k 10 200 python bench.py --steps $1 --warmup $2 $A > $OUT/s$1_w$2.json 2> $OUT/s$1_w$2.err || exit 1
  python tools/ab_line.py "steps $1 warmup $2" $OUT/s$1_w$2.json
done
BGX_FUSED_PROF=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --timing-steps 20 $A > $OUT/prof.json 2> $OUT/prof.err || exit 1
grep "fused prof" $OUT/prof.err
