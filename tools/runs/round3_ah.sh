# Round-3 session 2: per-workgroup spans of a balanced 20-step launch (prof
# build dump): which workgroups end late, and why (steps, tier-2 jobs, rows).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r7ah; rm -rf $OUT; mkdir -p $OUT
for k in 1 2 3; do
  BGX_FUSED_PROF=1 BGX_FUSED_PROF_DUMP=$OUT/wg_20_$k.csv timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --two-ply-steps 0 --kall-steps 0 --config1-steps 0 --timing-steps 20 > $OUT/prof_20_$k.json 2> $OUT/prof_20_$k.err || { tail $OUT/prof_20_$k.err; exit 1; }
  grep "last launch" $OUT/prof_20_$k.err
done
python tools/wg_spans.py $OUT/wg_20_*.csv
