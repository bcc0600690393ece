# share of the bear-off-range (uncovered) reply roots in the reply movegen launch:
# BGX_REPLY_GROUPS=0x7f runs every item, 0xff leaves the uncovered roots' 15
# non-doubles per-roll jobs out (bgx_movegen.hip reply_groups & 0x80 hook)
set -o pipefail
export TMPDIR=/tmp; OUT=gpurun_out/r6bo; mkdir -p $OUT
for g in 0x7f 0xff 0x7f 0xff; do
  rm -rf $OUT/p_$g
  BGX_REPLY_GROUPS=$g BGX_MG_FEW=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/p_$g -o run --output-format csv -- python tools/reply_micro.py 32768 child > $OUT/m_$g.log 2>&1 || { tail -10 $OUT/m_$g.log; exit 1; }
  f=$(find $OUT/p_$g -name "*kernel_stats.csv" | head -1); echo "== $g"; grep -E "movegen_reply|movegen_block" $f | cut -d, -f1-4
done
