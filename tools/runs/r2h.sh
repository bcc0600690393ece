# diagnostic: fused tier-1 job section clocks (stamp build)
set -o pipefail
export TMPDIR=/tmp; OUT=gpurun_out/r2h; mkdir -p $OUT
BGX_LIB=tools/diag/libbgx_stamp.so timeout -k 10 200 python tools/stamp_fused.py 8192 > $OUT/stamps.json 2> $OUT/stamps.err || { tail $OUT/stamps.err; exit 1; }
cat $OUT/stamps.json
