# fused tier-1 overflow causes (stamp build, 8,192 lanes = 32-lane / 12-wave workgroups)
set -o pipefail
export TMPDIR=/tmp; OUT=gpurun_out/r2y; mkdir -p $OUT
BGX_LIB=tools/diag/libbgx_stamp.so timeout -k 10 200 python tools/stamp_fused.py 8192 > $OUT/stamps.json 2> $OUT/stamps.err || { tail $OUT/stamps.err; exit 1; }
cat $OUT/stamps.json
