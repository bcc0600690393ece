# Round-3 session, GPU call 11: LDS-staged reply MLP (mlp_kernel_il v2) and the
# 4-lane top-5 kernel: 2-ply parity, then K=4 / K=all A/B against BGX_MLP_IL=1
# (the previous reply MLP) with kernel traces.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5j; rm -rf $OUT; mkdir -p $OUT
echo "[1] parity"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread -k "two_ply or mlp or value or ply2 or 2ply or reply" > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
ARGS="--ply 2 --k-top 4 --steps 100 --warmup 20 --timing-steps 1 --two-ply-steps 0 --kall-steps 0 --config1-steps 0 --no-cpu-baseline"
for v in new old new old; do
  if [ $v = old ]; then export BGX_MLP_IL=1; else unset BGX_MLP_IL; fi
  timeout -k 10 200 python bench.py $ARGS > $OUT/k4_$v.json 2> $OUT/k4_$v.err || { tail $OUT/k4_$v.err; exit 1; }
  python -c "import json; j=json.load(open('$OUT/k4_$v.json')); print('$v k4', round(j['value']/1e6,3), 'M', round(j['ms_per_step']*1e3,1), 'us/step')"
done
unset BGX_MLP_IL
for v in new old; do
  if [ $v = old ]; then export BGX_MLP_IL=1; else unset BGX_MLP_IL; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt_$v -o run --output-format csv -- python bench.py $ARGS > $OUT/kt_$v.json 2> $OUT/kt_$v.err || { tail $OUT/kt_$v.err; exit 1; }
  f=$(find $OUT/kt_$v -name "*kernel_stats.csv" | head -1); echo "[$v]"; cut -d, -f1-4 $f | head -12
done
unset BGX_MLP_IL
timeout -k 10 300 python bench.py --ply 2 --k-top 0 --steps 20 --warmup 5 --timing-steps 1 --two-ply-steps 0 --kall-steps 0 --config1-steps 0 --no-cpu-baseline > $OUT/kall.json 2> $OUT/kall.err || { tail $OUT/kall.err; exit 1; }
python -c "import json; j=json.load(open('$OUT/kall.json')); print('kall', round(j['value']/1e6,3), 'M', round(j['ms_per_step']*1e3,1), 'us/step')"
