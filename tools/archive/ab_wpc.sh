# A/B: fused 1-ply kernel with 1 workgroup per CU (W in LDS) vs 2 (W from global)
set -o pipefail
export TMPDIR=/tmp; OUT=gpurun_out/${1:-ab_wpc}; mkdir -p $OUT
ARGS="--steps 600 --warmup 300 --two-ply-steps 0 --kall-steps 0 --config1-steps 0 --no-cpu-baseline --timing-steps 300"
for wpc in 1 2; do
  for lanes in 8192 16384; do
    BGX_FUSED_WPC=$wpc timeout -k 10 120 python bench.py $ARGS --lanes $lanes > $OUT/b_${wpc}_${lanes}.json 2> $OUT/b_${wpc}_${lanes}.err || { tail -5 $OUT/b_${wpc}_${lanes}.err; exit 1; }
    python -c "import json,sys;d=json.loads(open('$OUT/b_${wpc}_${lanes}.json').read().strip().splitlines()[-1]);print('wpc $wpc lanes $lanes', round(d['value']/1e6,2),'M', round(d['ms_per_step']*1e3,1),'us/step', 'kernel', round(d['kernels']['fused_step']['avg_launch_ms'],3),'ms/launch')"
  done
  BGX_FUSED_WPC=$wpc BGX_FUSED_PROF=1 timeout -k 10 120 python bench.py $ARGS --lanes 8192 > $OUT/p_${wpc}.json 2> $OUT/p_${wpc}.err || exit 1
  grep "fused prof" $OUT/p_${wpc}.err
done
BGX_FUSED_WPC=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -k "fused" -v --timeout 200 --timeout-method thread > $OUT/tests_wpc2.log 2>&1; tail -6 $OUT/tests_wpc2.log
