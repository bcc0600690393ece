# development: fused-kernel phase profile per BGX_FUSED_EXP variant
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out/fexp
[ -n "$SKIPT" ] || timeout -k 10 200 python -u -m pytest tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread -k "fused_step_matches and not tier" > gpurun_out/fexp/t.log 2>&1 || { tail -30 gpurun_out/fexp/t.log; exit 1; }
for x in ${@:-0 1}; do
  BGX_FUSED_EXP=$x BGX_FUSED_PROF=1 timeout -k 10 200 python bench.py --steps 300 --warmup 100 --two-ply-steps 0 --kall-steps 0 --no-cpu-baseline --timing-steps 100 > gpurun_out/fexp/p$x.json 2> gpurun_out/fexp/p$x.err || exit 1
  echo "exp=$x"; grep "fused prof" gpurun_out/fexp/p$x.err
  BGX_FUSED_EXP=$x timeout -k 10 200 python bench.py --steps 400 --warmup 100 --two-ply-steps 0 --kall-steps 0 --no-cpu-baseline --timing-steps 100 > gpurun_out/fexp/b$x.json 2> gpurun_out/fexp/b$x.err || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/fexp/b$x.json').read().strip().splitlines()[-1]);print('exp=$x', round(d['value']/1e6,2),'M', round(d['ms_per_step']*1e3,1),'us/step')"
done
