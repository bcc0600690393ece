# Fused-kernel GPU check: parity tests (-k fused), phase profile (BGX_FUSED_PROF), fused vs phased bench.
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out/fused
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -x -v --timeout 120 --timeout-method thread -k "fused or transitions_match or sampling or greedy" > gpurun_out/fused/t.log 2>&1 || { tail -40 gpurun_out/fused/t.log; exit 1; }
tail -2 gpurun_out/fused/t.log
BGX_FUSED_PROF=1 timeout -k 10 200 python bench.py --steps 300 --warmup 100 --two-ply-steps 0 --kall-steps 0 --no-cpu-baseline --timing-steps 100 > gpurun_out/fused/prof.json 2> gpurun_out/fused/prof.err || exit 1
grep "fused prof" gpurun_out/fused/prof.err
for m in "" "--no-fused"; do
  timeout -k 10 200 python bench.py --steps 400 --warmup 100 --two-ply-steps 0 --kall-steps 0 --no-cpu-baseline --timing-steps 100 $m > gpurun_out/fused/b$m.json 2>gpurun_out/fused/b$m.err || { tail -20 gpurun_out/fused/b$m.err; exit 1; }
  python -c "import json,sys;d=json.loads(open('gpurun_out/fused/b$m.json').read().strip().splitlines()[-1]);print('$m', round(d['value']/1e6,2),'M', round(d['ms_per_step']*1e3,1),'us/step', d['roofline'])"
done
