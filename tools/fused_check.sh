# GPU check for the fused 1-ply step kernel: parity tests, then fused vs phased bench legs.
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out/fused
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -x -v --timeout 120 --timeout-method thread -k "fused" > gpurun_out/fused/t.log 2>&1 || { tail -40 gpurun_out/fused/t.log; exit 1; }
tail -3 gpurun_out/fused/t.log
for m in "" "--no-fused"; do
  timeout -k 10 200 python bench.py --steps 400 --warmup 100 --two-ply-steps 0 --kall-steps 0 --no-cpu-baseline --timing-steps 100 $m > gpurun_out/fused/b$m.json 2>gpurun_out/fused/b$m.err || { tail -20 gpurun_out/fused/b$m.err; exit 1; }
  python -c "import json,sys;d=json.loads(open('gpurun_out/fused/b$m.json').read().strip().splitlines()[-1]);print('$m', round(d['value']/1e6,2),'M', round(d['ms_per_step']*1e3,1),'us/step', json.dumps(d['kernels']))"
done
