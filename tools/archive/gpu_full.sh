# Full GPU test suite, then the fused phase profile and the fused vs phased bench legs.
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out/fused
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/fused/full.log 2>&1 || { tail -40 gpurun_out/fused/full.log; exit 1; }
tail -2 gpurun_out/fused/full.log
BGX_FUSED_PROF=1 timeout -k 10 200 python bench.py --steps 300 --warmup 100 --two-ply-steps 0 --kall-steps 0 --no-cpu-baseline --timing-steps 100 > gpurun_out/fused/prof.json 2> gpurun_out/fused/prof.err || exit 1
grep "fused prof" gpurun_out/fused/prof.err
timeout -k 10 300 python bench.py --steps 400 --warmup 100 --two-ply-steps 60 --kall-steps 0 --no-cpu-baseline --timing-steps 100 > gpurun_out/fused/b.json 2>gpurun_out/fused/b.err || { tail -20 gpurun_out/fused/b.err; exit 1; }
python -c "import json,sys;d=json.loads(open('gpurun_out/fused/b.json').read().strip().splitlines()[-1]);print('1ply', round(d['value']/1e6,2),'M', round(d['ms_per_step']*1e3,1),'us/step | 2ply', round(d['two_ply_k4']['value']/1e6,3), 'M', d['two_ply_k4']['kernels'])"
