# development: fused kernel with 8 vs 16 waves per workgroup (parity tests + phase profile + bench each)
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out/fw
for nw in ${@:-8 16}; do
  BGX_FUSED_WAVES=$nw timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread -k "fused or transitions_match" > gpurun_out/fw/t$nw.log 2>&1 || { tail -30 gpurun_out/fw/t$nw.log; exit 1; }
  echo "waves=$nw $(tail -1 gpurun_out/fw/t$nw.log)"
  BGX_FUSED_WAVES=$nw BGX_FUSED_PROF=1 timeout -k 10 200 python bench.py --steps 300 --warmup 100 --two-ply-steps 0 --kall-steps 0 --no-cpu-baseline --timing-steps 100 > gpurun_out/fw/p$nw.json 2> gpurun_out/fw/p$nw.err || exit 1
  grep "fused prof" gpurun_out/fw/p$nw.err
  BGX_FUSED_WAVES=$nw timeout -k 10 200 python bench.py --steps 400 --warmup 100 --two-ply-steps 0 --kall-steps 0 --no-cpu-baseline --timing-steps 100 > gpurun_out/fw/b$nw.json 2> gpurun_out/fw/b$nw.err || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/fw/b$nw.json').read().strip().splitlines()[-1]);print('waves=$nw', round(d['value']/1e6,2),'M', round(d['ms_per_step']*1e3,1),'us/step')"
done
