set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out/sweep
for L in 4096 16384 65536; do
  timeout -k 10 200 python bench.py --lanes $L --steps 200 --warmup 100 --two-ply-steps 0 --kall-steps 0 --no-cpu-baseline --timing-steps 50 > gpurun_out/sweep/l$L.json 2>gpurun_out/sweep/l$L.err || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/sweep/l$L.json').read().strip().splitlines()[-1]);print($L, round(d['value']/1e6,1),'M', round(d['ms_per_step']*1e3,1),'us', d['kernels']['movegen']['avg_launch_ms'], d['kernels']['mlp']['avg_launch_ms'])"
done
timeout -k 10 200 python tools/mg_latency.py 2>&1 | grep -v amdgpu.ids
