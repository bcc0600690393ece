# full GPU suite, then the fused phase profile, then the bench legs (no CPU baseline)
set -o pipefail
export TMPDIR=/tmp; OUT=gpurun_out/${1:-full}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread 2>&1 | tee $OUT/tests.log | grep -E "PASSED|FAILED|ERROR|passed|failed" || exit 1
bash tools/fprof.sh ${1:-full} || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 300 --warmup 100 > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
python -c "
import json;d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
print('1ply', round(d['value']/1e6,2), 'M', round(d['ms_per_step']*1e3,1), 'us | k4', round(d['two_ply_k4']['value']/1e6,3), 'M', round(d['two_ply_k4']['ms_per_step'],3), 'ms | kall', round(d['two_ply_kall']['value']/1e6,3), 'M | c1', round(d['configs1_4096_lanes']['value']/1e6,2))
print('k4 kernels', {k: round(v['avg_launch_ms'],3) for k,v in d['two_ply_k4']['kernels'].items()})"
