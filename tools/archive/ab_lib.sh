# A/B two builds of libbgx.so on the same box, interleaved: $2 = the other library (A = in-tree)
set -o pipefail
export TMPDIR=/tmp; OUT=gpurun_out/${1:-ab_lib}; mkdir -p $OUT; B=${2:-tools/diag/libbgx_prev.so}
ARGS="--steps 600 --warmup 300 --kall-steps 0 --config1-steps 0 --two-ply-steps 100 --no-cpu-baseline --timing-steps 300"
for rep in 1 2; do
  for lib in mlp-ppo-2ply-multi_amd/bgx/libbgx.so $B; do
    tag=$(basename $lib .so)_$rep
    BGX_LIB=$lib timeout -k 10 180 python bench.py $ARGS > $OUT/$tag.json 2> $OUT/$tag.err || { tail -5 $OUT/$tag.err; exit 1; }
    python -c "import json;d=json.loads(open('$OUT/$tag.json').read().strip().splitlines()[-1]);k=d['two_ply_k4'];print('$tag', '1ply', round(d['value']/1e6,2),'M', round(d['ms_per_step']*1e3,1),'us | k4', round(k['ms_per_step'],3),'ms', {n: round(v['avg_launch_ms'],3) for n,v in k['kernels'].items()})"
  done
done
