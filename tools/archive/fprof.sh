set -o pipefail
export TMPDIR=/tmp; OUT=gpurun_out/${1:-fprof}; mkdir -p $OUT
ARGS="--steps 600 --warmup 300 --two-ply-steps 0 --kall-steps 0 --config1-steps 0 --no-cpu-baseline --timing-steps 300"
BGX_FUSED_PROF=1 timeout -k 10 120 python bench.py $ARGS > $OUT/p.json 2> $OUT/p.err || { tail $OUT/p.err; exit 1; }
grep "fused prof" $OUT/p.err
timeout -k 10 120 python bench.py $ARGS > $OUT/b.json 2> $OUT/b.err || exit 1
python -c "import json;d=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]);print(round(d['value']/1e6,2),'M', round(d['ms_per_step']*1e3,1),'us/step')"
