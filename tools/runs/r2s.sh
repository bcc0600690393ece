# action choice by quarter-waves (four lanes per wave, one round for 32 lanes on 12 waves): suite, phase profile, A/B
set -o pipefail
export TMPDIR=/tmp; OUT=gpurun_out/r2s; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
BGX_FUSED_PROF=1 timeout -k 10 200 python bench.py --steps 300 --warmup 100 --two-ply-steps 0 --kall-steps 0 --config1-steps 0 --no-cpu-baseline --timing-steps 100 > $OUT/prof.json 2> $OUT/prof.err || exit 1
grep "fused prof" $OUT/prof.err
AB_ARGS="--steps 600 --warmup 300 --kall-steps 0 --two-ply-steps 60 --no-cpu-baseline --timing-steps 300 --config1-steps 300" bash tools/ab_multi.sh r2s/ab tools/diag/libbgx_prev.so
for f in $OUT/ab/*.json; do python -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$f', round(d['value']/1e6,2), round(d['configs1_4096_lanes']['value']/1e6,2))"; done
