#!/bin/bash
# round 5: the reply launch's workgroup row chunks sized by a quarter of the
# items in flight (in-tree) vs half of them (libbgx_v1, the committed form),
# (libbgx_v1): reply GPU tests on the in-tree build, then K=4 / K=all legs A/B
# with the gap-row fraction
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5q; mkdir -p $O
B=$PWD/mlp-ppo-2ply-multi_amd/bgx
echo "[1] 2-ply tests"
timeout -k 10 300 python -u -m pytest tests/test_gpu_reply.py -x -q --timeout 240 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
echo "[2] legs"
K4="--ply 2 --steps 100 --warmup 20 --kall-steps 0 --config1-steps 0 --two-ply-steps 0 --no-cpu-baseline --timing-steps 50"
KA="--ply 2 --k-top 0 --steps 20 --warmup 5 --kall-steps 0 --config1-steps 0 --two-ply-steps 0 --no-cpu-baseline --timing-steps 10"
for rep in 1 2; do for lib in libbgx libbgx_v1; do
  BGX_LIB=$B/$lib.so timeout -k 10 180 python bench.py $K4 > $O/k4_${lib}_$rep.json 2> $O/e.err || { tail -5 $O/e.err; exit 1; }
  BGX_LIB=$B/$lib.so timeout -k 10 180 python bench.py $KA > $O/ka_${lib}_$rep.json 2> $O/e.err || { tail -5 $O/e.err; exit 1; }
done; done
python tools/ab_vals.py $O/k4_*.json $O/ka_*.json
for f in $O/k4_*.json $O/ka_*.json; do python tools/ab_line.py $(basename $f .json) $f; python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('  gap_rows_frac %.4f' % d['gap_rows_frac'])" $f; done
