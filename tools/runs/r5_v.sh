#!/bin/bash
# round 5: the workgroup row chunks' size cap (8 x BGX_FLAT_CHUNK rows: 2,048 /
# 4,096 (default) / 8,192)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5v; mkdir -p $O
K4="--ply 2 --steps 100 --warmup 20 --kall-steps 0 --config1-steps 0 --two-ply-steps 0 --no-cpu-baseline --timing-steps 50"
KA="--ply 2 --k-top 0 --steps 20 --warmup 5 --kall-steps 0 --config1-steps 0 --two-ply-steps 0 --no-cpu-baseline --timing-steps 10"
for rep in 1 2; do
  for c in 256 512 1024; do
    BGX_FLAT_CHUNK=$c timeout -k 10 180 python bench.py $K4 > $O/k4_c${c}_$rep.json 2> $O/e.err || { tail -5 $O/e.err; exit 1; }
    BGX_FLAT_CHUNK=$c timeout -k 10 180 python bench.py $KA > $O/ka_c${c}_$rep.json 2> $O/e.err || { tail -5 $O/e.err; exit 1; }
  done
done
python tools/ab_vals.py $O/k4_*.json $O/ka_*.json
for f in $O/k4_*.json $O/ka_*.json; do python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1].split('/')[-1], 'gap %.4f' % d['gap_rows_frac'])" $f; done
