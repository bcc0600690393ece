#!/bin/bash
# round 5: the in-tree build (tile prefetch + MFMA chain at priority 1 + half
# tickets) vs whole-group tickets (nohalf) and priority through the epilogue
# (epi): 20-step windows with the event-timed launch beside, 600 steps, and
# the prof build's workgroup spans of a 20-step launch for in-tree / nohalf
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5d; mkdir -p $O
B=mlp-ppo-2ply-multi_amd/bgx
LIBS="libbgx libbgx_nohalf libbgx_epi"
A20="--steps 20 --warmup 5 --kall-steps 0 --config1-steps 0 --two-ply-steps 0 --no-cpu-baseline --timing-steps 20"
A600="--steps 600 --warmup 300 --kall-steps 0 --config1-steps 0 --two-ply-steps 0 --no-cpu-baseline --timing-steps 0"
echo "[1] 20 steps"
for rep in 1 2 3 4 5; do for lib in $LIBS; do
  BGX_LIB=$B/$lib.so timeout -k 10 180 python bench.py $A20 > $O/b20_${lib}_$rep.json 2> $O/b20.err || { tail -5 $O/b20.err; exit 1; }
done; done
python tools/ab_vals.py $O/b20_*.json
for lib in $LIBS; do python - $lib $O <<'PY'
import glob, json, sys
lib, o = sys.argv[1], sys.argv[2]
ms = [json.loads(open(f).read().strip().splitlines()[-1])["kernels"]["fused_step"]["avg_launch_ms"] for f in sorted(glob.glob(f"{o}/b20_{lib}_[0-9].json"))]
print(f"{lib}: event-timed 20-step launch ms {[round(x, 4) for x in ms]} mean {sum(ms) / len(ms):.4f}")
PY
done
echo "[2] 600 steps"
for rep in 1 2; do for lib in $LIBS; do
  BGX_LIB=$B/$lib.so timeout -k 10 180 python bench.py $A600 > $O/b600_${lib}_$rep.json 2> $O/b600.err || { tail -5 $O/b600.err; exit 1; }
done; done
python tools/ab_vals.py $O/b600_*.json
echo "[3] workgroup spans, prof build"
for lib in libbgx libbgx_nohalf; do
  BGX_LIB=$B/$lib.so BGX_FUSED_PROF=1 BGX_FUSED_PROF_DUMP=$O/wg20_$lib.csv timeout -k 10 180 python bench.py ${A20/--timing-steps 20/--timing-steps 0} > $O/p20_$lib.json 2> $O/p20_$lib.err || { tail -5 $O/p20_$lib.err; exit 1; }
  grep "last launch" $O/p20_$lib.err
  python tools/wg_spans.py $O/wg20_$lib.csv | head -2
done
