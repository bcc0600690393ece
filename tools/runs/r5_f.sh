#!/bin/bash
# round 5: the board-major doubles build (BGX_DBL_BM=1, unguarded) after its
# guarded build passed the reply test: the reply and 2-ply engine tests on it,
# then the 2-ply legs A/B against the in-tree (per-roll doubles) build.
# Record of a run: the build flag has since become the runtime switch
# BGX_REPLY_DBL, so this script no longer builds.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5f; mkdir -p $O
B=$PWD/mlp-ppo-2ply-multi_amd/bgx
echo "[1] reply launch test on the board-major doubles build"
BGX_LIB=$B/libbgx_dbl.so timeout -k 10 150 python -u -m pytest "tests/test_gpu_reply.py::test_reply_moves_vs_oracle[1-0]" -x -q --timeout 120 --timeout-method thread > $O/t1.log 2>&1 || { tail -30 $O/t1.log; exit 1; }
tail -1 $O/t1.log
echo "[2] reply + 2-ply engine tests on it"
BGX_LIB=$B/libbgx_dbl.so timeout -k 10 600 python -u -m pytest tests/test_gpu_reply.py tests/test_gpu_engine.py -k "reply or two_ply or 2ply" tests/test_gpu_replay.py -x -q --timeout 240 --timeout-method thread > $O/t2.log 2>&1 || { tail -30 $O/t2.log; exit 1; }
tail -1 $O/t2.log
echo "[3] 2-ply legs A/B"
K4="--ply 2 --steps 100 --warmup 20 --kall-steps 0 --config1-steps 0 --two-ply-steps 0 --no-cpu-baseline --timing-steps 50"
KA="--ply 2 --k-top 0 --steps 20 --warmup 5 --kall-steps 0 --config1-steps 0 --two-ply-steps 0 --no-cpu-baseline --timing-steps 10"
for rep in 1 2; do for lib in libbgx libbgx_dbl; do
  BGX_LIB=$B/$lib.so timeout -k 10 180 python bench.py $K4 > $O/k4_${lib}_$rep.json 2> $O/k4.err || { tail -5 $O/k4.err; exit 1; }
  BGX_LIB=$B/$lib.so timeout -k 10 180 python bench.py $KA > $O/ka_${lib}_$rep.json 2> $O/ka.err || { tail -5 $O/ka.err; exit 1; }
done; done
python tools/ab_vals.py $O/k4_*.json $O/ka_*.json
for f in $O/k4_*.json $O/ka_*.json; do python tools/ab_line.py $(basename $f .json) $f; done
