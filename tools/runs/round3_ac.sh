# Round-3 session 2, GPU call 5: the idle-gap probe (round3_ab.sh), then the
# final tree's GPU suite, smoke() and round profile (tools/profile_round.sh r7prof).
set -o pipefail
export TMPDIR=/tmp
bash tools/runs/round3_ab.sh || exit 1
OUT=gpurun_out/r7x; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
bash tools/profile_round.sh r7prof > $OUT/profile.log 2>&1 || { tail -20 $OUT/profile.log; exit 1; }
python -c "
import json; j=json.load(open('gpurun_out/r7prof/bench.json'))
print('default bench', round(j['value']/1e6,2), 'M; K=4', round(j['two_ply_k4']['value']/1e6,3), 'K=all', round(j['two_ply_kall']['value']/1e6,3), 'c1', round(j['configs1_4096_lanes']['value']/1e6,1))"
