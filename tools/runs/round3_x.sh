# Round-3 session 2, GPU call 1: the restored HEAD tree (pipelined fused step with
# carried tier-1 expansion): full GPU suite, smoke(), then the round profile.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r6x; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
bash tools/profile_round.sh r6prof
