# fixed cost per fused launch: k-step launches, host-timed, then with BGX_FUSED_PROF
set -o pipefail
export TMPDIR=/tmp; OUT=gpurun_out/r4d; mkdir -p $OUT
timeout -k 10 200 python tools/launch_cost.py > $OUT/cost.txt 2> $OUT/cost.err && cat $OUT/cost.txt &&
BGX_FUSED_PROF=1 timeout -k 10 200 python tools/launch_cost.py > $OUT/cost_prof.txt 2> $OUT/cost_prof.err && cat $OUT/cost_prof.txt && grep "last launch" $OUT/cost_prof.err
