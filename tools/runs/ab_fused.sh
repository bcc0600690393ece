# A/B of the fused 1-ply kernel: the default build (libbgx.so) against an
# alternative build bgx/libbgx_ab0.so (make EXTRA=-D... BUILD=build_ab0
# OUT=../bgx/libbgx_ab0.so): fused / replay tests on the default, then
# interleaved bench runs (600-step and the driver's 20-step window).
#   bash tools/runs/ab_fused.sh <out dir under gpurun_out> [reps]
set -o pipefail
O=gpurun_out/${1:-ab}; mkdir -p $O; R=${2:-3}
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_engine.py tests/test_gpu_replay.py -k "fused or replay or shard or balanced" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
A="--no-cpu-baseline --two-ply-steps 0 --kall-steps 0 --config1-steps 0 --config2-steps 0 --timing-steps 0"
for rep in $(seq 1 $R); do for lib in new ab0; do
  if [ $lib = ab0 ]; then export BGX_LIB=$PWD/mlp-ppo-2ply-multi_amd/bgx/libbgx_ab0.so; else unset BGX_LIB; fi
  timeout -k 10 200 python bench.py $A --steps 600 --warmup 100 > $O/l_${lib}_$rep.json 2> $O/l_${lib}_$rep.err || { tail -20 $O/l_${lib}_$rep.err; exit 1; }
  timeout -k 10 200 python bench.py $A --steps 20 --warmup 5 > $O/s_${lib}_$rep.json 2> $O/s_${lib}_$rep.err || { tail -20 $O/s_${lib}_$rep.err; exit 1; }
  echo "$lib rep$rep 600: $(grep -o '[0-9.]* M env' $O/l_${lib}_$rep.err)  20: $(grep -o '[0-9.]* M env' $O/s_${lib}_$rep.err)"
done; done
unset BGX_LIB
