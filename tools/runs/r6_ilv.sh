# round 6: lane-order fused step queue (BGX_FUSED_ILV=1, libbgx.so) vs phase order
# (libbgx_ilv0.so): fused == phased / replay tests on the new default, then
# interleaved 1-ply bench A/B (600-step and the driver's 20-step window)
set -o pipefail
O=gpurun_out/r6ilv; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_engine.py tests/test_gpu_replay.py -k "fused or replay or shard or balanced" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
A="--no-cpu-baseline --two-ply-steps 0 --kall-steps 0 --config1-steps 0 --config2-steps 0 --timing-steps 0"
for rep in 1 2 3; do for lib in ilv1 ilv0; do
  if [ $lib = ilv0 ]; then export BGX_LIB=$PWD/mlp-ppo-2ply-multi_amd/bgx/libbgx_ilv0.so; else unset BGX_LIB; fi
  timeout -k 10 200 python bench.py $A --steps 600 --warmup 100 > $O/l_${lib}_$rep.json 2> $O/l_${lib}_$rep.err || { tail -20 $O/l_${lib}_$rep.err; exit 1; }
  timeout -k 10 200 python bench.py $A --steps 20 --warmup 5 > $O/s_${lib}_$rep.json 2> $O/s_${lib}_$rep.err || { tail -20 $O/s_${lib}_$rep.err; exit 1; }
  echo "$lib rep$rep 600: $(grep -o '[0-9.]* M env' $O/l_${lib}_$rep.err)  20: $(grep -o '[0-9.]* M env' $O/s_${lib}_$rep.err)"
done; done
unset BGX_LIB
