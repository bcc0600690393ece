# round 6: does the driver's 20-step window depend on how long the GPU ran
# before it (clock / cache warm-up)? --desync-steps 300 (default) vs 1200,
# interleaved, and the window after the CPU baseline leg as the driver runs it
set -o pipefail
O=gpurun_out/r6ds; mkdir -p $O
A="--two-ply-steps 0 --kall-steps 0 --config1-steps 0 --config2-steps 0 --timing-steps 0 --steps 20 --warmup 5"
for rep in 1 2 3; do for ds in 300 1200; do
  timeout -k 10 200 python bench.py $A --no-cpu-baseline --desync-steps $ds > $O/d${ds}_$rep.json 2> $O/d${ds}_$rep.err || { tail -20 $O/d${ds}_$rep.err; exit 1; }
  echo "desync $ds rep$rep: $(grep -o '[0-9.]* M env' $O/d${ds}_$rep.err)"
done; done
timeout -k 10 300 python bench.py $A > $O/cpu_first.json 2> $O/cpu_first.err || { tail -20 $O/cpu_first.err; exit 1; }
echo "with the CPU baseline first: $(grep -o '[0-9.]* M env' $O/cpu_first.err)"
