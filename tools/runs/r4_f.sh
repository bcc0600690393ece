#!/bin/bash
# round 4: spin-then-block harvest wait A/B on the driver's window (3 reps, interleaved)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4f; mkdir -p $O
B="--no-cpu-baseline --two-ply-steps 0 --kall-steps 0 --config1-steps 0 --timing-steps 20"
for rep in 1 2 3; do for sp in 1 0; do
  BGX_SPIN_WAIT=$sp timeout -k 10 200 python bench.py --steps 20 --warmup 5 $B > $O/b20_s${sp}_$rep.json 2>> $O/b.err || { tail -20 $O/b.err; exit 1; }
  python tools/ab_line.py b20_s${sp}_$rep $O/b20_s${sp}_$rep.json
done; done
