#!/bin/bash
# round 4: 1-ply regression bisect on one box -- the round-3 tree (ae77218), the
# first round-4 commit (8b71728) and HEAD, interleaved, 20-step driver windows
# and 600-step runs
set -o pipefail
export TMPDIR=/tmp
O=$PWD/gpurun_out/r4c; mkdir -p $O
A="--no-cpu-baseline --two-ply-steps 0 --kall-steps 0 --config1-steps 0 --timing-steps 20"
for rep in 1 2; do
  for t in . tools/diag/tree_ae77218 tools/diag/tree_8b71728; do
    tag=$(basename $t)_$rep
    (cd $t && timeout -k 10 200 python bench.py --steps 20 --warmup 5 $A > $O/b20_$tag.json 2> $O/b20_$tag.err) || { tail -5 $O/b20_$tag.err; exit 1; }
    python tools/ab_line.py b20_$tag $O/b20_$tag.json
    (cd $t && timeout -k 10 200 python bench.py --steps 600 --warmup 300 $A > $O/b600_$tag.json 2> $O/b600_$tag.err) || { tail -5 $O/b600_$tag.err; exit 1; }
    python tools/ab_line.py b600_$tag $O/b600_$tag.json
  done
done
