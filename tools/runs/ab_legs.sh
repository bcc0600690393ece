#!/bin/bash
# A/B of bench.py legs over builds / environment settings, interleaved, on one
# GPU box (the round-5 experiments of tools/runs/README.md are instances).
#   bash tools/runs/ab_legs.sh OUT REPS "LEGS" VARIANT...
# LEGS: any of k4 (2-ply K=4, 100 steps), kall (2-ply K=all, 20 steps),
#       p600 (1-ply, 600 steps), p20 (1-ply, the driver's 20 steps),
#       c1 (1-ply, 4,096 lanes, 600 steps)
# VARIANT: name[:ENV=v,ENV=v][:lib]  (lib: a build under mlp-ppo-2ply-multi_amd/bgx,
#       e.g. libbgx_nowg for `make ... OUT=../bgx/libbgx_nowg.so`; default the in-tree libbgx)
# Output: gpurun_out/OUT/<leg>_<name>_<rep>.json, then tools/ab_vals.py's table.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1; REPS=$2; LEGS=$3; shift 3
mkdir -p $O
B=$PWD/mlp-ppo-2ply-multi_amd/bgx
COMMON="--config1-steps 0 --two-ply-steps 0 --kall-steps 0 --no-cpu-baseline"
args_of() {
  case $1 in
    k4) echo "--ply 2 --steps 100 --warmup 20 --timing-steps 50 $COMMON" ;;
    kall) echo "--ply 2 --k-top 0 --steps 20 --warmup 5 --timing-steps 10 $COMMON" ;;
    p600) echo "--steps 600 --warmup 100 --timing-steps 300 $COMMON" ;;
    p20) echo "--steps 20 --warmup 5 --timing-steps 20 $COMMON" ;;
    c1) echo "--lanes 4096 --steps 600 --warmup 100 --timing-steps 300 $COMMON" ;;
  esac
}
for rep in $(seq 1 $REPS); do
  for v in "$@"; do
    IFS=: read -r name envs lib <<< "$v"
    for leg in $LEGS; do
      env_args=(); [ -n "$envs" ] && IFS=, read -r -a env_args <<< "$envs"
      env "${env_args[@]}" BGX_LIB=$B/${lib:-libbgx}.so timeout -k 10 300 python bench.py $(args_of $leg) \
        > $O/${leg}_${name}_$rep.json 2> $O/e.err || { tail -5 $O/e.err; exit 1; }
    done
  done
done
python tools/ab_vals.py $O/*.json
