# A/B several builds of libbgx.so on one box, interleaved (2 reps each).
# $1 = output tag; the rest = library paths (the in-tree build is always first).
set -o pipefail
export TMPDIR=/tmp; OUT=gpurun_out/${1:-ab_multi}; shift; mkdir -p $OUT
ARGS=${AB_ARGS:-"--steps 600 --warmup 300 --kall-steps 0 --config1-steps 0 --two-ply-steps 100 --no-cpu-baseline --timing-steps 300"}
for rep in 1 2; do
  for lib in mlp-ppo-2ply-multi_amd/bgx/libbgx.so "$@"; do
    tag=$(basename $lib .so)_$rep
    BGX_LIB=$lib timeout -k 10 180 python bench.py $ARGS > $OUT/$tag.json 2> $OUT/$tag.err || { tail -5 $OUT/$tag.err; exit 1; }
    python tools/ab_line.py $tag $OUT/$tag.json
  done
done
