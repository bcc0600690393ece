# K=4 step timeline (kernel trace) for the in-tree build and another library: $1 = out tag, $2 = other lib
set -o pipefail
export TMPDIR=/tmp; OUT=gpurun_out/$1; mkdir -p $OUT
for lib in mlp-ppo-2ply-multi_amd/bgx/libbgx.so $2; do
  tag=$(basename $lib .so)
  BGX_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/kt_$tag -o run --output-format csv -- python bench.py --ply 2 --k-top 4 --steps 120 --warmup 300 --timing-steps 1 --two-ply-steps 0 --kall-steps 0 --config1-steps 0 --no-cpu-baseline > $OUT/kt_$tag.json 2> $OUT/kt_$tag.err || { tail $OUT/kt_$tag.err; exit 1; }
  f=$(find $OUT/kt_$tag -name "*kernel_trace.csv" | head -1); echo "== $tag"; python tools/step_timeline.py $f movegen_few_kernel 100 > $OUT/timeline_$tag.txt; head -12 $OUT/timeline_$tag.txt
done
