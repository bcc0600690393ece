# N > 1 plumbing with the current tree: 2 gloo ranks sharing the one GPU, the driver's command shape and a gathering run
set -o pipefail
export TMPDIR=/tmp; OUT=gpurun_out/r3q; mkdir -p $OUT
BGX_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 20 --warmup 5 > $OUT/rank2_driver.json 2> $OUT/rank2_driver.err || { tail $OUT/rank2_driver.err; exit 1; }
tail -c 400 $OUT/rank2_driver.json; echo
BGX_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --lanes 4096 --steps 600 --warmup 300 --two-ply-steps 0 --kall-steps 0 --config1-steps 0 --no-cpu-baseline --timing-steps 100 > $OUT/rank2_gather.json 2> $OUT/rank2_gather.err || { tail $OUT/rank2_gather.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/rank2_gather.json'));print({k:d.get(k) for k in ('value','n_gpus','ms_per_step','gathered_episodes','gathered_records')})"
