# round 6: the phased engines' root MLP launch on the throughput kernel (nt = 2):
# engine / replay / 2-ply tests, then the 2-ply legs and a kernel trace of K=4
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6g; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_engine.py tests/test_gpu_replay.py tests/test_gpu_scale.py tests/test_gpu_reply.py -k "not bench_shape_1ply" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
A="--no-cpu-baseline --config1-steps 0 --config2-steps 0 --steps 20 --warmup 5"
timeout -k 10 300 python bench.py $A > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
grep "\[bench\]" $O/b.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python bench.py --ply 2 --k-top 4 --steps 60 --warmup 10 --timing-steps 1 --two-ply-steps 0 --kall-steps 0 --config1-steps 0 --config2-steps 0 --no-cpu-baseline > $O/kt.json 2> $O/kt.err || { tail $O/kt.err; exit 1; }
f=$(find $O/kt -name "*kernel_stats.csv" | head -1); cut -d, -f1-4 $f | head -12
