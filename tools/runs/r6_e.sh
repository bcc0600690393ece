# round 6: 2-ply tests after the opt-in delta reply MLP (default: full), the
# configs[2] legs, and one default bench line
set -o pipefail
O=gpurun_out/r6e; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_reply.py tests/test_gpu_scale.py tests/test_gpu_replay.py tests/test_gpu_engine.py -k "2ply or two_ply or kall or k4 or reply or same_seed or golden or delta" > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -3 $O/t.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
grep "\[bench\]" $O/bench.err
