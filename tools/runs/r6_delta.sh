set -o pipefail
O=gpurun_out/r6d; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_reply.py tests/test_gpu_scale.py tests/test_gpu_replay.py tests/test_gpu_engine.py tests/test_gpu_parity.py -k "2ply or two_ply or kall or k4 or reply or same_seed or golden" > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -3 $O/t.log
A="--no-cpu-baseline --config1-steps 0 --config2-steps 0 --timing-steps 20 --steps 20 --warmup 5 --two-ply-steps 100 --kall-steps 20"
for rep in 1 2; do for d in 1 0; do
  BGX_REPLY_DELTA=$d timeout -k 10 300 python bench.py $A > $O/b_${d}_$rep.json 2> $O/b_${d}_$rep.err || { tail -20 $O/b_${d}_$rep.err; exit 1; }
  grep "\[bench\] 2ply" $O/b_${d}_$rep.err | sed "s/^/delta=$d /"
done; done
