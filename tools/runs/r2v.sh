# device TD(0) trainer kernel: trainer tests, then the self-play + training loop with both backends
set -o pipefail
export TMPDIR=/tmp; OUT=gpurun_out/r2v; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_trainer.py tests/test_abi.py -x -v --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -60 $OUT/tests.log; exit 1; }
tail -4 $OUT/tests.log
timeout -k 10 300 python tools/train_loop.py --updates 20 --backend hip > $OUT/loop_hip.json 2> $OUT/loop_hip.err || { tail $OUT/loop_hip.err; exit 1; }
cat $OUT/loop_hip.json
timeout -k 10 300 python tools/train_loop.py --updates 10 --backend torch > $OUT/loop_torch.json 2> $OUT/loop_torch.err || { tail $OUT/loop_torch.err; exit 1; }
cat $OUT/loop_torch.json
