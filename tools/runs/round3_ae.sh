# Round-3 session 2, GPU call 7: SDMA copies split over the available engines
# (BGX_DMA_ENGINES = 1, 2, 4, all) with a spin-then-block wait; the host-gather
# GPU test; the 2-rank rehearsal of the multi-GPU command (gloo, one GPU) with
# the split copies and the spinning collect vs one engine.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r7ae; rm -rf $OUT; mkdir -p $OUT
for n in 1 2 4 all; do
  if [ $n = all ]; then unset BGX_DMA_ENGINES; else export BGX_DMA_ENGINES=$n; fi
  timeout -k 10 120 python tools/dma_split_probe.py > $OUT/dma_$n.json 2> $OUT/dma_$n.err || { tail $OUT/dma_$n.err; exit 1; }
  cat $OUT/dma_$n.json
done
unset BGX_DMA_ENGINES
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for n in all 1 all 1; do
  if [ $n = all ]; then unset BGX_DMA_ENGINES; else export BGX_DMA_ENGINES=$n; fi
  BGX_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 20 --warmup 5 --two-ply-steps 0 --kall-steps 0 > $OUT/rehearsal_$n.json 2> $OUT/rehearsal_$n.err || { tail -20 $OUT/rehearsal_$n.err; exit 1; }
  python -c "
import json
for ln in open('$OUT/rehearsal_$n.json'):
    if ln.startswith('{'):
        j=json.loads(ln); print('engines $n: 2 ranks on one GPU', round(j['value']/1e6,2), 'M total, ms/step', round(j['ms_per_step']*1e3,1), 'us; gathered', j.get('gathered_episodes'))"
done
