# Round-3 session 2, GPU call 6: issue priority of the fused kernel's item kinds
# (s_setprio; libbgx_p1 = choice items raised, libbgx_p2 = + MLP tiles) vs the
# committed tree (libbgx), then a 2-rank rehearsal of the driver's multi-GPU
# command shape (gloo, both ranks on the one GPU, host gather).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r7ad; rm -rf $OUT; mkdir -p $OUT
for lib in libbgx_p1 libbgx_p2 libbgx libbgx_p1 libbgx_p2 libbgx; do
  BGX_LIB=$PWD/mlp-ppo-2ply-multi_amd/bgx/$lib.so timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --two-ply-steps 0 --kall-steps 0 --config1-steps 0 > $OUT/${lib}_20.json 2> $OUT/${lib}_20.err || { tail $OUT/${lib}_20.err; exit 1; }
  BGX_LIB=$PWD/mlp-ppo-2ply-multi_amd/bgx/$lib.so timeout -k 10 200 python bench.py --steps 600 --warmup 5 --no-cpu-baseline --two-ply-steps 0 --kall-steps 0 --config1-steps 0 > $OUT/${lib}_600.json 2> $OUT/${lib}_600.err || { tail $OUT/${lib}_600.err; exit 1; }
  python -c "
import json
a=json.load(open('$OUT/${lib}_20.json')); b=json.load(open('$OUT/${lib}_600.json'))
print('$lib', '20:', round(a['value']/1e6,2), 'M  600:', round(b['value']/1e6,2), 'launch600 ms', round(b['kernels']['fused_step']['avg_launch_ms'],3))"
done
BGX_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 20 --warmup 5 --two-ply-steps 5 --kall-steps 2 > $OUT/rehearsal2.json 2> $OUT/rehearsal2.err || { tail -20 $OUT/rehearsal2.err; exit 1; }
python -c "
import json; j=json.load(open('$OUT/rehearsal2.json'))
print('2 ranks on one GPU (gloo):', round(j['value']/1e6,2), 'M total; per rank', j['env_steps_per_rank'], 'gathered eps/recs', j.get('gathered_episodes'), j.get('gathered_records'), 'K=4', round(j['two_ply_k4']['value']/1e6,3))"
