# Round-3 session 2, closing rehearsal of the in-tree build: the whole GPU suite, smoke(), the
# driver's bench command on the final tree.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r7ak; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/driver_cmd.json 2> $OUT/driver_cmd.err || { tail $OUT/driver_cmd.err; exit 1; }
python -c "
import json; j=json.load(open('$OUT/driver_cmd.json'))
print('driver cmd', round(j['value']/1e6,2), 'M', round(j['ms_per_step']*1e3,1), 'us/step; eps/s', round(j['episodes_per_s']/1e6,2), 'M; K=4', round(j['two_ply_k4']['value']/1e6,3), 'K=all', round(j['two_ply_kall']['value']/1e6,3), 'c1', round(j['configs1_4096_lanes']['value']/1e6,1), 'cpu', round(j['cpu_baseline']['value']), 'roof frac', round(j['roofline']['frac'],3), 'traffic', j['roofline']['traffic'])"
timeout -k 10 200 python bench.py --steps 600 --warmup 5 --no-cpu-baseline --two-ply-steps 0 --kall-steps 0 --config1-steps 0 > $OUT/bench600.json 2> $OUT/bench600.err || { tail $OUT/bench600.err; exit 1; }
python -c "import json; j=json.load(open('$OUT/bench600.json')); print('600 steps', round(j['value']/1e6,2), 'M')"
