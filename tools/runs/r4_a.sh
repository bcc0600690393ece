#!/bin/bash
# round 4: new scale / flag tests, the full GPU suite, bench lines, a prof run
set -o pipefail
O=gpurun_out/r4a; mkdir -p $O
B="--no-cpu-baseline --two-ply-steps 0 --kall-steps 0 --config1-steps 0"
echo "[1] new tests"
timeout -k 10 420 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_engine.py -x -v --timeout 200 --timeout-method thread \
  -k "scale or flags or capacity or bench_shape or kall_4096 or same_seed or pipelined" > $O/t1.log 2>&1 || { tail -40 $O/t1.log; exit 1; }
tail -3 $O/t1.log
echo "[2] full gpu suite"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/t2.log 2>&1 || { tail -40 $O/t2.log; exit 1; }
tail -3 $O/t2.log
echo "[3] bench"
timeout -k 10 200 python bench.py --steps 600 --warmup 100 $B > $O/b600.json 2> $O/b600.err || { tail $O/b600.err; exit 1; }
for i in 1 2; do timeout -k 10 200 python bench.py --steps 20 --warmup 5 $B > $O/b20_$i.json 2>> $O/b20.err || exit 1; done
python - <<'PY'
import json
for f in ("b600", "b20_1", "b20_2"):
    d = json.loads(open(f"gpurun_out/r4a/{f}.json").read().strip().splitlines()[-1])
    print(f, round(d["value"] / 1e6, 1), "M", round(d["ms_per_step"], 4), "ms/step")
PY
echo "[4] prof"
BGX_FUSED_PROF=1 timeout -k 10 200 python bench.py --steps 300 --warmup 0 --timing-steps 1 $B > $O/prof.json 2> $O/prof.err || { tail $O/prof.err; exit 1; }
grep "fused prof" $O/prof.err | tail -12
