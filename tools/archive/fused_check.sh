# fused kernel: correctness (fused == phased, tiers, ragged, greedy, replay) then the phase profile and bench
set -o pipefail
export TMPDIR=/tmp; OUT=gpurun_out/${1:-fcheck}; mkdir -p $OUT
timeout -k 10 60 python -u -c "
import sys; sys.path[:0]=['mlp-ppo-2ply-multi_amd','tests']
import numpy as np
from conftest import golden
from bgx import Engine
w={k: golden('weights_seed0.npz')[k] for k in ('W1','b1','w2','b2')}
e=Engine(lanes=37, seed=3); e.set_weights(w, 1.5, 1); e.step(5); e.sync(); print('fused smoke ok', e.stats()['env_steps'])
" 2>&1 | tee $OUT/smoke.log || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_replay.py -k "fused or replay or shard" -v --timeout 120 --timeout-method thread 2>&1 | tee $OUT/tests.log || exit 1
bash tools/fprof.sh ${1:-fcheck}
