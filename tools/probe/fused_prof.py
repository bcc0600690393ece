"""Phase clocks of the fused 1-ply kernel (BGX_FUSED_PROF=1 build path):
N launches of K steps at 8,192 balanced lanes after a 300-step desync, then
the engine is closed and the library prints its per-workgroup-step report
(item wave-us, tier-1 job costs, the last launch's workgroup spans) on
stderr. Development tool.   BGX_FUSED_PROF=1 python tools/probe/fused_prof.py N K"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "mlp-ppo-2ply-multi_amd"))
from bgx import Engine  # noqa: E402

d = np.load(os.path.join(REPO, "tests", "golden", "weights_seed0.npz"))
w = {k: d[k] for k in ("W1", "b1", "w2", "b2")}
n, k = int(sys.argv[1]), int(sys.argv[2])
torch.cuda.set_device(0)
e = Engine(lanes=8192, seed=0, balance=True)
e.set_weights(w, 1.5, 1)
e.step(300)
e.harvest_fetch(e.harvest_enqueue(), wrap=False)
for _ in range(n):
    e.step(k)
    e.harvest_fetch(e.harvest_enqueue(), wrap=False)
e.sync()
e.close()
