"""bench.py's host gap between the warmup and t0 (eng.sync, eng.stats,
barrier): how long the GPU idles before the timed window. Development tool."""
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "mlp-ppo-2ply-multi_amd"))
from bench import load_weights  # noqa: E402
from bgx import Engine  # noqa: E402

torch.cuda.set_device(0)
e = Engine(lanes=8192, seed=0, balance=True)
e.set_weights(load_weights(), 1.5, 1)
e.step(300)
e.harvest()
out = []
for _ in range(5):
    e.step(5)
    t = e.harvest_enqueue()
    e.harvest_fetch(t, wrap=False)
    t0 = time.perf_counter()
    e.sync()
    t1 = time.perf_counter()
    e.stats()
    t2 = time.perf_counter()
    torch.cuda.synchronize()
    torch.cuda.synchronize()
    t3 = time.perf_counter()
    out.append({"sync_us": (t1 - t0) * 1e6, "stats_us": (t2 - t1) * 1e6, "barrier_us": (t3 - t2) * 1e6})
print(json.dumps(out))
e.close()
