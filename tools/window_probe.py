"""What a 20-step timed window holds (the driver's bench.py --steps 20): ten
windows of [sync, step(20), harvest_enqueue, harvest_fetch] on 8,192
balanced lanes after 300 desync steps, host-timed, spaced by 20 ms so a
rocprofv3 --kernel-trace of this script shows each window's kernels apart
(tools/window_check.py splits them). Development tool."""
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mlp-ppo-2ply-multi_amd"))
from bgx import Engine  # noqa: E402

d = np.load(os.path.join(REPO, "tests", "golden", "weights_seed0.npz"))
w = {k: d[k] for k in ("W1", "b1", "w2", "b2")}
steps = int(os.environ.get("STEPS", "20"))
sleep_s = float(os.environ.get("SLEEP_MS", "20")) / 1e3   # idle gap before each window
torch.cuda.set_device(0)
e = Engine(lanes=8192, seed=0, balance=True)
e.set_weights(w, 1.5, 1)
for _ in range(3):
    e.step(100)
    e.harvest()
e.sync()
out = []
for i in range(10):
    if sleep_s > 0:
        time.sleep(sleep_s)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e.step(steps)
    t = e.harvest_enqueue()
    h = e.harvest_fetch(t)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    out.append({"us": (t1 - t0) * 1e6, "episodes": h.n_episodes, "records": h.n_records})
print(json.dumps({"steps": steps, "sleep_ms": sleep_s * 1e3, "windows": out,
                  "median_us": float(np.median([o["us"] for o in out]))}))
e.close()
