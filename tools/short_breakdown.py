#!/usr/bin/env python3
"""Where the driver-like short run's time goes (tools only): host clock around
step(20) (launch call, device completion), harvest(), and the barrier, over
fresh engines at 8,192 lanes after 5 warm-up steps, as bench.py runs it."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "mlp-ppo-2ply-multi_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import torch  # noqa: E402
from bgx import Engine  # noqa: E402
from bench import load_weights  # noqa: E402

lanes = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
w = load_weights()
rows = []
for rep in range(6):
    eng = Engine(lanes=lanes, seed=rep, ply=1, k_top=4)
    eng.set_weights(w, temperature=1.5, version=1)
    eng.step(5)
    eng.harvest()
    eng.sync()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.step(steps)
    t1 = time.perf_counter()
    eng.sync()
    t2 = time.perf_counter()
    h = eng.harvest()
    t3 = time.perf_counter()
    torch.cuda.synchronize()
    t4 = time.perf_counter()
    rows.append({"launch_us": (t1 - t0) * 1e6, "device_us": (t2 - t1) * 1e6, "harvest_us": (t3 - t2) * 1e6,
                 "barrier_us": (t4 - t3) * 1e6, "total_us": (t4 - t0) * 1e6, "episodes": h.n_episodes})
    eng.close()
print(json.dumps(rows, indent=1))
