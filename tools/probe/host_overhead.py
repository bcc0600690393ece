"""Probe (tools only): where the driver's 20-step window spends its time
outside the kernels. Host clock around bench.py's window (step(20),
harvest_enqueue, count-only harvest_fetch, synchronize) next to torch events
on the step stream, plus the bare round trips (an event sync on an idle GPU,
an empty step(0) call)."""
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "mlp-ppo-2ply-multi_amd"))
from bgx import Engine  # noqa: E402

d = np.load(os.path.join(REPO, "tests", "golden", "weights_seed0.npz"))
w = {k: d[k] for k in ("W1", "b1", "w2", "b2")}
steps = int(os.environ.get("STEPS", "20"))
torch.cuda.set_device(0)
e = Engine(lanes=8192, seed=0, balance=True)
e.set_weights(w, 1.5, 1)
for _ in range(3):
    e.step(100)
    e.harvest()
e.sync()
rows = []
for i in range(12):
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    a.record()
    e.step(steps)
    b.record()
    t1 = time.perf_counter()
    tk = e.harvest_enqueue()
    t2 = time.perf_counter()
    e.harvest_fetch(tk, wrap=False)
    t3 = time.perf_counter()
    torch.cuda.synchronize()
    t4 = time.perf_counter()
    rows.append({"host_us": (t4 - t0) * 1e6, "step_call_us": (t1 - t0) * 1e6, "enqueue_us": (t2 - t1) * 1e6,
                 "fetch_us": (t3 - t2) * 1e6, "final_sync_us": (t4 - t3) * 1e6, "fused_gpu_us": a.elapsed_time(b) * 1e3})
idle = []
for i in range(20):
    torch.cuda.synchronize()
    ev = torch.cuda.Event()
    t0 = time.perf_counter()
    ev.record()
    ev.synchronize()
    idle.append((time.perf_counter() - t0) * 1e6)
calls = []
for i in range(20):
    t0 = time.perf_counter()
    e.step(0)
    calls.append((time.perf_counter() - t0) * 1e6)
med = {k: float(np.median([r[k] for r in rows[2:]])) for k in rows[0]}
print(json.dumps({"steps": steps, "median": med, "idle_event_sync_us": float(np.median(idle)),
                  "step0_call_us": float(np.median(calls))}, indent=1))
e.close()
