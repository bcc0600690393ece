"""Host latency around the driver's 20-step window (development probe).

Mimics bench.py's order per trial -- a 300-step launch, a 5-step warm-up,
stats(), synchronize, then the timed window [step(20), harvest_enqueue,
harvest_fetch, synchronize] -- and reports the window's host wall time next
to the device time of the same launch (HIP events recorded on the engine's
stream around it, read after the window), so the difference is what the
host adds at both ends (launch submission, completion wake-up). Run it under
different HSA/HIP wait settings (e.g. HSA_ENABLE_INTERRUPT=0: the runtime
polls completion signals instead of sleeping on an interrupt).
  python tools/probe/window_latency.py [trials]"""
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
trials = int(sys.argv[1]) if len(sys.argv) > 1 else 6
torch.cuda.set_device(0)
e = Engine(lanes=8192, seed=0, balance=True)
e.set_weights(w, 1.5, 1)
s = torch.cuda.current_stream()
out = []
for i in range(trials):
    e.step(300)
    e.harvest_fetch(e.harvest_enqueue(), wrap=False)
    e.step(5)
    e.harvest_fetch(e.harvest_enqueue(), wrap=False)
    e.sync()
    e.stats()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(s)
    e.step(20)
    t = e.harvest_enqueue()
    ev1.record(s)
    e.harvest_fetch(t, wrap=False)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    out.append({"host_us": (t1 - t0) * 1e6, "device_us": ev0.elapsed_time(ev1) * 1e3})
e.close()
h = [o["host_us"] for o in out[1:]]
dv = [o["device_us"] for o in out[1:]]
print(json.dumps({"env": {k: os.environ.get(k) for k in ("HSA_ENABLE_INTERRUPT", "HIP_FORCE_QUEUE_PROFILING")},
                  "host_us_median": float(np.median(h)), "device_us_median": float(np.median(dv)),
                  "host_minus_device_us": float(np.median(np.array(h) - np.array(dv))), "trials": out}))
