"""Per-launch fixed cost of the fused 1-ply kernel: host wall time of one
k-step launch (synchronised) for k in 1..300 at 8,192 lanes, fit t = F + k s.
With BGX_FUSED_PROF=1 each engine also prints its last launch's per-workgroup
durations at close. BALANCE=1: balanced launches (bgx_config.balance).
Development tool."""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mlp-ppo-2ply-multi_amd"))
from bgx import Engine  # noqa: E402

d = np.load(os.path.join(REPO, "tests", "golden", "weights_seed0.npz"))
w = {k: d[k] for k in ("W1", "b1", "w2", "b2")}
lanes = int(os.environ.get("LANES", "8192"))
balance = os.environ.get("BALANCE", "0") == "1"
res = []
for k in (1, 2, 5, 20, 60, 300):
    e = Engine(lanes=lanes, seed=3, ply=1, balance=balance)
    e.set_weights(w, temperature=1.5, version=1)
    e.step(300)
    e.harvest()
    e.sync()
    ts = []
    for rep in range(5):
        t0 = time.perf_counter()
        e.step(k)
        e.sync()
        ts.append(time.perf_counter() - t0)
        e.harvest()
        e.sync()
    t = float(np.median(ts)) * 1e6
    res.append((k, t))
    print(f"k={k:4d} launch {t:9.1f} us  {t / k:7.2f} us/step", flush=True)
    sys.stdout.flush()
    e.close()
ks = np.array([r[0] for r in res], float)
tt = np.array([r[1] for r in res], float)
s, F = np.polyfit(ks, tt, 1)
print(f"fit: fixed {F:.1f} us per launch + {s:.2f} us per step", flush=True)
