"""Host-side costs around a bench window (tools only): torch.cuda.synchronize()
on an idle GPU, a hipEventQuery-style poll, and the launch-to-start latency of
the fused step kernel (1-step launches, host-timed)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "mlp-ppo-2ply-multi_amd"))


def main():
    torch.cuda.set_device(0)
    torch.cuda.synchronize()
    n = 2000
    t = time.perf_counter()
    for _ in range(n):
        torch.cuda.synchronize()
    print(f"torch.cuda.synchronize() idle: {(time.perf_counter() - t) / n * 1e6:.2f} us")
    ev = torch.cuda.Event()
    ev.record()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        ev.query()
    print(f"event.query() done event: {(time.perf_counter() - t) / n * 1e6:.2f} us")
    from bgx import Engine
    d = np.load(os.path.join(os.path.dirname(__file__), "..", "..", "tests", "golden", "weights_seed0.npz"))
    w = {k: d[k] for k in ("W1", "b1", "w2", "b2")}
    e = Engine(lanes=8192, seed=0, balance=True)
    e.set_weights(w, 1.5, 1)
    e.step(50)
    e.sync()
    for k in (1, 2, 5, 20):
        ts = []
        for _ in range(30):
            torch.cuda.synchronize()
            t = time.perf_counter()
            e.step(k)
            tk = e.harvest_enqueue()
            e.harvest_fetch(tk, wrap=False)
            torch.cuda.synchronize()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t)
        print(f"window of {k} steps (step + harvest + 2 syncs): median {np.median(ts) * 1e6:.1f} us")
    for gap_us in (0, 100, 300, 1000, 3000, 10000):
        ts = []
        for _ in range(30):
            torch.cuda.synchronize()
            t_end = time.perf_counter() + gap_us * 1e-6
            while time.perf_counter() < t_end:
                pass
            t = time.perf_counter()
            e.step(20)
            tk = e.harvest_enqueue()
            e.harvest_fetch(tk, wrap=False)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t)
        print(f"20-step window after an idle gap of {gap_us} us: median {np.median(ts) * 1e6:.1f} us")
    t = time.perf_counter()
    for _ in range(20):
        e.stats()
    print(f"Engine.stats(): {(time.perf_counter() - t) / 20 * 1e6:.1f} us")
    e.close()


if __name__ == "__main__":
    main()
