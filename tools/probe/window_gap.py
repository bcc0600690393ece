"""What the host does between the warm-up and the timed window costs the
window (tools only): bench.py's 20-step window (8,192 lanes, balanced fused
1-ply) timed as bench.py times it, with Engine.stats() between the warm-up and
the barrier (as now) and without it, alternating, 20 windows each."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "mlp-ppo-2ply-multi_amd"))


def main():
    from bgx import Engine
    torch.cuda.set_device(0)
    d = np.load(os.path.join(os.path.dirname(__file__), "..", "..", "tests", "golden", "weights_seed0.npz"))
    w = {k: d[k] for k in ("W1", "b1", "w2", "b2")}
    e = Engine(lanes=8192, seed=0, balance=True)
    e.set_weights(w, 1.5, 1)

    def window(k):
        e.step(k)
        t = e.harvest_enqueue()
        e.harvest_fetch(t, wrap=False)

    window(300)   # desync (bench.py: one 300-step launch)
    # bench.py's sequence once, from a fresh desync: the window right after it
    first = []
    for _ in range(3):
        window(5)
        e.sync()
        e.stats()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        window(20)
        torch.cuda.synchronize()
        first.append((time.perf_counter() - t0) * 1e6)
        window(300)
    print("bench sequence (300-step launch, 5-step warm-up, stats, 20-step window), x3: " +
          " ".join(f"{x:.0f}" for x in first) + " us")

    def seq(pre):
        out = []
        for _ in range(3):
            pre()
            window(5)
            e.sync()
            e.stats()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            window(20)
            torch.cuda.synchronize()
            out.append((time.perf_counter() - t0) * 1e6)
        return " ".join(f"{x:.0f}" for x in out)

    def idle(us):
        t_end = time.perf_counter() + us * 1e-6
        while time.perf_counter() < t_end:
            pass

    print("300 steps as 15 x 20-step launches, then the sequence: " + seq(lambda: [window(20) for _ in range(15)]))
    print("300-step launch, 3 ms idle, then the sequence: " + seq(lambda: (window(300), idle(3000))))
    print("300-step launch, 20 ms idle, then the sequence: " + seq(lambda: (window(300), idle(20000))))
    print("300-step launch without harvest fetch between: " + seq(lambda: (e.step(300),)))
    print("100-step launch: " + seq(lambda: window(100)))
    res = {"stats": [], "no_stats": [], "sleep_100us": []}
    for rep in range(20):
        for mode in res:
            window(5)   # warm-up
            e.sync()
            if mode == "stats":
                e.stats()
            elif mode == "sleep_100us":
                t_end = time.perf_counter() + 100e-6
                while time.perf_counter() < t_end:
                    pass
            torch.cuda.synchronize()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            window(20)
            torch.cuda.synchronize()
            torch.cuda.synchronize()
            res[mode].append(time.perf_counter() - t0)
    for mode, v in res.items():
        v = np.array(v) * 1e6
        print(f"{mode:12s}: first windows " + " ".join(f"{x:.0f}" for x in v[:6]))
        print(f"{mode:12s}: 20-step window median {np.median(v):.1f} us (min {v.min():.1f}, max {v.max():.1f}) "
              f"-> {20 * 8192 / np.median(v):.1f} M env steps/s")
    t = time.perf_counter()
    for _ in range(50):
        e.stats()
    print(f"Engine.stats(): {(time.perf_counter() - t) / 50 * 1e6:.1f} us")
    e.close()


if __name__ == "__main__":
    main()
