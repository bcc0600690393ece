#!/usr/bin/env python3
"""Episode delivery rates of the drop-in path (src/multi on MI355X).

  producer    the pipelined Worker (multi/worker.py: each cycle queues the next
              launch and its harvest before the host copies the previous one)
              against a bare engine loop of the same cadence that never reads
              its harvests on the host: env steps/s of both, so the ratio says
              whether the worker leaves the GPU idle between launches.
  end_to_end  main.py's shape (tests/main_harness.py restates it): a spawned
              worker_function process puts harvests on the ExperienceQueue
              (bulk shared-memory path) and this process takes Episodes with
              q.get(timeout=1) for --seconds: episodes/s and experiences/s
              delivered as Episode objects.
  pickle      the per-episode pickle round trip that mp.Queue costs the
              reference (src/multi/experience_queue.py:5-13), for scale.
One JSON line. Reference loop: src/multi/worker.py:47-76, src/main.py:115-137.
"""
import argparse
import json
import os
import pickle
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "mlp-ppo-2ply-multi_amd"), os.path.join(REPO, "tests")]


def _weights():
    w = np.load(os.path.join(REPO, "tests", "golden", "weights_seed0.npz"))
    return {k: w[k] for k in ("W1", "b1", "w2", "b2")}


class _PM:
    """A ParameterManager stand-in for the in-process producer run (version 1, T = 1.5)."""

    def __init__(self, w):
        self.w = w

    def get_temperature(self):
        return 1.5

    def get_parameters(self):
        return self.w

    def get_version(self):
        return 1


def producer(lanes, steps, cycles):
    from bgx import Engine
    from multi.worker import Worker
    w = _weights()
    os.environ["BGX_LANES"] = str(lanes)
    os.environ["BGX_STEPS_PER_HARVEST"] = str(steps)
    os.environ["BGX_GPU_MAP"] = "0"
    wk = Worker(0, _PM(w), None)
    for _ in range(3):
        wk.harvest_records()
    torch.cuda.synchronize()
    e0 = sum(e.stats()["env_steps"] for e in wk.engines)
    eps = recs = 0
    t0 = time.perf_counter()
    for _ in range(cycles):
        h, r = wk.harvest_records()
        eps += h.shape[0]
        recs += r.shape[0]
    for e in wk.engines:
        e.sync()
    el = time.perf_counter() - t0
    worker_rate = (sum(e.stats()["env_steps"] for e in wk.engines) - e0) / el
    for e in wk.engines:
        e.close()
    # the same cadence on a bare engine: launch, queue the harvest, fetch the
    # previous ticket without reading it (bench.py at N = 1)
    eng = Engine(lanes=lanes, seed=1000003, balance=True)
    eng.set_weights(w, 1.5, 1)
    pend = None
    for _ in range(3):
        eng.step(steps)
        t = eng.harvest_enqueue()
        if pend is not None:
            eng.harvest_fetch(pend, wrap=False)
        pend = t
    eng.sync()
    s0 = eng.stats()["env_steps"]
    t0 = time.perf_counter()
    for _ in range(cycles):
        eng.step(steps)
        t = eng.harvest_enqueue()
        eng.harvest_fetch(pend, wrap=False)
        pend = t
    eng.harvest_fetch(pend, wrap=False)
    eng.sync()
    bare_rate = (eng.stats()["env_steps"] - s0) / (time.perf_counter() - t0)
    eng.close()
    return {"lanes": lanes, "steps_per_harvest": steps, "cycles": cycles, "worker_env_steps_per_s": worker_rate,
            "bare_engine_env_steps_per_s": bare_rate, "worker_over_bare": worker_rate / bare_rate,
            "worker_episodes_per_s_produced": eps / el, "worker_records_per_s_produced": recs / el}


def end_to_end(lanes, steps, seconds):
    import multiprocessing
    import queue
    from multi import ExperienceQueue, ParameterManager, worker_function
    os.environ["BGX_LANES"] = str(lanes)
    os.environ["BGX_STEPS_PER_HARVEST"] = str(steps)
    os.environ["BGX_GPU_MAP"] = "0"
    ctx = multiprocessing.get_context("spawn")
    manager = ctx.Manager()
    pm = ParameterManager(manager.Lock(), manager.Value("i", 1), manager.dict())
    q = ExperienceQueue(ctx=ctx)
    p = ctx.Process(target=worker_function, args=(0, pm, q))
    p.start()
    try:
        first = q.get(timeout=300)   # the worker's start-up (engine creation, first harvests)
        n_eps, n_exp = 1, len(first.experiences)
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < seconds:
            try:
                ep = q.get(timeout=1)
            except queue.Empty:
                continue
            n_eps += 1
            n_exp += len(ep.experiences)
        el = time.perf_counter() - t0
    finally:
        p.terminate()
        p.join(timeout=30)
        q.close()
        manager.shutdown()
    return {"lanes": lanes, "seconds": el, "episodes_per_s": (n_eps - 1) / el, "experiences_per_s": n_exp / el,
            "consumer": "one Python process, q.get(timeout=1) -> Episode objects (main.py:115-137)"}


def pickle_rate(lanes):
    from bgx import Engine
    from bgx.episodes import to_episodes
    from environments import Episode, Experience, Player
    eng = Engine(lanes=lanes, seed=0)
    eng.set_weights(_weights(), 1.5, 1)
    eng.step(300)
    eng.harvest()
    eng.step(100)
    eps = to_episodes(eng.harvest(), Episode, Experience, Player)
    eng.close()
    t0 = time.perf_counter()
    for ep in eps:
        pickle.loads(pickle.dumps(ep))
    el = time.perf_counter() - t0
    return {"episodes": len(eps), "pickle_roundtrip_episodes_per_s": len(eps) / el,
            "pickle_bytes_per_episode": len(pickle.dumps(eps[0]))}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lanes", type=int, default=8192)
    ap.add_argument("--steps", type=int, default=100, help="steps per launch / harvest (BGX_STEPS_PER_HARVEST)")
    ap.add_argument("--cycles", type=int, default=60)
    ap.add_argument("--seconds", type=float, default=20.0)
    ap.add_argument("--modes", default="producer,end_to_end,pickle")
    a = ap.parse_args()
    out = {}
    modes = a.modes.split(",")
    if "producer" in modes:
        out["producer"] = producer(a.lanes, a.steps, a.cycles)
        print(json.dumps(out["producer"]), file=sys.stderr, flush=True)
    if "end_to_end" in modes:
        out["end_to_end"] = end_to_end(a.lanes, a.steps, a.seconds)
        print(json.dumps(out["end_to_end"]), file=sys.stderr, flush=True)
    if "pickle" in modes:
        out["pickle"] = pickle_rate(4096)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
