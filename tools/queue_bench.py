#!/usr/bin/env python3
"""Consumer-side rate of the bulk Episode path vs a per-episode pickle round
trip (what mp.Queue costs per Episode), on one harvest of a 4,096-lane engine."""
import json
import os
import pickle
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "mlp-ppo-2ply-multi_amd")]
from bgx import Engine  # noqa: E402
from bgx.episodes import to_episodes  # noqa: E402
from environments import Episode, Experience, Player  # noqa: E402
from multi.experience_queue import ExperienceQueue  # noqa: E402


def main():
    w = np.load(os.path.join(REPO, "tests", "golden", "weights_seed0.npz"))
    eng = Engine(lanes=4096, seed=0)
    eng.set_weights({k: w[k] for k in ("W1", "b1", "w2", "b2")}, 1.5, 1)
    eng.step(300)
    eng.harvest()
    eng.step(100)
    h = eng.harvest()
    hdr, rec = h.headers.cpu().numpy().view(np.uint32), h.records.cpu().numpy().view(np.uint32)
    n_eps, n_rec = hdr.shape[0], rec.shape[0]
    q = ExperienceQueue(capacity_mb=512)
    t0 = time.perf_counter()
    q.put_records(hdr, rec)
    got = [q.get(timeout=30) for _ in range(n_eps)]
    t_bulk = time.perf_counter() - t0
    eps = to_episodes(h, Episode, Experience, Player)
    t0 = time.perf_counter()
    for ep in eps:
        pickle.loads(pickle.dumps(ep))
    t_pickle = time.perf_counter() - t0
    q.close()
    print(json.dumps({"episodes": n_eps, "experiences": n_rec,
                      "bulk_s": t_bulk, "bulk_episodes_per_s": n_eps / t_bulk, "bulk_experiences_per_s": n_rec / t_bulk,
                      "pickle_roundtrip_s": t_pickle, "pickle_episodes_per_s": n_eps / t_pickle,
                      "pickle_bytes_per_episode": len(pickle.dumps(eps[0])),
                      "bulk_bytes_per_episode": (hdr.nbytes + rec.nbytes) / n_eps}))


if __name__ == "__main__":
    main()
