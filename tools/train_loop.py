#!/usr/bin/env python3
"""Self-play + training on one GPU without Python Episode objects (SURVEY §8f
rows 1-3 together): the engine plays, every finished episode's compact
records feed DeviceTrainer.update_records in the reference's batches of 200,
and each update's weights go straight back into the engine with the
reference temperature schedule (ParameterManager.get_temperature)."""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "mlp-ppo-2ply-multi_amd")]
from bgx import Engine  # noqa: E402
from bgx.net import BackgammonPolicyNetwork  # noqa: E402
from bgx.ops import weights_from  # noqa: E402
from bgx.trainer import DeviceTrainer  # noqa: E402


class LocalPM:
    """Versioned weights + temperature schedule (parameter_manager.py:79-111), single process."""

    def __init__(self, sd):
        self.sd, self.version = {k: v.detach().cpu() for k, v in sd.items()}, 1

    def get_parameters(self, device=None):
        return {k: v.to(device) if device else v for k, v in self.sd.items()}

    def set_parameters(self, sd):
        self.sd = {k: v.detach().cpu() for k, v in sd.items()}
        self.version += 1

    def get_temperature(self):
        v = self.version
        return 1.5 if v <= 1 else (0.5 if v >= 4001 else 1.5 - (v - 1) / 4000)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lanes", type=int, default=4096)
    ap.add_argument("--updates", type=int, default=20)
    ap.add_argument("--batched", action="store_true")
    ap.add_argument("--backend", default="hip", choices=("hip", "torch"))
    args = ap.parse_args()
    torch.manual_seed(0)
    pm = LocalPM(BackgammonPolicyNetwork().state_dict())
    trainer = DeviceTrainer(pm, device="cuda", batched=args.batched, backend=args.backend)
    eng = Engine(lanes=args.lanes, seed=0)
    w = dict(zip(("W1", "b1", "w2", "b2"), weights_from(pm.get_parameters())))
    eng.set_weights(w, pm.get_temperature(), pm.version)
    hdr_buf, rec_buf = [], []
    done, steps, t0, t_train = 0, 0, time.perf_counter(), 0.0
    while done < args.updates:
        eng.step(50)
        steps += 50
        h = eng.harvest()
        if h.n_episodes:
            hdr_buf.append(h.headers.cpu())
            rec_buf.append(h.records)
        n = sum(x.shape[0] for x in hdr_buf)
        while n >= 200 and done < args.updates:
            hdr, rec = torch.cat(hdr_buf), torch.cat(rec_buf)
            k = int(hdr[:200, 3].sum())
            t1 = time.perf_counter()
            m = trainer.update_records(hdr[:200], rec[:k])
            torch.cuda.synchronize()
            t_train += time.perf_counter() - t1
            hdr_buf, rec_buf = [hdr[200:]], [rec[k:]]
            n -= 200
            done += 1
            w = dict(zip(("W1", "b1", "w2", "b2"), weights_from(pm.get_parameters())))
            eng.set_weights(w, pm.get_temperature(), pm.version)
    el = time.perf_counter() - t0
    print(json.dumps({"updates": done, "episodes_trained": 200 * done, "env_steps": steps * args.lanes,
                      "wall_s": el, "train_s": t_train, "updates_per_s": done / el,
                      "train_episodes_per_s": 200 * done / t_train, "last_loss": m["loss"],
                      "version": pm.version, "temperature": pm.get_temperature(), "batched": args.batched,
                      "backend": trainer.backend}))


if __name__ == "__main__":
    main()
