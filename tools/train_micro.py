#!/usr/bin/env python3
"""Trainer micro-benchmark (tools only): one harvest of self-play episodes,
then DeviceTrainer.update_records over 200 of them, repeated, per backend;
prints episodes/s of the update calls (host work included)."""
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "mlp-ppo-2ply-multi_amd"), os.path.join(REPO, "tools")]
from bgx import Engine  # noqa: E402
from bgx.net import BackgammonPolicyNetwork  # noqa: E402
from bgx.ops import weights_from  # noqa: E402
from bgx.trainer import DeviceTrainer  # noqa: E402
from train_loop import LocalPM  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    torch.manual_seed(0)
    pm = LocalPM(BackgammonPolicyNetwork().state_dict())
    eng = Engine(lanes=4096, seed=0)
    eng.set_weights(dict(zip(("W1", "b1", "w2", "b2"), weights_from(pm.get_parameters()))), 1.5, 1)
    eng.step(300)
    h = eng.harvest()
    hdr = h.headers[:200].cpu()
    rec = h.records[:int(hdr[:, 3].sum())].clone()
    eng.close()
    out = {"records": int(rec.shape[0])}
    for backend in ("hip", "torch"):
        tr = DeviceTrainer(pm, device="cuda", batch_episode_size=200, backend=backend)
        tr.update_records(hdr, rec)
        torch.cuda.synchronize()
        n = reps if backend == "hip" else max(1, reps // 5)
        t0 = time.perf_counter()
        for _ in range(n):
            tr.update_records(hdr, rec)
        torch.cuda.synchronize()
        out[backend + "_episodes_per_s"] = 200 * n / (time.perf_counter() - t0)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
