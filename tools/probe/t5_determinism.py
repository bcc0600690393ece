"""Probe (tools only): repeat the stateless 2-ply op in exact and reference-
sampled mode on the golden fixture boards and report run-to-run mismatches."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "mlp-ppo-2ply-multi_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
from bgx import ops  # noqa: E402

g = np.load(os.path.join(os.path.dirname(__file__), "..", "..", "tests", "golden", "two_ply.npz"))
w = np.load(os.path.join(os.path.dirname(__file__), "..", "..", "tests", "golden", "weights_seed0.npz"))
net = ops.Net({k: w[k] for k in ("W1", "b1", "w2", "b2")})
B, O = torch.from_numpy(g["boards"]).cuda(), torch.from_numpy(g["opponent"]).cuda()
ex = [net.two_ply(B, O).cpu().numpy() for _ in range(3)]
sm = [net.two_ply(B, O, sample=50, seed=3).cpu().numpy() for _ in range(3)]
print("exact runs differ:", [int((ex[0] != e).sum()) for e in ex[1:]],
      "sampled runs differ:", [int((sm[0] != e).sum()) for e in sm[1:]],
      "sampled > exact:", int((sm[0] > ex[0] + 1e-12).sum()))
