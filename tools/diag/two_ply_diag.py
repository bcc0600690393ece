"""Diagnose bgx_two_ply mismatches against tests/golden/two_ply.npz (tools only):
per mismatching position, per roll: the GPU reply boards (stateless movegen)
vs the oracle's, and the top-5 means from oracle V."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "mlp-ppo-2ply-multi_amd"), os.path.join(REPO, "oracle"), os.path.join(REPO, "tests")]
import oracle as orc  # noqa: E402
from conftest import golden  # noqa: E402
from bgx import ops  # noqa: E402

ROLLS = [(a, b) for a in range(1, 7) for b in range(a, 7)]
w = {k: golden("weights_seed0.npz")[k] for k in ("W1", "b1", "w2", "b2")}
t = golden("two_ply.npz")
net = ops.Net(w)
B, O = torch.from_numpy(t["boards"]).cuda(), torch.from_numpy(t["opponent"]).cuda()
W = net.two_ply(B, O).cpu().numpy()
bad = np.nonzero(np.abs(W - t["w_seed0"]) > 1e-5)[0]
print("lib", os.environ.get("BGX_LIB", "default"), "mismatches", bad.tolist(), (W - t["w_seed0"])[bad].tolist())
for i in bad[:3]:
    b, o = t["boards"][i], int(t["opponent"][i])
    print("pos", i, "opp", o, "board", b.tolist())
    for ri, (d0, d1) in enumerate(ROLLS):
        n, res, _ = orc.movegen(b, o, d0, d1)
        out, cnt = ops.movegen(torch.from_numpy(b[None]).cuda(), torch.tensor([o], dtype=torch.uint8).cuda(),
                               torch.tensor([[d0, d1]], dtype=torch.uint8).cuda(), cap=1024)
        g = out[0, :int(cnt[0])].cpu().numpy()
        same = int(cnt[0]) == n and np.array_equal(g, res)
        if not same or n > 100:
            print("  roll", (d0, d1), "oracle", n, "gpu", int(cnt[0]), "same" if same else "DIFFERENT")
