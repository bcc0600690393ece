"""top5 block-load variant debug (tools only): the stateless 2-ply W of the
golden boards, exact and reference-sampled, from the library BGX_LIB names;
saved for a cross-library comparison."""
import os, sys
import numpy as np
import torch
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "mlp-ppo-2ply-multi_amd")]
from bgx import ops
t = np.load(os.path.join(REPO, "tests/golden/two_ply.npz"))
w = dict(np.load(os.path.join(REPO, "tests/golden/weights_seed0.npz")))
net = ops.Net({k: w[k] for k in ("W1", "b1", "w2", "b2")})
B, O = torch.from_numpy(t["boards"]).cuda(), torch.from_numpy(t["opponent"]).cuda()
out = {"exact": [net.two_ply(B, O).cpu().numpy() for _ in range(3)],
       "samp": [net.two_ply(B, O, sample=50, seed=3).cpu().numpy() for _ in range(3)]}
for k, v in out.items():
    print(k, "run-to-run equal:", all(np.array_equal(v[0], x) for x in v[1:]),
          "max diff", max(float(np.abs(v[0] - x).max()) for x in v[1:]))
np.savez(sys.argv[1], exact=np.stack(out["exact"]), samp=np.stack(out["samp"]))
