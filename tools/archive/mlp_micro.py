#!/usr/bin/env python3
"""Value-MLP micro-benchmark: bgx_value_boards (fused encode + split-fp16 MFMA)
over n random self-play afterstates; prints rows/s and algorithmic TFLOP/s."""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "mlp-ppo-2ply-multi_amd")]
from bgx import ops  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4_000_000
    d = np.load(os.path.join(REPO, "tests", "golden", "weights_seed0.npz"))
    net = ops.Net({k: d[k] for k in ("W1", "b1", "w2", "b2")})
    e = np.load(os.path.join(REPO, "tests", "golden", "encode.npz"))
    idx = np.random.default_rng(0).integers(0, len(e["boards"]), n)
    b = torch.from_numpy(e["boards"][idx]).cuda()
    p = torch.from_numpy(e["player"][idx]).cuda()
    net.value_boards(b, p)
    torch.cuda.synchronize()
    s, t = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 10
    s.record()
    for _ in range(reps):
        net.value_boards(b, p)
    t.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(t) / reps
    print(json.dumps({"rows": n, "ms": ms, "rows_per_s": n / ms * 1e3,
                      "tflops_algorithmic": 50944 * n / ms * 1e3 / 1e12,
                      "nt": os.environ.get("BGX_MLP_NT", "default")}))


if __name__ == "__main__":
    main()
